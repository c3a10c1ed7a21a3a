#!/bin/bash
# Round 6: stamps of configs 3 (500 / 250 symbols) and 4 (500) at HEAD, config 4 skeleton and
# phase ablations at HEAD (profiling build).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/q; mkdir -p $O
export PYTHONUNBUFFERED=1
for spec in "3 500" "3 250" "4 500"; do
  set -- $spec
  timeout -k 10 200 python3 scripts/stamps_tile.py $1 $2 > $O/stamps$1_$2.txt 2>&1 || { tail -5 $O/stamps$1_$2.txt; exit 1; }
  grep -v amdgpu.ids $O/stamps$1_$2.txt
done
for ab in 0 10 8 2 4096; do
  BT_LIB=dev/prof.so BT_ABLATE=$ab timeout -k 10 200 python3 bench.py --config 4 --symbols 500 --steps 10 --warmup 2 --no-cpu-baseline --topk 0 > $O/c4_abl$ab.log 2>&1 || { tail -5 $O/c4_abl$ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c4_abl$ab.log').read().strip().splitlines()[-1]); print('config 4 ablate $ab kernel', round(d['roofline']['kernel_avg_ms'],3))"
done
