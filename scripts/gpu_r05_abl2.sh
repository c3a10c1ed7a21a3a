#!/bin/bash
# Round 5: config 2 phase ablations (profiling build; timing only): 1 stage 1, 2 stage 2 (keys and
# drawdown table), 4 compare, 8 walk, and combinations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/abl
for a in 0 1 2 4 8 12 14 15 0; do
  BT_LIB=dev/prof.so BT_ABLATE=$a timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --topk 0 > gpurun_out/r05/abl/c2_$a.log 2>&1 || { tail -5 gpurun_out/r05/abl/c2_$a.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/abl/c2_$a.log').read().strip().splitlines()[-1]); print('config 2 ablate', $a, 'kernel', round(d['roofline']['kernel_avg_ms'],4))"
done
