#!/bin/bash
# Round 5: burn-in tiles of the speculative bar segments on the 250-symbol shards of configs 4
# and 3 (kernel time and fix-pass re-walks per step).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/burn
for spec in "4 64" "4 32" "4 16" "4 8" "4 4" "4 64" "3 0" "3 48" "3 32" "3 0"; do
  set -- $spec
  timeout -k 10 200 python3 bench.py --config $1 --symbols 250 --burn $2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/burn/b_$1_$2.log 2>&1 || { tail -5 gpurun_out/r05/burn/b_$1_$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/burn/b_$1_$2.log').read().strip().splitlines()[-1]); print('config $1 burn $2 kernel', round(d['roofline']['kernel_avg_ms'],3), d.get('bar_segments'))"
done
