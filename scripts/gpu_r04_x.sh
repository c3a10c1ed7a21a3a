#!/bin/bash
# Round 4: bar segments per symbol on the 250-symbol shards of configs 3 and 4 (bench --segments;
# automatic: 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/seg
for rep in 1 2; do
for c in 3 4; do
  for G in 2 3 4; do
    timeout -k 10 200 python3 bench.py --config $c --symbols 250 --segments $G --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/seg/b_${c}_$G.log 2>&1 || { tail -5 gpurun_out/seg/b_${c}_$G.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/seg/b_${c}_$G.log').read().strip().splitlines()[-1]); print('config $c 250 G $G kernel', round(d['roofline']['kernel_avg_ms'],3))"
  done
done
done
