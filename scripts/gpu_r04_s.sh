#!/bin/bash
# Round 4: Bollinger hardware-wave role maps (profiling build, BT_WAVEMAP) on config 4's shards:
# the default (accountant beside parameter wave 2) and three others, twice each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/wm
export BT_LIB=dev/prof.so
for rep in 1 2; do
for m in 45763210 45763120 54763210 47563210; do
  for s in 500 250; do
    BT_WAVEMAP=$m timeout -k 10 200 python3 bench.py --config 4 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/wm/b_${m}_$s.log 2>&1 || { tail -5 gpurun_out/wm/b_${m}_$s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/wm/b_${m}_$s.log').read().strip().splitlines()[-1]); print('map $m', $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
  done
done
done
