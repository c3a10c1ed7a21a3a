#!/bin/bash
# Round 4: config 4 task-only waves per block (profiling build, BT_XW): 1 vs the default 2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/xw
export BT_LIB=dev/prof.so
for rep in 1 2; do
for xw in 2 1; do
  for s in 500 250; do
    BT_XW=$xw timeout -k 10 200 python3 bench.py --config 4 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/xw/b_${xw}_$s.log 2>&1 || { tail -5 gpurun_out/xw/b_${xw}_$s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/xw/b_${xw}_$s.log').read().strip().splitlines()[-1]); print('xw $xw', $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
  done
done
done
