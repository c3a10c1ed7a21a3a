#!/bin/bash
# Task-only wave count sweep (BT_XW) for the tile kernels: config 4 and config 3 shards.
export BT_LIB=${BT_LIB:-libbt_prof.so}  # profiling build (make PROFILING=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in 1 2; do
for spec in ${SPECS:-"4:1" "4:2" "4:3" "3:4" "3:5" "3:6"}; do
  c=${spec%%:*}; x=${spec#*:}
  BT_XW=$x timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/xw.log 2>&1 || { tail -3 gpurun_out/xw.log; exit 1; }
  echo "c$c xw=$x $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/xw.log)"
done; done
