#!/bin/bash
# Tuning aid: config-3 shard time vs extra task-only waves (BT_XW).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for xw in ${XWS:-2 3 4 6}; do
  BT_XW=$xw timeout -k 10 120 python -u bench.py --config ${CFG:-3} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/xw.log 2>&1 || { tail -3 gpurun_out/xw.log; exit 1; }
  echo "xw=$xw $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/xw.log)"
done
