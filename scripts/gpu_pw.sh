#!/bin/bash
# Tuning aid: config-4 shard time vs parameter waves per block (BT_PW) and extra task waves (BT_XW).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for pw in ${PWS:-4 2 1}; do for xw in ${XWS:-0}; do
  BT_PW=$pw BT_XW=$xw timeout -k 10 120 python -u bench.py --config ${CFG:-4} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pw.log 2>&1 || { tail -3 gpurun_out/pw.log; exit 1; }
  echo "pw=$pw xw=$xw $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/pw.log)"
done; done
