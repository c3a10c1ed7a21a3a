#!/bin/bash
# Tuning aid: tile-kernel shard time vs parameter lanes per wave (BT_LPW) and extra task waves
# (BT_XW), for the configs in CFGS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for cfg in ${CFGS:-3 4}; do
  for lpw in ${LPWS:-64 32 16}; do
    for xw in ${XWS:-default}; do
      if [ "$xw" = default ]; then unset BT_XW; else export BT_XW=$xw; fi
      BT_LPW=$lpw timeout -k 10 120 python -u bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lpw.log 2>&1 || { tail -3 gpurun_out/lpw.log; exit 1; }
      echo "cfg=$cfg lpw=$lpw xw=$xw $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/lpw.log)"
    done
  done
done
