#!/bin/bash
# Round 5: EMA+OLS hardware-wave role maps (profiling build, BT_EMA_WAVEMAP; hardware waves w and
# w + 4 share a SIMD). Roles: 0 parameter wave, 1 helper A, 2 helper B (chain), 3-7 task waves.
#   76543210 identity: P|T A|T B|T T|T ; 76524310 B beside P ; 76524301 B beside A ; 76514320 P beside A
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/wmap
for rep in 1 2; do
for m in 76543210 76524310 76524301 76514320; do
  for s in 500 250; do
    BT_LIB=dev/prof.so BT_EMA_WAVEMAP=$m timeout -k 10 200 python3 bench.py --config 3 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/wmap/c3_${m}_$s.log 2>&1 || { tail -5 gpurun_out/r05/wmap/c3_${m}_$s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r05/wmap/c3_${m}_$s.log').read().strip().splitlines()[-1]); print('map $m config 3 $s kernel', round(d['roofline']['kernel_avg_ms'],3))"
  done
done
done
