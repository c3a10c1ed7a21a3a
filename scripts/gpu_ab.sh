#!/bin/bash
# A/B of a profiling bit: default bench and config 5 with BT_ABLATE=0 and BT_ABLATE=$AB, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in 1 2; do for m in 0 ${AB:-32}; do
  BT_ABLATE=$m timeout -k 10 100 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/ab.log 2>&1 || exit 1
  echo "c2 mask $m $(grep -o '"ms_per_step": [0-9.]*\|"kernel_avg_ms": [0-9.]*' gpurun_out/ab.log | tr '\n' ' ')"
done; done
for m in 0 ${AB:-32}; do
  BT_ABLATE=$m timeout -k 10 100 python -u bench.py --config 5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab.log 2>&1 || exit 1
  echo "c5 mask $m $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/ab.log)"
done
grep -o '"valu_issue": {[^}]*}' gpurun_out/ab.log
