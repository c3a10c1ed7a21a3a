#!/bin/bash
# Interleaved A/B of an environment knob on the config-2 bench: VAR unset vs VAR=$VAL, R rounds.
export BT_LIB=${BT_LIB:-libbt_prof.so}  # profiling build (make PROFILING=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in $(seq ${R:-3}); do for m in unset set; do
  if [ $m = set ]; then export $VAR=$VAL; else unset $VAR; fi
  timeout -k 10 100 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/envab.log 2>&1 || { tail -3 gpurun_out/envab.log; exit 1; }
  echo "c2 $VAR $m $(grep -o '"ms_per_step": [0-9.]*\|"kernel_avg_ms": [0-9.]*' gpurun_out/envab.log | tr '\n' ' ')"
done; done
