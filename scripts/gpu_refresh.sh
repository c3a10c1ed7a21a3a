#!/bin/bash
# Round profile refresh in one call: config-2 profile (tests, smoke, bench, kernel trace, PMC),
# the config 3/4/5 shard traces + PMC, and the per-config bench lines with CPU baselines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash scripts/gpu_profile.sh || exit $?
bash scripts/gpu_profile_cfgs.sh || exit $?
for c in 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 2 > gpurun_out/bench_config$c.log 2>&1 || { tail -3 gpurun_out/bench_config$c.log; exit 1; }
  echo "bench config $c ok"
done
