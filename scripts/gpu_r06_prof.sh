#!/bin/bash
# Round 6 profiles at HEAD: the per-GPU shards of configs 3-5 (config 2, the driver's command,
# in a first call), each under rocprofv3 --kernel-trace --stats plus separate --pmc passes of the
# same bench.py command (scripts/gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
for spec in "3 500" "3 250" "4 500" "4 250" "5 1250"; do
  set -- $spec
  bash scripts/gpu_profile.sh config$1_s$2 --config $1 --symbols $2 --steps 10 --warmup 2 || exit 1
done
