#!/bin/bash
# Config 3's shards re-profiled after the EMA helper's add-with-carry scans (scripts/gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
for S in 500 250; do
  bash scripts/gpu_profile.sh config3_s$S --config 3 --symbols $S --steps 10 --warmup 2 || exit 1
done
