#!/bin/bash
# Profiles of the per-GPU shards of BASELINE configs 3-5 (strong scaling: the shard rank 0 runs
# at the quoted GPU counts), each with scripts/gpu_profile.sh (trace + PMC passes of the same
# bench.py command). Shards: config 3 500 (1 GPU) / 250 (2 GPUs); config 4 500 (4 GPUs) / 250
# (8 GPUs); config 5 1,250 (8 GPUs).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for spec in ${SHARDS:-"3 500" "3 250" "4 500" "4 250" "5 1250"}; do
  set -- $spec
  bash scripts/gpu_profile.sh config$1_s$2 --config $1 --symbols $2 --steps ${STEPS:-10} --warmup 2 ${EXTRA_ARGS} || exit 1
done
