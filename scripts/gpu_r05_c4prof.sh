#!/bin/bash
# Round 5: config 4 shards re-profiled after the finder / accountant peels (trace + PMC passes),
# and the per-role stamps of configs 4 and 3 (profiling build).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05
for s in 500 250; do
  bash scripts/gpu_profile.sh config4_s$s --config 4 --symbols $s --steps 10 --warmup 2 || exit 1
done
timeout -k 10 200 python3 scripts/stamps_tile.py 4 500 > gpurun_out/r05/stamps4_head.txt 2>&1 || { tail -5 gpurun_out/r05/stamps4_head.txt; exit 1; }
timeout -k 10 200 python3 scripts/stamps_tile.py 3 500 > gpurun_out/r05/stamps3_head.txt 2>&1 || { tail -5 gpurun_out/r05/stamps3_head.txt; exit 1; }
cat gpurun_out/r05/stamps4_head.txt gpurun_out/r05/stamps3_head.txt
