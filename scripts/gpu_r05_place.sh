#!/bin/bash
# Round 5: hardware placement of the tile kernels' blocks and waves (profiling build stamps)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for c in 3 4; do
  timeout -k 10 200 python3 scripts/dev/placement.py $c 500 >> gpurun_out/r05/placement.txt 2>&1 || { tail -20 gpurun_out/r05/placement.txt; exit 1; }
done
timeout -k 10 200 python3 scripts/dev/placement.py 3 250 >> gpurun_out/r05/placement.txt 2>&1 || { tail -20 gpurun_out/r05/placement.txt; exit 1; }
cat gpurun_out/r05/placement.txt
