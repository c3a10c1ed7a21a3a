#!/bin/bash
# Occupancy sensitivity of the SMA kernel: pad its LDS so 2 (mask 128) or 1 (mask 384) blocks fit
# per CU instead of 3, timed interleaved in one process (scripts/ablate.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
MASKS=0,128,384 timeout -k 10 200 python -u scripts/ablate.py > gpurun_out/occ.log 2>&1; rc=$?; cat gpurun_out/occ.log; exit $rc
