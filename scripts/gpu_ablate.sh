#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ablate.py > gpurun_out/ablate.log 2>&1; rc=$?; cat gpurun_out/ablate.log; exit $rc
