#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/stamps.py > gpurun_out/stamps.log 2>&1; rc=$?; cat gpurun_out/stamps.log; exit $rc
