#!/bin/bash
# parity tests (verbose), then configs 3/4/5 throughput; each step time-limited
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_gpu.log | tail -60 | cut -c1-250; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_cfgs.sh
