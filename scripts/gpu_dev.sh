#!/bin/bash
# Development GPU call: parity tests, then kernel ablation timings, then the bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -u scripts/ablate.py > gpurun_out/ablate.log 2>&1; rc=$?; cat gpurun_out/ablate.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; cat gpurun_out/bench.log; exit $rc
