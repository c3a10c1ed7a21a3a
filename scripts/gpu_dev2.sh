#!/bin/bash
# parity tests, stamps, bench (each step time-limited; stop on crash/timeout)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 200 python -u scripts/stamps.py > gpurun_out/stamps.log 2>&1; rc=$?; cat gpurun_out/stamps.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; cut -c1-700 gpurun_out/bench.log; exit $rc
