#!/bin/bash
# Round-5 check at HEAD: the whole GPU suite (whole-shard oracle checks included), smoke, the
# default bench line, and the driver's command (config 2) under rocprofv3 (scripts/gpu_profile.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread --durations=8"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r05/pytest_gpu_head.log 2>&1 || { tail -30 gpurun_out/r05/pytest_gpu_head.log; exit 1; }
tail -11 gpurun_out/r05/pytest_gpu_head.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke.log 2>&1 || { tail -5 gpurun_out/r05/smoke.log; exit 1; }
tail -1 gpurun_out/r05/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r05/bench_default.log 2>&1 || { tail -5 gpurun_out/r05/bench_default.log; exit 1; }
tail -1 gpurun_out/r05/bench_default.log | cut -c1-300
[ -n "$NO_PROFILE" ] || bash scripts/gpu_profile.sh config2
