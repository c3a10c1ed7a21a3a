#!/bin/bash
# Round-4 final check at HEAD: the whole GPU suite (whole-shard oracle checks included), smoke,
# and the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread --durations=8"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_gpu_final2.log 2>&1 || { tail -30 gpurun_out/r04/pytest_gpu_final2.log; exit 1; }
tail -11 gpurun_out/r04/pytest_gpu_final2.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
