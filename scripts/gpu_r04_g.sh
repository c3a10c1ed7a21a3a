#!/bin/bash
# Round 4 refresh at HEAD: the whole GPU suite, smoke, the driver's command profiled, config 5's
# shard profiled (automatic G = 6), the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_gpu_g.log 2>&1 || { tail -40 gpurun_out/r04/pytest_gpu_g.log; exit 1; }
tail -1 gpurun_out/r04/pytest_gpu_g.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/gpu_profile.sh config2 --gpus 1 --steps 20 --warmup 5 || exit 1
bash scripts/gpu_profile.sh config5_s1250 --config 5 --symbols 1250 --steps 10 --warmup 2 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
