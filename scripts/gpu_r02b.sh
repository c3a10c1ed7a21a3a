#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r02b
bash scripts/gpu_tests.sh || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02b/bench.log 2>&1 || { tail -20 gpurun_out/r02b/bench.log; exit 1; }
tail -1 gpurun_out/r02b/bench.log
timeout -k 10 300 python3 bench.py --leg ingest --steps 5 --warmup 1 > gpurun_out/r02b/ingest.log 2>&1 || { tail -20 gpurun_out/r02b/ingest.log; exit 1; }
tail -1 gpurun_out/r02b/ingest.log
bash scripts/gpu_profile.sh config2 --gpus 1 --steps 20 --warmup 5 || exit 1
