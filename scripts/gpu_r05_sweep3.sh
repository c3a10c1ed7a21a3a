#!/bin/bash
# Round 5: a deep random parity sweep over fresh seeds (2000-4999: 18,000 cases) at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
BT_RANDOM_SEEDS=3000 BT_RANDOM_SEED0=2000 timeout -k 10 840 python -u -m pytest tests/test_gpu_random.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05/random_sweep_seeds2000_4999.log 2>&1 || { tail -30 gpurun_out/r05/random_sweep_seeds2000_4999.log; exit 1; }
tail -1 gpurun_out/r05/random_sweep_seeds2000_4999.log
