#!/bin/bash
# Parity depth at the round's final kernels: a random sweep on fresh seeds 6,000-7,999 and every
# symbol x parameter of config 5's 1,250-symbol shard against the C oracle.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06/deep; mkdir -p $O
BT_RANDOM_SEED0=6000 BT_RANDOM_SEEDS=2000 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_random.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/random_sweep_seeds6000_7999.log 2>&1
rc=$?; tail -2 $O/random_sweep_seeds6000_7999.log; [ $rc -eq 0 ] || exit $rc
BT_CONFIG5_ALL=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k config5 --timeout 500 --timeout-method thread > $O/config5_all_symbols.log 2>&1
rc=$?; tail -2 $O/config5_all_symbols.log; exit $rc
