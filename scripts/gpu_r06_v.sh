#!/bin/bash
# Parity depth for the 128-bar EMA stages: the new stage-shape tests (split runs, edge trades,
# random grids in 128-bar stages), then a deep random sweep on fresh seeds 5,000-5,999.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06/v; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_segments.py tests/test_tile_edge_trades.py tests/test_gpu_random.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/stage_tests.log 2>&1
rc=$?; tail -3 $O/stage_tests.log; [ $rc -eq 0 ] || exit $rc
BT_RANDOM_SEED0=5000 BT_RANDOM_SEEDS=1000 timeout -k 10 700 python3 -u -m pytest tests/test_gpu_random.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/random_sweep_seeds5000_5999.log 2>&1
rc=$?; tail -3 $O/random_sweep_seeds5000_5999.log; exit $rc
