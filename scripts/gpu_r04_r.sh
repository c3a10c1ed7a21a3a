#!/bin/bash
# Round 4: the bar segments' Bollinger walkers keep their drawdown forms in int32 in narrow tiles
# (acct_close_rt_seg; kNegInf's low word is INT32_MIN) — dev/v16.so vs HEAD (dev/h16.so) on
# config 4's shards, then the whole GPU suite on v16.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/h16.so dev/v16.so dev/h16.so dev/v16.so" CFG=4 SYMS="250 500" bash scripts/gpu_ab_libs.sh || exit 1
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread --durations=5"
BT_LIB=dev/v16.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_r.log 2>&1 || { tail -30 gpurun_out/r04/pytest_r.log; exit 1; }
tail -9 gpurun_out/r04/pytest_r.log
