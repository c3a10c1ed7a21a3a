#!/bin/bash
# Round 4: Bollinger walkers with run-time int32 gap / mdd (acct_close_rt, dev/v5.so) vs HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/r4.so dev/v5.so dev/r4.so dev/v5.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
BT_LIB=dev/v5.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_j.log 2>&1 || { tail -30 gpurun_out/r04/pytest_j.log; exit 1; }
tail -1 gpurun_out/r04/pytest_j.log
