#!/bin/bash
# Round 4: window-task lane masks straight from the compares (dev/v7.so) vs HEAD (dev/h6.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/h6.so dev/v7.so dev/h6.so dev/v7.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
BT_LIB=dev/v7.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_l.log 2>&1 || { tail -30 gpurun_out/r04/pytest_l.log; exit 1; }
tail -1 gpurun_out/r04/pytest_l.log
