#!/bin/bash
# Round 4: the EMA drawdown table as the first task of each round instead of in helper A's scan
# (dev/v13.so; v14 also -DBT_CHAIN_OPAQUE=2) vs HEAD (dev/h11.so) on config 3's shards, then
# the whole GPU suite on v13.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/h11.so dev/v13.so dev/v14.so dev/h11.so dev/v13.so dev/v14.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
BT_LIB=dev/v13.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_p.log 2>&1 || { tail -30 gpurun_out/r04/pytest_p.log; exit 1; }
tail -1 gpurun_out/r04/pytest_p.log
