#!/bin/bash
# Round 4: Bollinger walker variants (v2 exit reads in one round trip, v3 int32 walk accounts,
# v4 both; v0 = the macros off) against HEAD (dev/r4.so) on config 4's shards, then the whole
# GPU suite on v4.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/r4.so dev/v0.so dev/v2.so dev/v3.so dev/v4.so dev/r4.so dev/v0.so dev/v2.so dev/v3.so dev/v4.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
BT_LIB=dev/v4.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_i.log 2>&1 || { tail -30 gpurun_out/r04/pytest_i.log; exit 1; }
tail -1 gpurun_out/r04/pytest_i.log
