#!/bin/bash
# Round 4: the accountant's record loop as one copy with the run-time narrow close (acct_close_rt)
# instead of a narrow and a wide copy — dev/v17.so vs HEAD (dev/h17.so) on config 4's shards,
# then the whole GPU suite on v17.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/h17.so dev/v17.so dev/h17.so dev/v17.so" CFG=4 SYMS="250 500" bash scripts/gpu_ab_libs.sh || exit 1
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread --durations=5"
BT_LIB=dev/v17.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_t.log 2>&1 || { tail -30 gpurun_out/r04/pytest_t.log; exit 1; }
tail -9 gpurun_out/r04/pytest_t.log
