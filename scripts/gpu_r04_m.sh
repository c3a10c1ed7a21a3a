#!/bin/bash
# Round 4: config 4 with a second finder/accountant pair (dev/v8.so, -DBT_SPLIT2) and the
# accountant at the walk's priority (dev/v9.so) vs HEAD (dev/h7.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/h7.so dev/v8.so dev/v9.so dev/h7.so dev/v8.so dev/v9.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
