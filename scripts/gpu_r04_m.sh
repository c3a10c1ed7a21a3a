#!/bin/bash
# Round 4: config 4 with a second finder/accountant pair (libbt_v8.so, -DBT_SPLIT2) and the
# accountant at the walk's priority (libbt_v9.so) vs HEAD (libbt_h7.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="libbt_h7.so libbt_v8.so libbt_v9.so libbt_h7.so libbt_v8.so libbt_v9.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
