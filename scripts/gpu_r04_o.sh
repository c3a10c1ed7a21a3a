#!/bin/bash
# Round 4: the EMA chain from opaque LDS pointers inside a restrict-parameter function
# (dev/v12.so, -DBT_CHAIN_OPAQUE=2: immediate offsets, reads still ahead of the stores) vs HEAD
# (dev/h11.so) on config 3's shards, then the whole GPU suite on v12.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/h11.so dev/v12.so dev/h11.so dev/v12.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
BT_LIB=dev/v12.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_o.log 2>&1 || { tail -30 gpurun_out/r04/pytest_o.log; exit 1; }
tail -1 gpurun_out/r04/pytest_o.log
