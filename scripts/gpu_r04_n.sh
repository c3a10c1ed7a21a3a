#!/bin/bash
# Round 4: config 3's phase ablation counters (profiling build), then OLS-window task lane masks
# straight from the compares (dev/v10.so; v11 also without task-kind selects) vs HEAD (dev/h7.so)
# on config 3's shards, then
# the whole GPU suite on v11.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
bash scripts/gpu_pmc_ablate3.sh || exit 1
LIBS="dev/h7.so dev/v10.so dev/v11.so dev/h7.so dev/v10.so dev/v11.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
BT_LIB=dev/v11.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_n.log 2>&1 || { tail -30 gpurun_out/r04/pytest_n.log; exit 1; }
tail -1 gpurun_out/r04/pytest_n.log
