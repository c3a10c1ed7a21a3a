#!/bin/bash
# Round 4: the Bollinger accountant and walker read each record's / exit's LDS data in one round
# trip (dev/v1.so) — the whole GPU suite on it, then A/B against HEAD (dev/r4.so) on config
# 4's shards, then the role stamps of both profiling builds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
BT_LIB=dev/v1.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_h.log 2>&1 || { tail -30 gpurun_out/r04/pytest_h.log; exit 1; }
tail -1 gpurun_out/r04/pytest_h.log
LIBS="dev/r4.so dev/v1.so dev/r4.so dev/v1.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
for lib in dev/prof_r4.so dev/prof.so; do
  BT_LIB=$lib timeout -k 10 120 python3 scripts/stamps_tile.py 4 > gpurun_out/r04/stamps4_$lib.txt 2>&1 || { tail -5 gpurun_out/r04/stamps4_$lib.txt; exit 1; }
  echo $lib; grep -v amdgpu.ids gpurun_out/r04/stamps4_$lib.txt
done
