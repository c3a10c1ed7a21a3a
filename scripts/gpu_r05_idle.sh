#!/bin/bash
# Round 5: EMA+OLS task waves beside a pacing role kept idle (BT_EMA_IDLE bits: 1 helper B's
# SIMD partner, 2 helper A's, 4 the parameter wave's) — parity of the all-idle build, then config 3
# kernel time, interleaved with the release build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/idle
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
BT_LIB=dev/i7.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_segments.py -m gpu -k "ema" > gpurun_out/r05/idle/tests.log 2>&1 || { tail -20 gpurun_out/r05/idle/tests.log; exit 1; }
tail -1 gpurun_out/r05/idle/tests.log
for rep in 1 2; do
  LIBS="libbt.so dev/i1.so dev/i2.so dev/i4.so dev/i7.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
