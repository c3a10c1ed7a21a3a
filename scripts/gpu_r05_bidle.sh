#!/bin/bash
# Round 5: Bollinger roles that take no tasks (BT_BOLL_IDLE bits: 1 the finder's SIMD partner, 2
# the finder, 4 the accountant, 8 the helper) — Bollinger parity of one build, then config 4
# kernel time, interleaved with the release build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/bidle
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
BT_LIB=dev/b1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_segments.py -m gpu -k "boll" > gpurun_out/r05/bidle/tests.log 2>&1 || { tail -20 gpurun_out/r05/bidle/tests.log; exit 1; }
tail -1 gpurun_out/r05/bidle/tests.log
for rep in 1 2; do
  LIBS="libbt.so dev/b1.so dev/b2.so dev/b4.so dev/b8.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
