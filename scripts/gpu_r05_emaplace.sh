#!/bin/bash
# Round 5: EMA pacing roles placed by the SIMD each wave landed on (dev/p1.so: walks twinned,
# scans twinned; dev/p2.so: walk beside the other block's scan), chains alone. EMA parity on
# both, then config 3 kernel time against the release map, interleaved twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/emaplace
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for lib in dev/p1.so dev/p2.so; do
  BT_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_narrow.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ema or config34" > gpurun_out/r05/emaplace/tests_$lib.log 2>&1 || { tail -20 gpurun_out/r05/emaplace/tests_$lib.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/r05/emaplace/tests_$lib.log)"
done
for rep in 1 2; do
  LIBS="libbt.so dev/p1.so dev/p2.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
