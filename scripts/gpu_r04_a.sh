#!/bin/bash
# Round 4, first GPU call: the narrow-flag fix (pre-fix library must FAIL the new wick test),
# the whole GPU suite at the working tree, then interleaved A/B (dev/base.so = last commit,
# libbt.so = working tree, dev/sn.so = + int32 SEG accountant) of config 3 and 4 shards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
BT_LIB=dev/pre.so timeout -k 10 300 $T tests/test_gpu_narrow.py -m gpu -k level_fills > gpurun_out/r04/narrow_pre.log 2>&1
rc=$?; echo "pre-fix library: rc=$rc (1 = the test caught the overflow)"; grep -E "passed|failed" gpurun_out/r04/narrow_pre.log | tail -2
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04/pytest_gpu.log
BT_LIB=dev/sn.so timeout -k 10 300 $T tests/test_gpu_segments.py tests/test_gpu_shards.py tests/test_gpu_narrow.py -m gpu -k "boll or Boll or 4" > gpurun_out/r04/pytest_sn.log 2>&1 || { tail -30 gpurun_out/r04/pytest_sn.log; exit 1; }
tail -1 gpurun_out/r04/pytest_sn.log
for r in 1 2; do
  LIBS="dev/base.so libbt.so dev/en0.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
  LIBS="dev/base.so libbt.so dev/sn.so" CFG=4 SYMS="250" bash scripts/gpu_ab_libs.sh || exit 1
done
LIBS="dev/base.so libbt.so dev/hp.so libbt.so dev/hp.so" CFG=4 SYMS="500" bash scripts/gpu_ab_libs.sh || exit 1
