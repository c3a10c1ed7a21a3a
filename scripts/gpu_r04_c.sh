#!/bin/bash
# Round 4: stage 1 as a task (16-wave SMA blocks; dev/s1all.so: every SMA block) — GPU suite,
# the SMA parity subset with the all-blocks variant, then config 5 and config 2 A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_gpu_c.log 2>&1 || { tail -40 gpurun_out/r04/pytest_gpu_c.log; exit 1; }
tail -1 gpurun_out/r04/pytest_gpu_c.log
BT_LIB=dev/s1all.so timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_narrow.py tests/test_gpu_random.py -m gpu -k "sma or SMA" > gpurun_out/r04/pytest_s1all.log 2>&1 || { tail -30 gpurun_out/r04/pytest_s1all.log; exit 1; }
tail -1 gpurun_out/r04/pytest_s1all.log
for r in 1 2; do
  LIBS="dev/base.so libbt.so dev/c16.so" CFG=5 SYMS="1250" bash scripts/gpu_ab_libs.sh || exit 1
  LIBS="dev/base.so libbt.so dev/s1all.so" CFG=2 SYMS="5000" bash scripts/gpu_ab_libs.sh || exit 1
done
