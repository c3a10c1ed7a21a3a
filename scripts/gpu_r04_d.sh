#!/bin/bash
# Round 4: SMA segment lookback with 8 tiles in flight, compare depth 16 in 16-wave blocks (own
# kernel without the 80-VGPR cap) — SMA GPU tests, then config 5 A/B (shard and whole workload).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_narrow.py tests/test_gpu_random.py tests/test_gpu_fullsize.py tests/test_gpu_shards.py -m gpu -k "sma or SMA or config5 or config2 or 5" > gpurun_out/r04/pytest_d.log 2>&1 || { tail -30 gpurun_out/r04/pytest_d.log; exit 1; }
tail -1 gpurun_out/r04/pytest_d.log
for r in 1 2; do
  LIBS="dev/base.so libbt.so dev/c2.so dev/s16.so" CFG=5 SYMS="1250" bash scripts/gpu_ab_libs.sh || exit 1
done
LIBS="dev/base.so libbt.so" CFG=5 SYMS="10000" bash scripts/gpu_ab_libs.sh || exit 1
for r in 1 2; do
  LIBS="dev/base.so libbt.so dev/i128.so dev/hp.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
