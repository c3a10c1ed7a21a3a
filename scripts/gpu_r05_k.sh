#!/bin/bash
# Round 5: EMA chain values stored every 4th bar (libbt.so) / 2nd bar (dev/k2.so), the rest
# recomputed by the condition-word tasks — EMA parity first, then config 3 kernel time at 500 /
# 250 symbols against the same source storing every bar (dev/base.so), interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/k4
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_narrow.py tests/test_gpu_segments.py tests/test_gpu_fullsize.py tests/test_tile_edge_trades.py -m gpu -k "ema or config3 or config34 or random or narrow or tile_edge" > gpurun_out/r05/k4/tests.log 2>&1 || { tail -30 gpurun_out/r05/k4/tests.log; exit 1; }
tail -1 gpurun_out/r05/k4/tests.log
for rep in 1 2; do
  LIBS="libbt.so dev/base.so dev/k2.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
