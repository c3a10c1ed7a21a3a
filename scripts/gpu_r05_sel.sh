#!/bin/bash
# Round 5: trade accounts with both sides' aggregate fields computed before the side selects
# (libbt.so) vs HEAD (dev/base.so): tile-kernel parity, then configs 4 and 3, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/sel
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_narrow.py tests/test_gpu_fullsize.py tests/test_tile_edge_trades.py -m gpu -k "boll or ema or config34 or narrow or tile_edge" > gpurun_out/r05/sel/tests.log 2>&1 || { tail -20 gpurun_out/r05/sel/tests.log; exit 1; }
tail -1 gpurun_out/r05/sel/tests.log
for rep in 1 2; do
  LIBS="libbt.so dev/base.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
  LIBS="libbt.so dev/base.so" CFG=3 SYMS="500" bash scripts/gpu_ab_libs.sh || exit 1
done
