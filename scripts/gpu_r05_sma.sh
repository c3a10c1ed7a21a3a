#!/bin/bash
# Round 5: an SMA kernel change (libbt.so) vs the same source without it (dev/base.so): SMA
# parity (incl. segments and the config-2 full shard), then config 2 and config 5's shard kernel
# times, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/sma
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_narrow.py tests/test_gpu_fullsize.py tests/test_tile_edge_trades.py -m gpu -k "sma or config2 or narrow or tile_edge" > gpurun_out/r05/sma/tests.log 2>&1 || { tail -20 gpurun_out/r05/sma/tests.log; exit 1; }
tail -1 gpurun_out/r05/sma/tests.log
for rep in 1 2 3; do
  LIBS="libbt.so dev/base.so" CFG=2 SYMS="5000" bash scripts/gpu_ab_libs.sh || exit 1
done
LIBS="libbt.so dev/base.so" CFG=5 SYMS="1250" bash scripts/gpu_ab_libs.sh || exit 1
