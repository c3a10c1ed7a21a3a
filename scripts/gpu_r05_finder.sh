#!/bin/bash
# Round 5: (current Bollinger change: libbt.so) vs the
# same source without (dev/base.so): Bollinger parity, then config 4 kernel time, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/finder
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_segments.py tests/test_gpu_narrow.py tests/test_gpu_fullsize.py tests/test_tile_edge_trades.py -m gpu -k "boll or config34 or narrow or tile_edge" > gpurun_out/r05/finder/tests.log 2>&1 || { tail -20 gpurun_out/r05/finder/tests.log; exit 1; }
tail -1 gpurun_out/r05/finder/tests.log
for rep in 1 2; do
  LIBS="libbt.so dev/base.so" CFG=4 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
