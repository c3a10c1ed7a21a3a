#!/bin/bash
# Round 5: EMA+OLS returns as a flags-round task (BT_EMA_RET_TASK) — EMA parity, then config 3
# kernel time at 500 / 250 symbols, interleaved against the same source built without it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/ret
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_narrow.py tests/test_gpu_segments.py tests/test_gpu_fullsize.py -m gpu -k "ema or config3 or config34 or random or narrow" > gpurun_out/r05/ret/tests.log 2>&1 || { tail -30 gpurun_out/r05/ret/tests.log; exit 1; }
tail -1 gpurun_out/r05/ret/tests.log
for rep in 1 2; do
  LIBS="libbt.so dev/base.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
