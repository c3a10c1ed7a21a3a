#!/bin/bash
# Round 5: config 2's sparse seventh parameter wave compared with four lanes per parameter
# (libbt.so) vs without (dev/base.so): SMA parity, then config 2 kernel time, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/quarter
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_random.py tests/test_gpu_segments.py tests/test_gpu_narrow.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sma or config2 or config5 or topk" > gpurun_out/r05/quarter/tests.log 2>&1 || { tail -30 gpurun_out/r05/quarter/tests.log; exit 1; }
tail -1 gpurun_out/r05/quarter/tests.log
for rep in 1 2 3; do
  LIBS="libbt.so dev/base.so" CFG=2 SYMS="5000" bash scripts/gpu_ab_libs.sh || exit 1
done
