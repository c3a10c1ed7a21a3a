#!/bin/bash
# Round 5: EMA chain replicas (libbt.so) vs the same source without (dev/base.so): the whole
# GPU suite on libbt.so, then config 3 kernel time at 500 / 250 symbols, interleaved twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/chainrep
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05/chainrep/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05/chainrep/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05/chainrep/pytest_gpu.log
for rep in 1 2; do
  LIBS="libbt.so dev/base.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
