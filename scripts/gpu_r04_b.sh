#!/bin/bash
# Round 4, second GPU call: config 2 and config 5 A/B (dev/base.so = round-3 kernels + the
# narrow fix, libbt.so = working tree, libbt_c<N>.so = N key-row pairs in flight in the 16-wave
# compare), then the diagnostics (stamps, per-dispatch HBM bytes of a config-5 step).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
LIBS="dev/base.so libbt.so dev/co.so dev/base.so libbt.so dev/co.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
LIBS="dev/base.so libbt.so dev/hp.so dev/base.so libbt.so dev/hp.so" CFG=2 SYMS="5000" bash scripts/gpu_ab_libs.sh || exit 1
LIBS="dev/base.so libbt.so dev/c4.so dev/c8.so dev/c16.so libbt.so dev/c4.so dev/c8.so" CFG=5 SYMS="1250" bash scripts/gpu_ab_libs.sh || exit 1
bash scripts/gpu_r04_diag.sh
