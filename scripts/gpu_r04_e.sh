#!/bin/bash
# Round 4: config-3 regression bisect (libbt_en0 = EMA narrow off, libbt_en0l = also no flag LDS)
# and config 5 at HEAD (shard and whole workload) after restoring the 16-wave kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
for r in 1 2; do
  LIBS="libbt_base.so libbt.so libbt_en0.so libbt_en0l.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
LIBS="libbt_base.so libbt.so" CFG=5 SYMS="1250 10000" bash scripts/gpu_ab_libs.sh || exit 1
