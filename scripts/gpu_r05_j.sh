#!/bin/bash
# Round 5: the EMA chain's per-bar LDS stores — config 3 kernel time with the chain's stores
# dropped (dev/ns.so, timing only: the condition words then read stale values) vs release.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/ns
for rep in 1 2; do
  LIBS="libbt.so dev/ns.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
