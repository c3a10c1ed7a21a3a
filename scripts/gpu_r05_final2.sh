#!/bin/bash
# Round 5 final: the whole GPU suite, smoke and the default bench line at HEAD, then config 4's
# shards re-profiled and the config-4 stamps (profiling build).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05
NO_PROFILE=1 bash scripts/gpu_r05_final.sh || exit 1
bash scripts/gpu_r05_c4prof.sh || exit 1
