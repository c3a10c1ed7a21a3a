#!/bin/bash
# Launch-shape sweep of the Bollinger kernel (profiling library: BT_LPW lanes per parameter
# wave, BT_XW task-only waves) on config-4 shards; kernel times only.
export BT_LIB=${BT_LIB:-libbt_prof.so}  # profiling build (make PROFILING=1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/shape
for s in ${SYMS:-500}; do
IFS=, read -ra SPL <<< "${SPECS:-64 3,37 0,43 1,52 2,32 0,32 1}"
for spec in "${SPL[@]}"; do
  set -- $spec
  BT_LPW=$1 BT_XW=$2 timeout -k 10 200 python3 bench.py --config ${CFG:-4} --symbols $s --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/shape/b.log 2>&1 || { tail -3 gpurun_out/shape/b.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/shape/b.log').read().strip().splitlines()[-1]); print('syms', $s, 'lpw', $1, 'xw', $2, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
done; done
