#!/bin/bash
# Phase ablation of the Bollinger kernel with the profiling library (dev/prof.so): kernel time
# with the walk (8), the condition words (2) or both (10) removed. Results are NOT valid
# backtests (the profiling build's ablation drops work); timing only.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/abl
for ab in 0 8 2 10; do
  BT_LIB=dev/prof.so BT_ABLATE=$ab timeout -k 10 200 python3 bench.py --config ${CFG:-4} --symbols ${SYMS:-500} --steps 10 --warmup 2 --no-cpu-baseline --topk 0 > gpurun_out/abl/b_$ab.log 2>&1 || { tail -5 gpurun_out/abl/b_$ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abl/b_$ab.log').read().strip().splitlines()[-1]); print('ablate', $ab, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
done
