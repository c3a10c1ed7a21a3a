#!/bin/bash
# Round 5: upper bounds by phase ablation (profiling build; timing only, results are not valid
# backtests). Config 4: no accountant records (4096), no walks (8). Config 3: no EMA chain (256),
# no walk (8), no condition-word tasks (2), no drawdown table (512).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/abl
for run in "4 0" "4 4096" "4 8" "3 0" "3 256" "3 8" "3 2" "3 512"; do
  set -- $run
  BT_LIB=dev/prof.so BT_ABLATE=$2 timeout -k 10 200 python3 bench.py --config $1 --symbols 500 --steps 10 --warmup 2 --no-cpu-baseline --topk 0 > gpurun_out/r05/abl/c$1_$2.log 2>&1 || { tail -5 gpurun_out/r05/abl/c$1_$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/abl/c$1_$2.log').read().strip().splitlines()[-1]); print('config', $1, 'ablate', $2, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
done
