#!/bin/bash
# Bench lines (with cpu_baseline) of the config 3/4/5 shards: gpurun_out/cpub/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/cpub
for spec in "3 500" "4 500" "5 1250"; do
  set -- $spec
  timeout -k 10 300 python3 bench.py --config $1 --symbols $2 --steps 10 --warmup 2 > gpurun_out/cpub/config$1_s$2.log 2>&1 || { tail -3 gpurun_out/cpub/config$1_s$2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cpub/config$1_s$2.log').read().strip().splitlines()[-1]); c=d['cpu_baseline']; print($1, $2, d['value'], c['value'], c['value_1t'], c['sample'][:120])"
done
