#!/bin/bash
# Kernel time on one GPU against the number of symbols (SIZES; config CFG, default 5): per-symbol
# cost of a small shard (config 5: 1,250 symbols per GPU at 8 GPUs) against larger ones.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c5
for s in ${SIZES:-1250 2500 1250 5000}; do
  timeout -k 10 200 python3 bench.py --config ${CFG:-5} --symbols $s --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/c5/b_$s.log 2>&1 || { tail -5 gpurun_out/c5/b_$s.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c5/b_$s.log').read().strip().splitlines()[-1]); print($s, 'kernel ms', round(d['roofline']['kernel_avg_ms'],2), 'per symbol us', round(d['roofline']['kernel_avg_ms']*1000/$s,2), 'bar-evals/s', '%.3g' % d['value'])"
done
