#!/bin/bash
# Bollinger parity tests + config-4 shard timings (500 and 250 symbols per GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/q4
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "boll or tile or segment or config34 or random" > gpurun_out/q4/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/q4/pytest.log; [ $rc -ne 0 ] && exit $rc
for s in ${SYMS:-500 250}; do
  timeout -k 10 200 python3 bench.py --config ${CFG:-4} --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/q4/b_$s.log 2>&1 || { tail -5 gpurun_out/q4/b_$s.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/q4/b_$s.log').read().strip().splitlines()[-1]); print('config', d['config']['workload'][:17], $s, 'ms/step', round(d['ms_per_step'],3), 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
done
