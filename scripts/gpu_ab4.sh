#!/bin/bash
# Bollinger parity tests on the release build, then an interleaved A/B of in-tree builds (LIBS)
# on the config-4 shards (SYMS). Output under gpurun_out/ab4/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ab4
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "${TESTS:-boll or tile or segment or config34 or random}" > gpurun_out/ab4/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ab4/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in ${ROUNDS:-1 2}; do
 for lib in ${LIBS:-libbt.so}; do
  for s in ${SYMS:-500 250}; do
    BT_LIB=$lib timeout -k 10 200 python3 bench.py --config ${CFG:-4} --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab4/b_${lib}_$s.log 2>&1 || { tail -5 gpurun_out/ab4/b_${lib}_$s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab4/b_${lib}_$s.log').read().strip().splitlines()[-1]); print('round $r', '$lib', 'config', ${CFG:-4}, $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3), 'ms/step', round(d['ms_per_step'],3))"
  done
 done
done
