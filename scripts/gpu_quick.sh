#!/bin/bash
# Quick development call: a pytest selection (-k "$1"), then the config-2 bench and the
# per-GPU shard of configs given in $2 (e.g. "3 5"). Each GPU step is time-limited; stop on
# the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
K=${1:-}; CFGS=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$K" > gpurun_out/pytest_quick.log 2>&1; rc=$?
  grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_quick.log | tail -30 | cut -c1-300; tail -2 gpurun_out/pytest_quick.log
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1 || exit $?
cut -c1-420 gpurun_out/bench_quick.log
for c in $CFGS; do
  timeout -k 10 240 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/cfg$c.log 2>&1 || { cat gpurun_out/cfg$c.log | tail -5; exit 1; }
  cut -c1-400 gpurun_out/cfg$c.log
done
exit 0
