#!/bin/bash
# Round 4: the level-fill slack in the Bollinger narrow flag. The new wick-series
# test against the pre-fix library (expected to FAIL: int32 accountant overflow) and against the
# fixed one, then the whole GPU suite and the config-4 shards' kernel times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
BT_LIB=dev/pre.so timeout -k 10 300 $T tests/test_gpu_narrow.py -m gpu -k level_fills > gpurun_out/r04/narrow_pre.log 2>&1
rc=$?; echo "pre-fix library: rc=$rc (1 = the test caught the overflow)"; tail -3 gpurun_out/r04/narrow_pre.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 $T tests -m gpu > gpurun_out/r04/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04/pytest_gpu.log
for s in 500 250; do
  timeout -k 10 200 python3 bench.py --config 4 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04/c4_$s.log 2>&1 || { tail -5 gpurun_out/r04/c4_$s.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/c4_$s.log').read().strip().splitlines()[-1]); print('config 4', $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3), 'ms/step', round(d['ms_per_step'],3))"
done
