#!/bin/bash
# Round 4: the SMA prefix ring stored twice when it fits (Grid::ring_mirror, R <= 2048: config 2),
# so the key stage reads a window's start with one add — dev/v18.so vs HEAD (dev/h18.so) on
# config 2 (the driver's line), then the whole GPU suite on v18.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ab
export PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for lib in dev/h18.so dev/v18.so; do
    BT_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab/c2_${lib}.log 2>&1 || { tail -5 gpurun_out/ab/c2_${lib}.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/c2_${lib}.log').read().strip().splitlines()[-1]); print('$lib config 2 kernel', round(d['roofline']['kernel_avg_ms'],4), 'ms/step', round(d['ms_per_step'],4))"
  done
done
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
BT_LIB=dev/v18.so timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_v.log 2>&1 || { tail -30 gpurun_out/r04/pytest_v.log; exit 1; }
tail -1 gpurun_out/r04/pytest_v.log
