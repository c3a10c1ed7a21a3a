#!/bin/bash
# Round 5: trade-parallel Bollinger kernel iteration — Bollinger parity (incl. the record-region
# overflow tests), config 4 timing vs the round-4 kernel (dev/r4.so), stamps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_gpu_narrow.py tests/test_gpu_segments.py -m gpu -k "boll or tile_strategies or lane_strategies or config34 or maximum" > gpurun_out/r05/boll_parity_d.log 2>&1 || { tail -40 gpurun_out/r05/boll_parity_d.log; exit 1; }
tail -1 gpurun_out/r05/boll_parity_d.log
for lib in libbt.so dev/r4.so; do
  for s in 500 250; do
    BT_LIB=$lib timeout -k 10 200 python3 bench.py --config 4 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/c4_${lib}_$s.log 2>&1 || { tail -5 gpurun_out/r05/c4_${lib}_$s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r05/c4_${lib}_$s.log').read().strip().splitlines()[-1]); print('$lib config 4', $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3), 'ms/step', round(d['ms_per_step'],3))"
  done
done
timeout -k 10 200 python3 scripts/stamps_tile.py 4 500 > gpurun_out/r05/stamps4.txt 2>&1 || { tail -5 gpurun_out/r05/stamps4.txt; exit 1; }
cat gpurun_out/r05/stamps4.txt
