#!/bin/bash
# Round 4: 120-B SMA segment records (SMA segment / full-size tests), segment counts for config
# 5's shard (automatic count: 5), base vs HEAD on that shard.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_segments.py tests/test_gpu_fullsize.py tests/test_gpu_shards.py -m gpu -k "sma or SMA or 5 or 2" > gpurun_out/r04/pytest_f.log 2>&1 || { tail -30 gpurun_out/r04/pytest_f.log; exit 1; }
tail -1 gpurun_out/r04/pytest_f.log
for G in 4 5 6 8; do
  timeout -k 10 200 python3 bench.py --config 5 --symbols 1250 --segments $G --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04/c5_G$G.log 2>&1 || { tail -5 gpurun_out/r04/c5_G$G.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/c5_G$G.log').read().strip().splitlines()[-1]); print('config 5 1250 G', $G, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
done
LIBS="dev/base.so libbt.so dev/base.so libbt.so" CFG=5 SYMS="1250" bash scripts/gpu_ab_libs.sh || exit 1
