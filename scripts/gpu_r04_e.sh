#!/bin/bash
# Round 4: config-3 regression bisect (libbt_en0 = EMA narrow off, libbt_en0l = also no flag LDS)
# and config 5 at HEAD (shard and whole workload) after restoring the 16-wave kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_segments.py tests/test_gpu_fullsize.py tests/test_gpu_shards.py tests/test_gpu_narrow.py -m gpu > gpurun_out/r04/pytest_e.log 2>&1 || { tail -30 gpurun_out/r04/pytest_e.log; exit 1; }
tail -1 gpurun_out/r04/pytest_e.log
for r in 1 2; do
  LIBS="dev/base.so libbt.so dev/csb.so dev/en0.so" CFG=3 SYMS="500 250" bash scripts/gpu_ab_libs.sh || exit 1
done
LIBS="dev/base.so libbt.so" CFG=5 SYMS="1250 10000" bash scripts/gpu_ab_libs.sh || exit 1
for G in 3 5 4; do
  timeout -k 10 200 python3 bench.py --config 5 --symbols 1250 --segments $G --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r04/c5_G$G.log 2>&1 || { tail -5 gpurun_out/r04/c5_G$G.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/c5_G$G.log').read().strip().splitlines()[-1]); print('config 5 1250 G', $G, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
done
bash scripts/gpu_refresh_r04.sh || exit 1
