#!/bin/bash
# Round-4 second refresh at HEAD (Bollinger walker / task VALU cuts, EMA task masks): the whole GPU
# suite, smoke, the driver's command profiled, config 3 and 4 shard profiles, the role stamps of
# both tile kernels (profiling build), the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu > gpurun_out/r04/pytest_gpu_final.log 2>&1 || { tail -30 gpurun_out/r04/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/r04/pytest_gpu_final.log
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/gpu_profile.sh config2 --gpus 1 --steps 20 --warmup 5 || exit 1
SHARDS='3 500|3 250|4 500|4 250'
IFS='|'; for spec in $SHARDS; do IFS=' '; set -- $spec
  bash scripts/gpu_profile.sh config$1_s$2 --config $1 --symbols $2 --steps 10 --warmup 2 || exit 1
done; IFS=' '
for c in 3 4; do timeout -k 10 120 python3 scripts/stamps_tile.py $c > gpurun_out/r04/stamps$c.txt 2>&1 || { tail -5 gpurun_out/r04/stamps$c.txt; exit 1; }; done
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.log 2>&1 || { tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
