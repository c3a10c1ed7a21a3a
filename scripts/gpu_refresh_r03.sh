#!/bin/bash
# Round-3 evidence refresh: GPU tests, smoke, the driver's bench command (profiled), the
# per-config shard profiles, the ingest leg, and the config-3/4 role stamps; all under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash scripts/gpu_tests.sh > /dev/null; rc=$?; tail -1 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/gpu_profile.sh config2 --gpus 1 --steps 20 --warmup 5 || exit 1
bash scripts/gpu_profile_cfgs.sh || exit 1
timeout -k 10 300 python3 bench.py --leg ingest --steps 5 --warmup 1 > gpurun_out/ingest.log 2>&1 || { tail -5 gpurun_out/ingest.log; exit 1; }
tail -1 gpurun_out/ingest.log | cut -c1-300
for c in 3 4; do timeout -k 10 120 python3 scripts/stamps_tile.py $c > gpurun_out/stamps$c.txt 2>&1 || exit 1; done
