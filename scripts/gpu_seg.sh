#!/bin/bash
# Segment tests + config-4 shards (auto split at 250 symbols) timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/seg
timeout -k 10 300 python -u -m pytest tests/test_gpu_segments.py -x -q --timeout 200 --timeout-method thread > gpurun_out/seg/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/seg/pytest.log; [ $rc -ne 0 ] && exit $rc
for s in 250 500; do
  timeout -k 10 200 python3 bench.py --config 4 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/seg/b4_$s.log 2>&1 || { tail -5 gpurun_out/seg/b4_$s.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/seg/b4_$s.log').read().strip().splitlines()[-1]); print($s, d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['value'])"
done
