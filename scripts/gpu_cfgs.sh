#!/bin/bash
# throughput of configs 3, 4, 5 (per-GPU shards); each step time-limited, stop on crash/timeout
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for c in 3 4 5; do
  timeout -k 10 240 python -u bench.py --config $c "$@" > gpurun_out/cfg$c.log 2>&1; rc=$?
  cat gpurun_out/cfg$c.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
done
exit 0
