#!/bin/bash
# Tile-kernel development call: GPU parity tests of the tile strategies, then per-role stamps and
# the per-GPU shard throughput of the given configs (default "3 4"). Stops on the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
CFGS=${1:-"3 4"}; K=${2:-"boll or tile or config34 or lane"}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/pt.log 2>&1; rc=$?
tail -4 gpurun_out/pt.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
for c in $CFGS; do
  timeout -k 10 120 python -u scripts/stamps_tile.py $c || exit 1
  timeout -k 10 120 python -u bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline | cut -c1-300 || exit 1
done
