#!/bin/bash
# Rehearsal of the N>1 bench path on a 1-GPU box: two ranks share the GPU (exchange over gloo).
# usage: bash scripts/gpu_n2.sh [bench.py args, e.g. --config 4]  -> gpurun_out/bench_n2*.log
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$(echo "$*" | tr -c 'a-z0-9' '_')
LOG=gpurun_out/bench_n2${TAG:+_$TAG}.log
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline "$@" > $LOG 2>&1; rc=$?
grep '^{' $LOG | cut -c1-600; exit $rc
