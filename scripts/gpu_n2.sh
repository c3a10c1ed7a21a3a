#!/bin/bash
# Rehearsal of the N>1 bench path on a 1-GPU box: two ranks share the GPU (exchange over gloo).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/bench_n2.log 2>&1; rc=$?
grep '^{' gpurun_out/bench_n2.log | cut -c1-400; exit $rc
