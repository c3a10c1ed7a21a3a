#!/bin/bash
# The driver's N = 8 launch rehearsed on the one-GPU box: eight ranks share the device (gloo
# exchange, bench.py picks it when ranks outnumber GPUs), configs 2 (weak, 5,000 symbols per
# rank) and 4 (strong, its 8-GPU shards of 250 symbols) with --verify: rank 0 re-runs every
# rank's symbols in one engine and asserts the exchanged top-100 and counters equal it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06/n8; mkdir -p $O
for cfg in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29611 + cfg)) bench.py --gpus 8 --config $cfg --steps 5 --warmup 2 --verify > $O/n8_config$cfg.log 2>&1
  rc=$?; grep '^{' $O/n8_config$cfg.log | tail -1 | cut -c1-300; [ $rc -eq 0 ] || { tail -20 $O/n8_config$cfg.log; exit $rc; }
done
