#!/bin/bash
# Round 6 item 5: the N > 1 step loop (two steps in flight) rehearsed with two ranks sharing the
# box's GPU (gloo exchange): config 4 (strong: 1,000 symbols per rank) and config 2 (weak), the
# per-rank exchange / host-wait / GPU-idle fields of the bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/${OUT:-t}; mkdir -p $O
export PYTHONUNBUFFERED=1 OMP_NUM_THREADS=4
for cfg in 4 2; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > $O/n2_c$cfg.log 2>&1 || { tail -20 $O/n2_c$cfg.log; exit 1; }
  grep '^{' $O/n2_c$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); pr=d['per_rank']; print('config $cfg', 'ms/step', round(d['ms_per_step'],3), 'kernel', [round(x,3) for x in pr['kernel_avg_ms']['by_rank']], 'exchange', [round(x,4) for x in pr['exchange_ms_per_step']['by_rank']], 'host_wait', [round(x,3) for x in pr['host_wait_ms_per_step']['by_rank']], 'depth', pr['pipeline_depth'], d['config']['parallelism'])"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_multirank.py -m gpu > $O/pytest_multirank.log 2>&1 || { tail -30 $O/pytest_multirank.log; exit 1; }
tail -2 $O/pytest_multirank.log
