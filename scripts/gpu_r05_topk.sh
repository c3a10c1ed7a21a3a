#!/bin/bash
# Round 5: does the top-k chain (second stream, overlapping the next step's kernel) slow the
# strategy kernel? Config 2 kernel time and step time with top-k 100 (default) and 0, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/topk
for rep in 1 2 3; do
  for k in 100 0; do
    timeout -k 10 200 python3 bench.py --topk $k --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r05/topk/b_$k.log 2>&1 || { tail -5 gpurun_out/r05/topk/b_$k.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r05/topk/b_$k.log').read().strip().splitlines()[-1]); print('topk $k kernel', round(d['roofline']['kernel_avg_ms'],4), 'ms/step', round(d['ms_per_step'],4))"
  done
done
