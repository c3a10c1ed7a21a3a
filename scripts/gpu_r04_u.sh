#!/bin/bash
# Round 4: config 3 wave priorities (profiling build; BT_ABLATE bit 20 + 2-bit fields: chain at
# bit 16, walk at 18, helper A's scan at 22): the default (0, 2, 0) against a raised scan.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prio3
export BT_LIB=dev/prof.so
for rep in 1 2; do
for m in 1572864 5767168 9961472 14155776 5832704 10027008; do
  for s in 500 250; do
    BT_ABLATE=$m timeout -k 10 200 python3 bench.py --config 3 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prio3/b_${m}_$s.log 2>&1 || { tail -5 gpurun_out/prio3/b_${m}_$s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/prio3/b_${m}_$s.log').read().strip().splitlines()[-1]); print('ablate $m', $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
  done
done
done
