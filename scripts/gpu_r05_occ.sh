#!/bin/bash
# Round 5: one block per CU vs two — config 3 / 4 kernel time at 250-256 symbols unsplit
# (--segments 1: one block per CU) and with the automatic 2 bar segments (two per CU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/occ
for spec in "3 250 1" "3 250 0" "3 256 1" "3 128 1" "4 250 1" "4 250 0" "4 128 1"; do
  set -- $spec
  timeout -k 10 200 python3 bench.py --config $1 --symbols $2 --segments $3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/occ/c$1_$2_$3.log 2>&1 || { tail -5 gpurun_out/r05/occ/c$1_$2_$3.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/occ/c$1_$2_$3.log').read().strip().splitlines()[-1]); print('config $1 symbols $2 segments $3 kernel', round(d['roofline']['kernel_avg_ms'],3), d.get('bar_segments'))"
done
