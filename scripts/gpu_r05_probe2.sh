#!/bin/bash
# Round 5: what binds config 2's compare — probe builds (timing only): libbt_p1 doubles the
# compare's key-row LDS reads (results unused), libbt_p2 doubles its VALU on opaque copies,
# libbt_p3 both; against the release build, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/abl
for rep in 1 2; do
for lib in libbt.so dev/p1.so dev/p2.so dev/p3.so; do
  BT_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05/abl/p2_$lib.log 2>&1 || { tail -5 gpurun_out/r05/abl/p2_$lib.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05/abl/p2_$lib.log').read().strip().splitlines()[-1]); print('config 2 $lib kernel', round(d['roofline']['kernel_avg_ms'],4))"
done
done
