#!/bin/bash
# Launch-variant / knob sweep with the profiling library: each ENVS entry
# ("NAME=V,NAME2=V2" or "-" for none) timed on the shards SYMS of config CFG (default 4), R
# interleaved rounds (e.g. ENVS="- BT_ONE_TRIP=1" CFG=2 SYMS=5000; ENVS="BT_LPW=32 BT_XW=3").
export BT_LIB=${BT_LIB:-dev/prof.so}
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/envs
for r in $(seq ${R:-2}); do
 for e in ${ENVS:--}; do
  for s in ${SYMS:-500 250}; do
    ( [ "$e" != "-" ] && for kv in ${e//,/ }; do export "$kv"; done
      timeout -k 10 200 python3 bench.py --config ${CFG:-4} --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/envs/b.log 2>&1 ) || { tail -5 gpurun_out/envs/b.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/envs/b.log').read().strip().splitlines()[-1]); print('round $r', '$e', $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
  done
 done
done
