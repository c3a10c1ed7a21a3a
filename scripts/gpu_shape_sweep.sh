#!/bin/bash
# Launch-shape sweep of the profiling library: bar segments per symbol x task-only waves per
# block, interleaved over R rounds. CASES entries are "config:symbols:segments:extra_waves"
# (segments 0 = automatic; extra_waves "-" = the launcher's choice).
#   CASES="3:500:1:- 3:500:2:2" R=2 bash scripts/gpu_shape_sweep.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/shape
for r in $(seq ${R:-2}); do
  for c in ${CASES}; do
    IFS=: read cfg s g xw <<< "$c"
    if [ "$xw" = "-" ]; then unset BT_XW; else export BT_XW=$xw; fi
    BT_LIB=${LIB:-dev/prof.so} timeout -k 10 200 python3 bench.py --config $cfg --symbols $s --segments $g --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/shape/b.log 2>&1 || { tail -5 gpurun_out/shape/b.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/shape/b.log').read().strip().splitlines()[-1]); print('round $r', 'config $cfg symbols $s segments $g xw $xw', 'kernel', round(d['roofline']['kernel_avg_ms'],4), 'ms/step', round(d['ms_per_step'],4), d.get('bar_segments'))"
  done
done
