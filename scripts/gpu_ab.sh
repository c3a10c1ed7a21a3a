#!/bin/bash
# Interleaved A/B of in-tree library builds over several shards: R rounds, each running every
# LIBS entry on every CASES entry ("config:symbols"), printing the kernel average and step time.
#   LIBS="dev/base.so libbt.so" CASES="4:500 4:250 3:500 2:5000" R=3 bash scripts/gpu_ab.sh
# Libraries are built beforehand on the CPU: make -C .../csrc OUT=../dev/base.so BUILD=../build_base
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ab
for r in $(seq ${R:-2}); do
  for lib in ${LIBS:-libbt.so}; do
    for c in ${CASES:-4:500}; do
      cfg=${c%%:*}; s=${c##*:}
      BT_LIB=$lib timeout -k 10 200 python3 bench.py --config $cfg --symbols $s --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/ab/b.log 2>&1 || { tail -5 gpurun_out/ab/b.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/ab/b.log').read().strip().splitlines()[-1]); print('round $r', '$lib', 'config', $cfg, $s, 'kernel', round(d['roofline']['kernel_avg_ms'],4), 'ms/step', round(d['ms_per_step'],4), 'segments', d.get('bar_segments'))"
    done
  done
done
