#!/bin/bash
# Interleaved A/B/C... of in-tree library builds named in LIBS (default "libbt_base.so libbt.so"):
# config-2 bench kernel/step time, R rounds (default 3), then the shards of the configs in CFGS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
LIBS=${LIBS:-"libbt_base.so libbt.so"}
for r in $(seq ${R:-3}); do for lib in $LIBS; do
  BT_LIB=$lib timeout -k 10 100 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/libs.log 2>&1 || { tail -3 gpurun_out/libs.log; exit 1; }
  echo "c2 $lib $(grep -o '"ms_per_step": [0-9.]*\|"kernel_avg_ms": [0-9.]*' gpurun_out/libs.log | tr '\n' ' ')"
done; done
for c in ${CFGS:-}; do for lib in $LIBS; do
  BT_LIB=$lib timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/libs.log 2>&1 || { tail -3 gpurun_out/libs.log; exit 1; }
  echo "c$c $lib $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/libs.log)"
done; done
