#!/bin/bash
# A/B of two in-tree library builds (BT_LIB=libbt_base.so vs libbt.so), interleaved: config-2
# bench kernel/step time, and the per-GPU shards of the configs in CFGS (default 5).
# Build the baseline first: scripts/build_base.sh <git-rev>
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for r in 1 2 3; do for lib in libbt_base.so libbt.so; do
  BT_LIB=$lib timeout -k 10 100 python -u bench.py --no-cpu-baseline --steps 20 > gpurun_out/abl.log 2>&1 || { tail -3 gpurun_out/abl.log; exit 1; }
  echo "c2 $lib $(grep -o '"ms_per_step": [0-9.]*\|"kernel_avg_ms": [0-9.]*' gpurun_out/abl.log | tr '\n' ' ')"
done; done
for c in ${CFGS:-5}; do for lib in libbt_base.so libbt.so; do
  BT_LIB=$lib timeout -k 10 150 python -u bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/abl.log 2>&1 || { tail -3 gpurun_out/abl.log; exit 1; }
  echo "c$c $lib $(grep -o '"kernel_avg_ms": [0-9.]*' gpurun_out/abl.log)"
done; done
