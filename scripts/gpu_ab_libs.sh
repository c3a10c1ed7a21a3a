#!/bin/bash
# A/B of in-tree library builds (LIBS="libbt.so dev/v1.so ...", built beforehand with
# `make OUT=../libbt_vN.so BUILD=../build_vN EXTRA=-D...`): kernel time of one bench shard each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ab
for lib in ${LIBS:-libbt.so}; do
  for s in ${SYMS:-500 250}; do
    BT_LIB=$lib timeout -k 10 200 python3 bench.py --config ${CFG:-4} --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/b_${lib}_$s.log 2>&1 || { tail -5 gpurun_out/ab/b_${lib}_$s.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/b_${lib}_$s.log').read().strip().splitlines()[-1]); print('$lib', 'config', ${CFG:-4}, $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3), 'ms/step', round(d['ms_per_step'],3))"
  done
done
