#!/bin/bash
# E12 (stream priorities: kernels high, top-k chain low; dev/e12.so) against HEAD (dev/head7.so):
# the driver's bench line (config 2) and config 3, alternating libraries, four rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export PYTHONUNBUFFERED=1
O=gpurun_out/r06/e12; mkdir -p $O
for r in 1 2 3 4; do
  for lib in head7 e12; do
    for cfg in 2 3; do
      BT_LIB=dev/$lib.so timeout -k 10 200 python3 bench.py --config $cfg --steps 40 --warmup 5 --no-cpu-baseline > $O/b_${lib}_c${cfg}_$r.log 2>&1 || { tail -5 $O/b_${lib}_c${cfg}_$r.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/b_${lib}_c${cfg}_$r.log').read().strip().splitlines()[-1]); print('round $r $lib config $cfg step', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_avg_ms'],4))"
    done
  done
done
