#!/bin/bash
# Round 5: Bollinger hardware-wave role maps after the peels (profiling build, BT_WAVEMAP; nibble w =
# logical role of hardware wave w: 0-3 parameter groups (0 the finder), 4 helper, 5 accountant,
# 6-7 task waves). 45763210 is the release map.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/bmap
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2; do
  for m in 45763210 54763210 63475210 34762150; do
    for s in 500 250; do
      BT_LIB=dev/prof.so BT_WAVEMAP=$m timeout -k 10 200 python3 bench.py --config 4 --symbols $s --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r05/bmap/b_${m}_$s.log 2>&1 || { tail -5 gpurun_out/r05/bmap/b_${m}_$s.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/r05/bmap/b_${m}_$s.log').read().strip().splitlines()[-1]); print('map', '$m', 'config 4', $s, 'kernel', round(d['roofline']['kernel_avg_ms'],3))"
    done
  done
done
