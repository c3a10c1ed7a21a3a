#!/bin/bash
# Round 6: per-kernel durations of the config-3 split run (250 symbols: speculative pass, fix pass,
# combine) at the round start and at HEAD, rocprofv3 kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/h; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for lib in dev/base.so libbt.so; do
  n=$(basename $lib .so)
  BT_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o $n -- python3 bench.py --config 3 --symbols 250 --steps 5 --warmup 2 --no-cpu-baseline > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['bar_segments'], d['roofline']['kernel_avg_ms'])"
  f=$(find $O/$n -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 $f | cut -c1-200
done
