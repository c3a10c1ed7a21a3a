#!/bin/bash
# Round 6: SQ counters of the config-3 split run (250 symbols), round start vs HEAD.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/r06/j; mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for lib in dev/base.so libbt.so; do
  n=$(basename $lib .so)
  BT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/$n -o $n -- python3 bench.py --config 3 --symbols 250 --steps 3 --warmup 1 --no-cpu-baseline --topk 0 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  f=$(find $O/$n -name '*counter_collection.csv' | head -1)
  python3 - "$f" "$n" <<'PY'
import csv,sys,collections
rows=[r for r in csv.DictReader(open(sys.argv[1])) if 'ema_tile_kernel' in r['Kernel_Name']]
# last speculative dispatch (the largest SQ_WAVE_CYCLES of the final dispatches)
by=collections.defaultdict(dict)
for r in rows: by[r['Dispatch_Id']][r['Counter_Name']]=float(r['Counter_Value'])
ds=sorted(by, key=lambda d:int(d))
big=[d for d in ds if by[d].get('SQ_WAVE_CYCLES',0)>1e8]
d=big[-1]
print(sys.argv[2], {k:'%.4g'%v for k,v in sorted(by[d].items())})
PY
done
