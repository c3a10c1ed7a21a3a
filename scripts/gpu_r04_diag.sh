#!/bin/bash
# Round 4 diagnostics: s_memtime stamps of the SMA kernel (config 2, config 5 on 1,250 symbols,
# the profiling build) and per-dispatch HBM bytes of one config-5 shard step (which of the
# segment kernel, fix passes and combine reads what).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r04/diag
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04/diag
timeout -k 10 120 python3 scripts/stamps.py > $O/stamps2.txt 2>&1 || { tail -5 $O/stamps2.txt; exit 1; }
cat $O/stamps2.txt
CFG=5 S=1250 timeout -k 10 200 python3 scripts/stamps.py > $O/stamps5.txt 2>&1 || { tail -5 $O/stamps5.txt; exit 1; }
cat $O/stamps5.txt
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | tr 'A-Z' 'a-z')
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o $n -- python3 bench.py --config 5 --scaling weak --symbols 1250 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_$n.log 2>&1 || { tail -5 $O/pmc_$n.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for sub in ("fetch_size", "write_size"):
    agg = collections.defaultdict(float)
    for f in glob.glob(f"gpurun_out/r04/diag/{sub}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            agg[(r["Dispatch_Id"], r["Kernel_Name"][:60])] += float(r["Counter_Value"])
    for (d, k), v in sorted(agg.items(), key=lambda x: int(x[0][0])):
        if v > 1024: print(sub, d, k, f"{v/1024/1024:.3f} GiB (KiB counter)")
PY
