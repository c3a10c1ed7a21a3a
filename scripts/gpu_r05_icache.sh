#!/bin/bash
# Round 5: instruction-cache behaviour of the strategy kernels (SQC_ICACHE_* in one --pmc pass
# per config; a short bench run each).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/icache
export TMPDIR=/tmp
for spec in "2 5000" "3 500" "4 500"; do
  set -- $spec
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d gpurun_out/r05/icache/c$1 -o p -- python3 bench.py --config $1 --symbols $2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r05/icache/c$1.log 2>&1 || { echo "pmc config $1 failed"; tail -5 gpurun_out/r05/icache/c$1.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for c in (2, 3, 4):
    f = glob.glob(f"gpurun_out/r05/icache/c{c}/**/*counter_collection.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "tile_kernel" in k or "sma_kernel" in k:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    last = per[sorted(per, key=int)[-1]]
    req, miss = last["SQC_ICACHE_REQ"], last["SQC_ICACHE_MISSES"]
    print("config", c, {k: "%.3g" % v for k, v in last.items()}, "miss rate %.4f" % (miss / max(req, 1)))
PY
