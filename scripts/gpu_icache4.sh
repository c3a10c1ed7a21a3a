#!/bin/bash
# Instruction-cache PMC (SQC_ICACHE_*) of the config-4 shard for each library in LIBS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/ic4; mkdir -p $O; export TMPDIR=/tmp
for lib in ${LIBS:-libbt.so}; do
  rm -rf $O/sq
  BT_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc ${CTRS:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH} --output-format csv -d $O/sq -o sq -- python3 bench.py --config ${CFG:-4} --symbols ${SYMS:-500} --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
  LIB=$lib python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(float)
for f in glob.glob("gpurun_out/ic4/sq/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "tile_kernel" in r["Kernel_Name"] or "sma_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(os.environ["LIB"], {k: f"{v / 4:.4g}" for k, v in sorted(agg.items())})
PY
done
