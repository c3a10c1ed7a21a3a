#!/bin/bash
# Instruction-mix PMC of one bench shard (default config 4, 500 symbols): VALU/SALU/LDS counts,
# LDS bank conflicts and wave cycles, per step (kernel passes of one step summed).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/pmc4; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d $O/sq -o sq -- python3 bench.py --config ${CFG:-4} --symbols ${SYMS:-500} --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(float)
for f in glob.glob("gpurun_out/pmc4/sq/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "tile_kernel" in r["Kernel_Name"] or "seg_combine" in r["Kernel_Name"] or "sma_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
print({k: f"{v / 4:.4g}" for k, v in sorted(agg.items())})
PY
