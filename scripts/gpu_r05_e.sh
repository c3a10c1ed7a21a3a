#!/bin/bash
# Round 5: LDS pressure of the tile kernels and the SMA kernel (PMC: LDS instructions, bank /
# address conflicts, LDS issue stalls, SALU) on the config 2 / 3 / 4 shards, one pass each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r05/lds
export TMPDIR=/tmp
C="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES"
for cfg in "4 500" "3 500" "2 5000"; do
  set -- $cfg
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r05/lds/c$1 -o c$1 -- python3 bench.py --config $1 --symbols $2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r05/lds/c$1.log 2>&1 || { echo "pmc config $1 failed"; tail -5 gpurun_out/r05/lds/c$1.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for c in (4, 3, 2):
    f = glob.glob(f"gpurun_out/r05/lds/c{c}/**/*counter_collection.csv", recursive=True)
    if not f: print("no csv", c); continue
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if not ("tile_kernel" in k or "sma_kernel" in k): continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    d = {k: v / max(n[k], 1) * 1 for k, v in agg.items()}
    print(c, {k: f"{v:.4g}" for k, v in sorted(agg.items())}, "dispatch-rows", dict(n))
PY
