#!/bin/bash
# Instruction mix of one tile-kernel shard (default config 4, 500 symbols) under phase ablations
# of the profiling library (BT_ABLATE: 0 full, 8 no walks, 2 no condition-word / level tasks,
# 10 neither), two PMC passes per mask: (A) VALU / SALU / LDS instructions, VALU-active, wave and
# busy cycles, GRBM clock; (B) the VALU instruction classes (f64 add / mul / fma / trans, int64,
# int32, conversions). Results of ablated runs are wrong by design; only counts and times are read.
#   CFG=4 SYMS=500 MASKS="0 8 2 10" bash scripts/gpu_mix4.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/mix; mkdir -p $O; export TMPDIR=/tmp
PA="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
PB="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU"
for m in ${MASKS:-0 8 2 10}; do
  for p in A B; do
    [ $p = A ] && C="$PA" || C="$PB"
    BT_LIB=${LIB:-dev/prof.so} BT_ABLATE=$m timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/m$m$p -o sq -- python3 bench.py --config ${CFG:-4} --symbols ${SYMS:-500} --steps 3 --warmup 1 --no-cpu-baseline --topk 0 > $O/m$m$p.log 2>&1 || { tail -5 $O/m$m$p.log; exit 1; }
  done
  python3 - "$O/m$m" "$m" <<'PY'
import csv, glob, collections, json, sys
d, m = sys.argv[1], sys.argv[2]
out = {"mask": int(m)}
for p in "AB":
    agg = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(d + p + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "tile_kernel" in r["Kernel_Name"] or "sma_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    line = json.loads([l for l in open(d + p + ".log") if l.startswith("{")][-1])
    out["kernel_ms_" + p] = round(line["roofline"]["kernel_avg_ms"], 3)
    out.update({k + ("" if p == "A" or k != "SQ_INSTS_VALU" else "_B"): float(f"{v / max(n[k], 1):.4g}") for k, v in sorted(agg.items())})
print(json.dumps(out))
PY
done
