"""Turn one scripts/gpu_profile.sh run (gpurun_out/prof/NAME/) into the committed summary
profiles/TAG/NAME/: the rocprofv3 kernel-stats CSV, the bench JSON line of the same process,
the steady-state statistics of the dominant kernel (its last `steps` dispatches: the timed
region, warm-up excluded) and the PMC summary; with --pmc-ref also profiles/pmc_config<C>.json,
the measured traffic bench.py reports for that shard.

HBM bytes per launch (MI355X_MICROARCH.md §HBM): FETCH_SIZE / WRITE_SIZE are KiB from separate
--pmc passes; on gfx950 FETCH_SIZE reports 1/2 of a coalesced stream's read bytes, so
read bytes = 2 x FETCH_SIZE x 1024.

usage: python scripts/summarize_profile.py NAME TAG [--pmc-ref]"""
import collections
import csv
import glob
import json
import os
import shutil
import statistics
import sys

name, tag = sys.argv[1], sys.argv[2]
pmc_ref = "--pmc-ref" in sys.argv
src = os.path.join("gpurun_out", "prof", name)
dst = os.path.join("profiles", tag, name)
os.makedirs(dst, exist_ok=True)
line = json.loads([x for x in open(f"{src}/bench.log") if x.startswith("{")][-1])
kname = line["roofline"]["kernel"].split("::")[-1]
steps = line["steps"]

# One step launches the strategy kernel once, or, for a bar-split run, the speculative pass,
# one fix pass per boundary and the combine pass (k_tile.hip): a step's kernel time is the sum
# of its group of dispatches, the same span the bench line's HIP events bracket.
def ours(name):
    # SMA bar segments launch sma_seg_kernel (speculative + fix passes) and sma_seg_combine
    return kname in name or "seg_combine" in name or (kname == "sma_kernel" and "sma_seg_kernel" in name)


rows = list(csv.DictReader(open(glob.glob(f"{src}/trace/*kernel_trace.csv")[0])))
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in rows if ours(r["Kernel_Name"])]
per_step = max(1, len(durs) // (steps + line["warmup"]))
tail = durs[-steps * per_step:]
steady = [sum(tail[i:i + per_step]) for i in range(0, len(tail), per_step)]
stats_csv = glob.glob(f"{src}/trace/*kernel_stats.csv")[0]
shutil.copy(stats_csv, os.path.join(dst, "kernel_stats.csv"))
json.dump(line, open(os.path.join(dst, "bench.json"), "w"), indent=1)


def pmc(sub):
    """Per step (the PMC passes run --warmup 1 --steps 3: 4 steps): counters summed over the
    step's dispatches of our kernels."""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{src}/{sub}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if ours(r["Kernel_Name"]):
                agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: sum(d.values()) / 4 for c, d in agg.items()}


c = {}
for sub in ("fetch_size", "write_size", "sq_waves", "grbm_gui_active"):
    c.update(pmc(sub))
avg_steady_ns = statistics.mean(steady)
read_b = 2 * c.get("FETCH_SIZE", 0) * 1024
write_b = c.get("WRITE_SIZE", 0) * 1024
alg = line["roofline"]["alg_bytes_per_launch"]
summary = {
    "command": "python3 bench.py (see bench.json config) under rocprofv3 --kernel-trace --stats",
    "kernel": kname, "dispatches": len(durs), "dispatches_per_step": per_step, "steady_steps": len(steady),
    "steady_avg_ms": avg_steady_ns / 1e6, "steady_min_ms": min(steady) / 1e6,
    "steady_max_ms": max(steady) / 1e6, "all_dispatch_avg_ms": statistics.mean(durs) / 1e6,
    "bench_ms_per_step": line["ms_per_step"], "bench_kernel_avg_ms": line["roofline"]["kernel_avg_ms"],
    "avg_le_ms_per_step": avg_steady_ns / 1e6 <= line["ms_per_step"],
    "alg_bytes_per_launch": alg,
    "frac_from_rocprof_avg": alg / avg_steady_ns / 8000.0,
    "frac_in_bench_line": line["roofline"]["frac"],
    "FETCH_SIZE_KiB": c.get("FETCH_SIZE"), "WRITE_SIZE_KiB": c.get("WRITE_SIZE"),
    "hbm_read_bytes": read_b, "hbm_write_bytes": write_b,
    "hbm_bytes_per_launch": read_b + write_b,
    "hbm_GBps_measured": (read_b + write_b) / avg_steady_ns,
    "sq": {k: v for k, v in c.items() if k.startswith("SQ_")},
    "grbm": {k: v for k, v in c.items() if k.startswith("GRBM_")},
    "valu_busy_frac_est": c.get("SQ_ACTIVE_INST_VALU", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1),
    "wait_any_frac": c.get("SQ_WAIT_ANY", 0) / max(c.get("SQ_WAVE_CYCLES", 1), 1),
    "valu_issue_frac": c.get("SQ_INSTS_VALU", 0) / (avg_steady_ns * 1e-9) / 1e9 / (256 * 4 * 2.4 / 2),
    "effective_clock_ghz": c.get("GRBM_GUI_ACTIVE", 0) / 8 / (avg_steady_ns * 1e-9) / 1e9,
}
json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
if pmc_ref:
    cfg = int(line["config"]["workload"].split("config ")[1].split(":")[0])
    json.dump({"symbols": line["config"]["symbols_per_gpu"], "hbm_bytes_per_launch": read_b + write_b,
               "SQ_INSTS_VALU": c.get("SQ_INSTS_VALU"), "source": f"profiles/{tag}/{name}/pmc_summary.json"},
              open(os.path.join("profiles", f"pmc_config{cfg}.json"), "w"), indent=1)
print(json.dumps({k: summary[k] for k in ("kernel", "steady_avg_ms", "bench_ms_per_step", "avg_le_ms_per_step",
                                          "frac_from_rocprof_avg", "frac_in_bench_line", "hbm_GBps_measured",
                                          "wait_any_frac", "valu_issue_frac")}))
