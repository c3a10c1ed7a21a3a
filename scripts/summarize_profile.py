"""Turn one gpu_profile.sh run (gpurun_out/) into the committed profiles/<tag>/ summary and
profiles/pmc_sma_config2.json (the `traffic` bench.py reports).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB from
separate --pmc passes; on gfx950 FETCH_SIZE reports 1/2 of a coalesced stream's read bytes, so
read bytes = 2 x FETCH_SIZE x 1024 (checked below against the known close-array size)."""
import csv, collections, json, os, shutil, sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src, dst = "gpurun_out", os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)
K = "sma_kernel"


def per_dispatch(name, sub):
    rows = list(csv.DictReader(open(f"{src}/prof/{sub}/{sub}_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if K in r["Kernel_Name"]:
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: sum(d.values()) / len(d) for c, d in agg.items()}


fetch = per_dispatch("FETCH_SIZE", "fetch")["FETCH_SIZE"]
write = per_dispatch("WRITE_SIZE", "write")["WRITE_SIZE"]
sq = per_dispatch("sq", "sq")
grbm = per_dispatch("grbm", "grbm")
stats = list(csv.DictReader(open(f"{src}/prof/trace/trace_kernel_stats.csv")))
kstat = next(r for r in stats if K in r["Name"])
avg_ns = float(kstat["AverageNs"])
S, B, P = 5000, 2520, 400
read_bytes = 2 * fetch * 1024
write_bytes = write * 1024
out = {
    "kernel": kstat["Name"], "calls": int(kstat["Calls"]), "avg_ns": avg_ns,
    "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write,
    "read_bytes_corrected": read_bytes, "write_bytes": write_bytes,
    "hbm_bytes_per_launch": read_bytes + write_bytes,
    "known_bytes": {"close_array_read": S * B * 4, "summaries_written": S * P * 48,
                    "topk_keys_written": S * P * 8},
    "alg_bytes_per_launch_survey_model": S * B * (8 + 16 * 40) + 32 * S * P,
    "sq": sq, "grbm": grbm,
    "effective_clock_ghz": grbm.get("GRBM_GUI_ACTIVE", 0) / 8 / (avg_ns * 1e-9) / 1e9,
    "valu_busy_frac_est": sq.get("SQ_ACTIVE_INST_VALU", 0) / max(sq.get("SQ_WAVE_CYCLES", 1), 1),
}
json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
json.dump({"hbm_bytes_per_launch": out["hbm_bytes_per_launch"], "source": f"profiles/{tag}/pmc_summary.json"},
          open(os.path.join("profiles", "pmc_sma_config2.json"), "w"), indent=1)
shutil.copy(f"{src}/prof/trace/trace_kernel_stats.csv", os.path.join(dst, "kernel_stats.csv"))
for f in ("bench.log", "pytest_gpu.log", "smoke.log"):
    if os.path.exists(f"{src}/{f}"):
        shutil.copy(f"{src}/{f}", os.path.join(dst, f))
print(json.dumps({k: out[k] for k in ("avg_ns", "hbm_bytes_per_launch", "read_bytes_corrected", "write_bytes", "effective_clock_ghz")}, indent=1))
