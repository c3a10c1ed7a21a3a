"""Profiling aid: time the SMA kernel with phases removed (env BT_ABLATE bit mask), interleaved
rounds in one process (cdna_hip_programming.md §5.4 rule 24). Outputs are wrong by design."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation / stamps / launch overrides exist only in the profiling build (make PROFILING=1)
os.environ.setdefault("BT_LIB", "dev/prof.so")
import dbx_amd as D

S = int(os.environ.get("S", 5000)); BARS = 2520
masks = [int(x) for x in os.environ.get("MASKS", "0,1,2,4,8,15").split(",")]
engines = {}
for m in masks:
    os.environ["BT_ABLATE"] = str(m)
    e = D.Engine(D.config2_grid(), timing=True)
    e.load_synthetic(0x5EED, 0, S, BARS, D.BT_DAILY)
    e.run(); e.sync(); e.reset_timing()
    engines[m] = e
res = {m: [] for m in masks}
for r in range(3):
    for m in masks:
        e = engines[m]
        e.reset_timing()
        for _ in range(3):
            e.run()
        e.sync()
        ms, n, _ = e.kernel_timing()
        res[m].append(ms / n)
names = {1: "scan+dst", 2: "keys", 4: "cmp", 8: "events"}
for m in masks:
    lab = "+".join(v for k, v in names.items() if m & k) or "full"
    print(f"skip {lab:28s} mask={m:3d}  min {min(res[m]):.3f} ms  all {[round(x,3) for x in res[m]]}")
