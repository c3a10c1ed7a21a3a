"""Profiling aid: shard kernel time with phases removed (BT_ABLATE bit masks; results are
meaningless, only the time is read).   [S=symbols] python scripts/ablate_probe.py CFG MASK [MASK ...]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation / stamps / launch overrides exist only in the profiling build (make PROFILING=1)
os.environ.setdefault("BT_LIB", "dev/prof.so")
cfg = int(sys.argv[1])
S_OVERRIDE = int(os.environ.get("S", "0"))
for m in sys.argv[2:]:
    os.environ["BT_ABLATE"] = m
    import dbx_amd as D
    grid = {2: D.config2_grid, 3: D.config3_grid, 4: D.config4_grid, 5: D.config5_grid}[cfg]()
    S, B, f = {2: (5000, 2520, D.BT_DAILY), 3: (500, 98280, D.BT_MINUTE),
               4: (500, 98280, D.BT_MINUTE), 5: (1250, 491400, D.BT_MINUTE)}[cfg]
    e = D.Engine(grid, timing=True)
    e.load_synthetic(0x5EED, 0, S_OVERRIDE or S, B, f)
    e.run(); e.sync(); e.reset_timing()
    for _ in range(3):
        e.run()
    e.sync()
    ms, n, _ = e.kernel_timing()
    print(f"cfg{cfg} mask {m}: kernel {ms / n:.3f} ms", flush=True)
    e.close()
