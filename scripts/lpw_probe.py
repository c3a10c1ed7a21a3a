"""Probe: tile-kernel time vs parameter lanes per wave (BT_LPW) at the one-block-per-CU shards
(config 4 on 8 GPUs: 250 symbols; config 3 on 2 GPUs: 250 symbols).   python scripts/lpw_probe.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation / stamps / launch overrides exist only in the profiling build (make PROFILING=1)
os.environ.setdefault("BT_LIB", "libbt_prof.so")
import dbx_amd as D
for cfg, S in ((4, 250), (3, 250), (4, 500)):
    for lpw in (64, 32, 16):
        os.environ["BT_LPW"] = str(lpw)
        grid = D.config4_grid() if cfg == 4 else D.config3_grid()
        e = D.Engine(grid, timing=True)
        e.load_synthetic(0x5EED, 0, S, 98280, D.BT_MINUTE)
        e.run(); e.sync(); e.reset_timing()
        for _ in range(3):
            e.run()
        e.sync()
        ms, n, _ = e.kernel_timing()
        print(f"cfg{cfg} S={S} lpw={lpw}: kernel {ms / n:.2f} ms", flush=True)
        e.close()
