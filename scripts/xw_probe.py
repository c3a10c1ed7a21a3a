"""Probe: Bollinger kernel time vs extra task-only waves (BT_XW) at the 8-GPU (250 symbols) and
4-GPU (500 symbols) config-4 shards.   python scripts/xw_probe.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation / stamps / launch overrides exist only in the profiling build (make PROFILING=1)
os.environ.setdefault("BT_LIB", "libbt_prof.so")
import dbx_amd as D
for S in (250, 500):
    for xw in (0, 2, 3, 4, 6):
        os.environ["BT_XW"] = str(xw)
        e = D.Engine(D.config4_grid(), timing=True)
        e.load_synthetic(0x5EED, 0, S, 98280, D.BT_MINUTE)
        e.run(); e.sync(); e.reset_timing()
        for _ in range(3):
            e.run()
        e.sync()
        ms, n, _ = e.kernel_timing()
        print(f"cfg4 S={S} xw={xw}: kernel {ms/n:.2f} ms", flush=True)
        e.close()
