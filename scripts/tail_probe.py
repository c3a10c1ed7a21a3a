"""Probe: config-2 SMA kernel time against the symbol count around whole rounds of resident
blocks (3 blocks per CU x 256 CUs = 768 per round), to size the last-round (tail) waste.
  python scripts/tail_probe.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbx_amd as D
grid = D.config2_grid()
for S in (3840, 4224, 4608, 4800, 5000, 5376, 6144):
    e = D.Engine(grid, timing=True)
    e.load_synthetic(0x5EED, 0, S, 2520, D.BT_DAILY)
    e.run(); e.sync(); e.reset_timing()
    for _ in range(10):
        e.run()
    e.sync()
    ms, n, _ = e.kernel_timing()
    print(f"S={S} rounds={S/768:.2f}: kernel {ms/n:.3f} ms, {ms/n/S*1e3:.3f} us/symbol", flush=True)
    e.close()
