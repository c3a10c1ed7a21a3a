"""Probe: config-4 kernel time when the same bar-evals come as more, shorter symbols
(S x B/s for s = 1..8): the parallelism a bar-axis split would buy, before its fix-up cost.
  python scripts/seg_probe.py [cfg]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbx_amd as D
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
grid = D.config4_grid() if cfg == 4 else D.config3_grid()
for S0 in (500, 250):
    for s in (1, 2, 3, 4, 6, 8):
        e = D.Engine(grid, timing=True)
        e.load_synthetic(0x5EED, 0, S0 * s, 98280 // s, D.BT_MINUTE)
        e.run(); e.sync(); e.reset_timing()
        for _ in range(3):
            e.run()
        e.sync()
        ms, n, _ = e.kernel_timing()
        print(f"cfg{cfg} S0={S0} split={s}: {S0*s} x {98280//s} bars  kernel {ms/n:.2f} ms", flush=True)
        e.close()
