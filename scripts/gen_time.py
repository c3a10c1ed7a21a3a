"""Time of the on-device synthetic generator (gen_kernel, outside every timed region) for the
config-2 and config-5 per-GPU shards.   python scripts/gen_time.py"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbx_amd as D  # noqa: E402
for name, grid, syms, bars, freq in (("config 2", D.config2_grid(), 5000, 2520, D.BT_DAILY),
                                     ("config 4", D.config4_grid(), 500, 98280, D.BT_MINUTE),
                                     ("config 5", D.config5_grid(), 1250, 491400, D.BT_MINUTE)):
    with D.Engine(grid) as e:
        e.load_synthetic(0x5EED, 0, syms, bars, freq); e.sync()
        t = time.perf_counter(); e.load_synthetic(0x5EED, 0, syms, bars, freq); e.sync()
        print(f"{name}: {syms} symbols x {bars} bars generated in {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
