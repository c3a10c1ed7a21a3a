"""Probe: tile-kernel time vs parameter waves per block (BT_PW) at a given shard size, for the
8-GPU (250 symbols) and 4-GPU (500 symbols) config-4 shards and the config-3 shard.
  python scripts/pw_probe.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation / stamps / launch overrides exist only in the profiling build (make PROFILING=1)
os.environ.setdefault("BT_LIB", "dev/prof.so")
import dbx_amd as D
cases = [(4, 250, (4, 2, 1)), (4, 500, (4, 2)), (3, 250, (1,)), (3, 500, (1,))]
for cfg, S, pws in cases:
    grid = D.config4_grid() if cfg == 4 else D.config3_grid()
    for pw in pws:
        os.environ["BT_PW"] = str(pw)
        e = D.Engine(grid, timing=True)
        e.load_synthetic(0x5EED, 0, S, 98280, D.BT_MINUTE)
        e.run(); e.sync(); e.reset_timing()
        for _ in range(3):
            e.run()
        e.sync()
        ms, n, _ = e.kernel_timing()
        print(f"cfg{cfg} S={S} pw={pw}: kernel {ms/n:.2f} ms", flush=True)
        e.close()
