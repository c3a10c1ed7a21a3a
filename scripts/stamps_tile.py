"""Profiling aid: per-role cycle shares of the tile kernels (diagnostic s_memtime build,
BT_ABLATE=64) on the config-3 / config-4 per-GPU shard. Shares only — stamps perturb the
schedule (cdna_hip_programming.md §7).   python scripts/stamps_tile.py 3|4"""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation / stamps / launch overrides exist only in the profiling build (make PROFILING=1)
os.environ.setdefault("BT_LIB", "dev/prof.so")
os.environ["BT_ABLATE"] = os.environ.get("BT_ABLATE", "64")
import dbx_amd as D
from dbx_amd import engine as E
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
S = int(sys.argv[2]) if len(sys.argv) > 2 else 500
L = E.lib(); L.bt_read_debug.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
grid = D.config3_grid() if cfg == 3 else D.config4_grid()
bars = 98280
ntiles = (bars + 63) // 64
e = D.Engine(grid, timing=True)
e.load_synthetic(0x5EED, 0, S, bars, D.BT_MINUTE)
e.run(); e.sync()
G = e.last_segments()
if G > 1:  # split run (speculative pass stamped): tiles per block incl. burn-in and lookback
    burn = max(64, (6 * max(grid.axes[0]) + 63) // 64) if cfg == 3 else 64
    look = (max(grid.axes[1] if cfg == 3 else grid.axes[0]) - 1 + 63) // 64
    ntiles = (ntiles + (G - 1) * (burn + look)) / G
    print(f"split run: {G} segments, ~{ntiles:.0f} tiles per block")
buf = (C.c_uint64 * 80)()
L.bt_read_debug(e._h, buf, 80)
roles = (("param waves", "helper A (scan)", "helper B (chain)", "task waves") if cfg == 3 else
         ("param wave 0", "param wave 1", "param wave 2", "param wave 3+", "helper (scan)", "task waves",
          "accountant"))
for role, who in enumerate(roles):
    n = max(buf[8 * role + 7], 1)
    w, b = buf[8 * role] / n / ntiles, buf[8 * role + 1] / n / ntiles
    x = [buf[8 * role + 2 + i] / n / ntiles for i in range(4)]
    print(f"config {cfg} {who:18s} waves {buf[8*role+7]:6d}  work {w:7.0f}  barrier {b:7.0f} cyc/tile"
          f"  [setup {x[0]:.0f} walk {x[1]:.0f} tile-end {x[2]:.0f} iters {x[3]:.2f}]"
          + (f" tasks: words {buf[8 * role + 6] / n / ntiles:.0f} levels {buf[64 + role] / n / ntiles:.0f}" if cfg == 4 else ""))
if cfg == 4:
    ids = [buf[56 + w] - 1 for w in range(8) if buf[56 + w]]
    print("block 0 hardware waves: SIMD", [(i >> 4) & 3 for i in ids], "wave slot", [i & 15 for i in ids], "CU", [(i >> 8) & 15 for i in ids])
ms, nl, _ = e.kernel_timing(); print("kernel ms (stamped build)", ms / max(nl, 1))
