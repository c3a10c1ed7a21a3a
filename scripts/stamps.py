"""Profiling aid: per-phase cycle shares of the SMA kernel (diagnostic s_memtime build,
BT_ABLATE=64). Shares only — stamps perturb the schedule (cdna_hip_programming.md §7)."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# ablation / stamps / launch overrides exist only in the profiling build (make PROFILING=1)
os.environ.setdefault("BT_LIB", "dev/prof.so")
os.environ["BT_ABLATE"] = os.environ.get("BT_ABLATE", "64")
import dbx_amd as D
from dbx_amd import engine as E
L = E.lib(); L.bt_read_debug.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
CFG = int(os.environ.get("CFG", "2"))
if CFG == 5:
    e = D.Engine(D.config5_grid(), timing=True)
    e.load_synthetic(0x5EED, 0, int(os.environ.get("S", 1250)), 491400, D.BT_MINUTE)
    NT = 7679
else:
    e = D.Engine(D.config2_grid(), timing=True)
    e.load_synthetic(0x5EED, 0, 5000, 2520, D.BT_DAILY)
    NT = 40
e.run(); e.sync()
buf = (C.c_uint64 * 16)()
L.bt_read_debug(e._h, buf, 16)
names = ["stage1(helper)", "stage2 keys", "compare", "ties+latch", "events", "tile-end", "barrier"]
for base, who in ((0, "param waves"), (8, "helper waves")):
    n = buf[base + 7]
    tot = sum(buf[base + i] for i in range(7))
    print(f"{who}: {n} waves, {tot / max(n,1) / NT:.0f} cycles per tile per wave")
    for i, nm in enumerate(names):
        print(f"   {nm:16s} {buf[base+i]/max(tot,1)*100:5.1f}%  {buf[base+i]/max(n,1)/NT:7.0f} cyc/tile")
ms, nl, _ = e.kernel_timing(); print("kernel ms (stamped build)", ms / nl)
