"""Profiling aid: where the tile kernels' waves run (profiling build, BT_ABLATE=64 stamps):
which blocks share a CU, and on which SIMDs each block's first 8 hardware waves landed.
python scripts/dev/placement.py 3|4 [symbols]"""
import collections
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("BT_LIB", "dev/prof.so")
os.environ["BT_ABLATE"] = os.environ.get("BT_ABLATE", "64")
import dbx_amd as D
from dbx_amd import engine as E

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
S = int(sys.argv[2]) if len(sys.argv) > 2 else 500
SLOTS, BLOCKS = 80, 1024
L = E.lib()
L.bt_read_debug.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
e = D.Engine(D.config3_grid() if cfg == 3 else D.config4_grid(), timing=True)
e.load_synthetic(0x5EED, 0, S, 98280, D.BT_MINUTE)
e.run()
e.sync()
n = SLOTS + 8 * BLOCKS
buf = (C.c_uint64 * n)()
L.bt_read_debug(e._h, buf, n)
cu_of, simds = {}, {}
for b in range(min(S, BLOCKS)):
    ids = [buf[SLOTS + 8 * b + w] for w in range(8)]
    if not all(ids):
        continue
    hw = [i & 0xFFFFFFFF for i in ids]
    xcc = [(i >> 32) & 0xF for i in ids]
    key = {(x, (h >> 13) & 7, (h >> 12) & 1, (h >> 8) & 15) for x, h in zip(xcc, hw)}
    assert len(key) == 1, (b, key)  # a block's waves share one CU
    cu_of[b] = key.pop()
    simds[b] = tuple((h >> 4) & 3 for h in hw)
by_cu = collections.defaultdict(list)
for b, k in cu_of.items():
    by_cu[k].append(b)
print(f"config {cfg}, {S} symbols: {len(cu_of)} blocks stamped on {len(by_cu)} CUs;",
      "blocks per CU:", dict(collections.Counter(len(v) for v in by_cu.values())))
print("SIMD patterns of hardware waves 0-7:", dict(collections.Counter(simds.values()).most_common(6)))
pairs = [v for v in by_cu.values() if len(v) == 2]
twins = sum(simds[a] == simds[b] for a, b in pairs)
print(f"CUs with two blocks: {len(pairs)}; same SIMD pattern in both: {twins}")
print("block-index gaps of co-resident pairs:",
      dict(collections.Counter(abs(a - b) for a, b in pairs).most_common(8)))
print("XCD of blocks 0-15:", [cu_of[b][0] for b in range(16) if b in cu_of])
for a, b in pairs[:6]:
    print(f"  CU {cu_of[a]}: block {a} SIMDs {simds[a]}  block {b} SIMDs {simds[b]}")
