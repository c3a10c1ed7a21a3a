import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "oracle"))
import numpy as np
import dbx_amd as D
import orc_ffi as F
grid = D.Grid.boll([3, 10, 45, 240], [1, 3, 6], [50, 100], [50, 400], k_den=2)
bars = 3000
o, h, lo, c, v = F.gen(0x5EED, 0, bars, 1)
with D.Engine(grid, parity=True, trade_cap=4096) as e:
    e.load_synthetic(0x5EED, 0, 1, bars, D.BT_MINUTE)
    e.run()
    got, tr = e.summaries(), e.trades()
for p in range(grid.n_params):
    kw = grid.param(p)
    s, otr = F.boll(h, lo, c, kw["w"], kw["k_num"], kw["k_den"], kw["sl"], kw["tp"], 98280, 4096)
    n = int(s["n_trades"]); ng = int(got[0, p]["n_trades"])
    if n != ng or int(s["hash"]) != int(got[0, p]["hash"]):
        g = tr[0, p][:ng]
        for i in range(max(n, ng)):
            a = tuple(int(x) for x in g[i]) if i < ng else None
            b = tuple(int(x) for x in otr[i]) if i < n else None
            if a != b:
                print("param", p, kw, "first diff at trade", i, "gpu", a, "orc", b)
                print("  prev gpu", [tuple(int(x) for x in t) for t in g[max(0,i-2):i+2]])
                print("  prev orc", [tuple(int(x) for x in t) for t in otr[max(0,i-2):i+2]])
                t0 = (a or b)[0]
                print("  bars", t0 - 2, "..", t0 + 4, "c", c[t0-2:t0+5].tolist(), "h", h[t0-2:t0+5].tolist(), "l", lo[t0-2:t0+5].tolist())
                break
