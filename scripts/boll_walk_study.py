"""Offline study of the Bollinger walk's serial work (config-4 grid, oracle trade lists): how many
wave-iterations per 64-bar block-tile the kernel's walk needs under different schedules.

Per lane and tile an event is a trade closing in the tile, or a trade opened in the tile that
stays open past it; every lane also spends one iteration per tile on its end-of-tile check.
  * current kernel: each wave runs, per tile, the maximum over its 64 lanes of (events + 1);
  * lagged walk (lanes may trail the newest tile by up to D tiles, with the per-tile check
    counted): what a barrier step must run so no lane falls further behind;
  * narrower waves (32 or 16 lanes): the critical path per wave and the total wave-iterations.
    python scripts/boll_walk_study.py [n_sym] [bars]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import orc_ffi as F  # noqa: E402

W, K, SL, TP = [10, 20, 30, 45, 60, 90, 120, 240], [3, 4, 5, 6], [50, 100], [50, 100, 200, 400]
nsym = int(sys.argv[1]) if len(sys.argv) > 1 else 3
bars = int(sys.argv[2]) if len(sys.argv) > 2 else 98280
T = (bars + 63) // 64
params = [(iw, ik, isl, itp) for iw in range(8) for ik in range(4) for isl in range(2) for itp in range(4)]
P = len(params)
EV = np.zeros((nsym, P, T), np.int64)
for s in range(nsym):
    o, h, lo, c, v = F.gen(0x5EED, s, bars, 1)
    for p, (iw, ik, isl, itp) in enumerate(params):
        _, tr = F.boll(h, lo, c, W[iw], K[ik], 2, SL[isl], TP[itp], 98280, trades_cap=1 << 20)
        for e, x in zip(tr["entry_bar"], tr["exit_bar"]):
            EV[s, p, x // 64] += 1
            if e // 64 != x // 64:
                EV[s, p, e // 64] += 1
kmaj = np.array(sorted(range(P), key=lambda p: (params[p][1], params[p][0], params[p][2], params[p][3])))


def lagged(ev_all, D):
    g = ev_all[:, kmaj, :].reshape(nsym, P // 64, 64, T)
    if D == 0:
        return g.max(axis=2).sum() / (nsym * T)
    total = 0
    for s in range(nsym):
        for w in range(P // 64):
            ev = g[s, w]
            cs = np.concatenate([np.zeros((64, 1), np.int64), np.cumsum(ev, axis=1)], axis=1)
            back = np.zeros(64, np.int64)
            for k in range(T):
                back += ev[:, k]
                allowed = cs[:, k + 1] - cs[:, max(0, k - D + 1)]
                n = int(max(0, (back - allowed).max()))
                back = np.maximum(0, back - n)
                total += n
            total += int(back.max())
    return total / (nsym * T)


print(f"mean events per lane-tile {EV.mean():.2f}")
for D in (0, 1, 2, 4):
    print(f"wave-iterations per block-tile, lag D={D}: {lagged(EV + 1, D):.2f}")
for L in (64, 32, 16):
    g = (EV + 1)[:, kmaj, :].reshape(nsym, P // L, L, T)
    per = g.max(axis=2).mean()
    print(f"{L} lanes per wave: {per:.2f} iterations per wave-tile (critical path), "
          f"{per * P / L:.2f} wave-iterations per block-tile")
