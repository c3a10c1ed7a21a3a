"""Offline study: walk iterations of the Bollinger kernel under different parameter->lane
orders (oracle trade lists, config-4 grid). A wave iterates, per 64-bar tile, the maximum over
its lanes of (trades exiting in the tile + 1 if a trade is open at the tile end); the sum over
waves and tiles is the walk's serial work.   python scripts/boll_lane_order.py [n_sym] [bars]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import orc_ffi as F

W, K, SL, TP = [10, 20, 30, 45, 60, 90, 120, 240], [3, 4, 5, 6], [50, 100], [50, 100, 200, 400]
nsym = int(sys.argv[1]) if len(sys.argv) > 1 else 3
bars = int(sys.argv[2]) if len(sys.argv) > 2 else 98280
T = (bars + 63) // 64
# params in result order ((iw * nk + ik) * nsl + isl) * ntp + itp
params = [(iw, ik, isl, itp) for iw in range(8) for ik in range(4) for isl in range(2) for itp in range(4)]
P = len(params)


def iters_per_tile(trades):
    it = np.zeros(T, np.int32)
    for e, x in trades:
        it[x // 64] += 1
        # open across tile ends: tiles e//64 .. x//64 - 1 end with the trade open
        if x // 64 > e // 64:
            it[e // 64: x // 64] += 1
    return it


ITER = np.zeros((nsym, P, T), np.int32)
for s in range(nsym):
    o, h, lo, c, v = F.gen(0x5EED, s, bars, 1)
    for p, (iw, ik, isl, itp) in enumerate(params):
        _, tr = F.boll(h, lo, c, W[iw], K[ik], 2, SL[isl], TP[itp], 98280, trades_cap=1 << 20)
        ITER[s, p] = iters_per_tile(zip(tr["entry_bar"], tr["exit_bar"]))


def cost(order):  # order: lane slot -> param index
    g = ITER[:, order, :].reshape(nsym, P // 64, 64, T)
    return g.max(axis=2).sum() / (nsym * T)


def key_order(key):
    return np.array(sorted(range(P), key=key))


mean = ITER.mean() * P / 64
print(f"mean lane iterations x waves per block-tile (lower bound): {mean:.2f}")
print("result order (w-major):", round(cost(np.arange(P)), 2))
print("k-major (current):", round(cost(key_order(lambda p: (params[p][1], params[p][0], params[p][2], params[p][3]))), 2))
print("tp-major:", round(cost(key_order(lambda p: (params[p][3], params[p][1], params[p][0], params[p][2]))), 2))
print("(sl,tp)-major:", round(cost(key_order(lambda p: (params[p][2] + params[p][3], params[p][3], params[p][1], params[p][0]))), 2))
print("k,tp-major:", round(cost(key_order(lambda p: (params[p][1], params[p][3], params[p][0], params[p][2]))), 2))
rate = ITER[0].sum(axis=1)  # symbol 0's trade-segment counts
print("sorted by symbol-0 rate:", round(cost(np.argsort(rate, kind="stable")), 2))
rate_all = ITER.sum(axis=(0, 2))
print("sorted by all-symbol rate:", round(cost(np.argsort(rate_all, kind="stable")), 2))


def iters_span(trades, span):
    n = (bars + span - 1) // span
    it = np.zeros(n, np.int32)
    for e, x in trades:
        it[x // span] += 1
        if x // span > e // span:
            it[e // span: x // span] += 1
    return it


for span in (128, 256):
    n = (bars + span - 1) // span
    IT = np.zeros((nsym, P, n), np.int32)
    for s in range(nsym):
        o, h, lo, c, v = F.gen(0x5EED, s, bars, 1)
        for p, (iw, ik, isl, itp) in enumerate(params):
            _, tr = F.boll(h, lo, c, W[iw], K[ik], 2, SL[isl], TP[itp], 98280, trades_cap=1 << 20)
            IT[s, p] = iters_span(zip(tr["entry_bar"], tr["exit_bar"]), span)
    order = key_order(lambda p: (params[p][1], params[p][0], params[p][2], params[p][3]))
    g = IT[:, order, :].reshape(nsym, P // 64, 64, n)
    print(f"walk span {span} bars, k-major: {g.max(axis=2).sum() / (nsym * T):.2f} per 64-bar block-tile")

# how the measured rate depends on the axes (for a grid-only ordering heuristic)
r = rate_all.reshape(8, 4, 2, 4).astype(float)
print("mean rate by w:", np.round(r.mean(axis=(1, 2, 3)), 0))
print("by k:", np.round(r.mean(axis=(0, 2, 3)), 0), "by sl:", np.round(r.mean(axis=(0, 1, 3)), 0),
      "by tp:", np.round(r.mean(axis=(0, 1, 2)), 0))
for name, key in (("k, then sl+tp", lambda p: (params[p][1], params[p][2] + params[p][3])),
                  ("sl+tp, then k", lambda p: (params[p][2] + params[p][3], params[p][1])),
                  ("w, then k", lambda p: (params[p][0], params[p][1])),
                  ("k+w", lambda p: (params[p][1] + params[p][0] / 2, params[p][2]))):
    print(name, round(cost(key_order(key)), 2))
