"""The algebra of SMA bar segments (k_sma.hip SEG + sma_seg_combine) on the CPU, at trade level.

A segment cannot see the entry of the trade open at its first bar (an SMA position is held from one
crossover to the next, often longer than any burn-in), so it records that trade's exit bar, fill
and path from the segment start, and keeps every other trade's drawdown as max-plus forms of the
unknown entering gap. This test cuts the C oracle's trade lists at random tile boundaries, builds
each segment's record the way the kernel does, folds them the way the combine kernel does, and
requires pnl, max drawdown, trade count, exposure and the additive hash of the whole series
(tests only: the oracle is the checker)."""
import numpy as np
import pytest

import orc_ffi as F

NEG = -(1 << 60)
M64 = (1 << 64) - 1


def mix(w):
    z = ((w ^ (w >> 29)) * 0xBF58476D1CE4E5B9) & M64
    return z ^ (z >> 32)


def agg(c, a, b):
    """Path aggregate of closes c[a..b]: max, min, max drawdown, max draw-up."""
    seg = c[a:b + 1].astype(np.int64)
    run_max = np.maximum.accumulate(seg)
    run_min = np.minimum.accumulate(seg)
    return (int(seg.max()), int(seg.min()), int((run_max - seg).max()), int((seg - run_min).max()))


def merge(x, y):
    if x is None:
        return y
    return (max(x[0], y[0]), min(x[1], y[1]), max(x[2], y[2], x[0] - y[1]), max(x[3], y[3], y[0] - x[1]))


def terms(side, ce, st, px):
    lg = side > 0
    lo = st[1] - ce if lg else ce - st[0]
    hi = st[0] - ce if lg else ce - st[1]
    path = st[2] if lg else st[3]
    pnl = px - ce if lg else ce - px
    return lo, hi, path, pnl


def segment_record(c, trades, S, E):
    """What a segment [S, E) of bars records (SmaSegRec)."""
    r = dict(ntr=0, e0=-1, x1=-1, px1=0, agg1=None, end_pos=0, end_e=-1, end_ce=0, end_agg=None,
             R=0, A=0, B=NEG, C=NEG, D=NEG, h=0, start_pos=0)
    for (e, x, side, ce, cx) in trades:
        if e < S <= x:                        # open at the first accounted bar: carried
            r["start_pos"] = side
            if x < E:
                r.update(x1=x, px1=cx, agg1=agg(c, S, x), ntr=r["ntr"] + 1)
            else:
                r.update(agg1=agg(c, S, E - 1) if E > S else None, end_pos=side, end_e=-1)
        elif S <= e < E:
            if r["e0"] < 0 and r["ntr"] == 0 and r["start_pos"] == 0:
                r["e0"] = e
            if x < E:
                lo, hi, path, pnl = terms(side, ce, agg(c, e, x), cx)
                A0, B0 = r["A"], r["B"]
                r["C"] = max(r["C"], A0 - lo)
                r["D"] = max(r["D"], B0 - lo, path)
                r["A"] = A0 - pnl
                r["B"] = max(B0, hi) - pnl
                r["R"] += pnl
                r["h"] = (r["h"] + mix(e | (x << 31) | ((side > 0) << 62))) & M64
                r["ntr"] += 1
            else:
                r.update(end_pos=side, end_e=e, end_ce=ce, end_agg=agg(c, e, E - 1))
    return r


def combine(recs):
    pos = e = ce = 0
    e0 = -1
    ag = None
    R = gap = mdd = 0
    h = ntr = 0
    for r in recs:
        ntr += r["ntr"]
        R += r["R"]
        h = (h + r["h"]) & M64
        if e0 < 0:
            e0 = r["e0"]
        if pos != 0:
            assert r["start_pos"] == pos
            if r["x1"] >= 0:
                lo, hi, path, pnl = terms(pos, ce, merge(ag, r["agg1"]), r["px1"])
                mdd = max(mdd, gap - lo, path)
                gap = max(gap, hi) - pnl
                R += pnl
                h = (h + mix(e | (r["x1"] << 31) | ((pos > 0) << 62))) & M64
            elif r["agg1"] is not None:
                ag = merge(ag, r["agg1"])
        mdd = max(mdd, gap + r["C"], r["D"])
        gap = max(gap + r["A"], r["B"])
        if r["end_pos"] == 0:
            pos = 0
        elif r["end_e"] >= 0:
            pos, e, ce, ag = r["end_pos"], r["end_e"], r["end_ce"], r["end_agg"]
    return dict(pnl=R, mdd=mdd, n_trades=ntr, hash=h, e0=e0)


@pytest.mark.parametrize("seed", range(6))
def test_segment_records_fold_to_the_whole_series(seed):
    rng = np.random.default_rng(seed)
    B = int(rng.integers(3000, 20000))
    c = np.clip(1_000_000 + np.cumsum(rng.integers(-2500, 2600, B)), 10_000, 2**31 - 1).astype(np.int32)
    ntiles = (B + 63) // 64
    checked = 0
    for f, s in ((3, 40), (10, 200), (25, 900), (60, 2500)):
        orc, tr = F.sma(c, f, s, 98280, 100000)
        n = int(orc["n_trades"])
        trades = [(int(t["entry_bar"]), int(t["exit_bar"]), int(t["side"]), int(t["entry_px"]),
                   int(t["exit_px"])) for t in tr[:n]]
        for G in (2, 3, 5):
            cuts = sorted(set(int(x) for x in rng.choice(np.arange(1, ntiles), G - 1, replace=False)))
            bounds = [0] + [64 * t for t in cuts] + [B]
            recs = [segment_record(c, trades, bounds[q], bounds[q + 1]) for q in range(len(bounds) - 1)]
            got = combine(recs)
            where = f"seed {seed} f={f} s={s} cuts={cuts}"
            assert got["pnl"] == int(orc["pnl"]), where
            assert got["mdd"] == int(orc["mdd"]), where
            assert got["n_trades"] == n, where
            assert got["hash"] == int(orc["hash"]), where
            assert (B - 1 - got["e0"] if n else 0) == int(orc["exposure"]), where
            checked += 1
    assert checked == 12
