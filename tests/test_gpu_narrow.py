"""GPU parity of the SMA kernel's narrow accounts (k_sma.hip SmaAcct): while the total variation
TV = sum |c_t - c_(t-1)| of a symbol's closes stays below 2^30 the walk keeps gap, mdd and the
realized pnl in int32, then moves them into int64 for the rest of the series. These series
cross the bound at different tiles (and bars inside a tile), one by a single jump of 2^25 ticks
or more (the scan's clamped-term branch), one never crosses and one is wide from its first tile;
every summary field and every trade must equal the C oracle's, in the release and the parity
instantiations."""
import numpy as np
import pytest

import dbx_amd as D
from helpers import compare_summary, compare_trades, oracle_row

CAP = 4096
BARS = 2520
LO, HI = 10_000, 2**31 - 2**20


def _walk(rng, c0, step, bars=BARS, lo=LO):
    c = np.empty(bars, np.int64)
    c[0] = c0
    d = rng.integers(-step, step + 1, bars)
    for t in range(1, bars):
        c[t] = min(max(c[t - 1] + d[t], lo), HI)
    return c


def _series():
    rng = np.random.default_rng(20261017)
    out = []
    for step in (1 << 20, 3 << 19, 1 << 21, 1 << 22, 1 << 23):  # TV crosses 2^30 late ... early
        out.append(_walk(rng, 1 << 28, step))
    c = _walk(rng, 1 << 27, 1 << 15)                            # a jump of 2^26 at bar 1,000
    c[1000:] = np.clip(c[1000:] + (1 << 26), LO, HI)
    out.append(c)
    out.append(_walk(rng, 5_000_000, 20_000))                   # TV ~ 2.5e7: narrow throughout
    out.append(_walk(rng, 1 << 30, 1 << 26, lo=1 << 28))       # steps past 2^25: wide at once
    return [x.astype(np.int32) for x in out]


def _first_wide_tile(c):
    """The kernel's rule (k_sma.hip stage_ring): per 64-bar tile TV grows by the clamped sum of
    |c_t - c_(t-1)|, or by 2^40 if one term reaches 2^25; tiles are narrow while TV < 2^30."""
    d = np.zeros(len(c), np.int64)
    d[1:] = np.abs(np.diff(c.astype(np.int64)))
    tv = 0
    for k in range((len(c) + 63) // 64):
        x = d[64 * k:64 * k + 64]
        tv += (1 << 40) if (x >= (1 << 25)).any() else int(np.minimum(x, 1 << 25).sum())
        if tv >= (1 << 30):
            return k
    return None


def test_series_cross_the_narrow_bound_where_intended():
    ks = [_first_wide_tile(c) for c in _series()]
    assert all(k is not None and 0 < k < BARS // 64 - 1 for k in ks[:6]), ks
    assert len(set(ks[:6])) == 6, ks          # six different crossing tiles
    assert ks[5] == 1000 // 64, ks            # the jump's tile (clamped-term branch)
    assert ks[6] is None and ks[7] == 0, ks
    for c in _series():  # valid input (docs/oracle_spec.md: |ret| <= 1, i.e. c_t <= 2 c_(t-1))
        c = c.astype(np.int64)
        assert c.min() >= 1 and (c[1:] <= 2 * c[:-1]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("parity", [False, True])
def test_sma_narrow_to_wide_accounts_match_oracle(parity):
    grid = D.config2_grid()
    closes = _series()
    kw = dict(parity=True, trade_cap=CAP) if parity else {}
    with D.Engine(grid, **kw) as e:
        e.load_ohlc(closes)
        e.run()
        got = e.summaries()
        tr = e.trades() if parity else None
    for s, cl in enumerate(closes):
        orc, otr = oracle_row("sma", grid, (cl, cl, cl, cl), 252, CAP if parity else 0)
        big = max(int(o["mdd"]) for o in orc)
        for p in range(grid.n_params):
            where = f"series {s} (first wide tile {_first_wide_tile(cl)}, max mdd {big}) {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            if parity:
                compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


def _level_fill_slack(h, lo, c):
    """tile_common.h level_fill_slack per bar: what an SL/TP fill at a level can add to the
    close path's total variation (twice this is added to TV)."""
    c = c.astype(np.int64)
    h = h.astype(np.int64)
    lo = lo.astype(np.int64)
    cp = np.concatenate([c[:1], c[:-1]])
    mlo, mhi = np.minimum(c, cp), np.maximum(c, cp)
    cl = lambda x: np.clip(x, 0, 1 << 24)
    return cl(mlo - lo) + cl(h - mhi) + cl(lo - c) + cl(c - h)


def _first_wide_tile_hl(h, lo, c):
    """The Bollinger scan's rule: per bar |c_t - c_(t-1)| + 2 x the level-fill slack."""
    d = np.zeros(len(c), np.int64)
    d[1:] = np.abs(np.diff(c.astype(np.int64)))
    d += 2 * _level_fill_slack(h, lo, c)
    tv = 0
    for k in range((len(c) + 63) // 64):
        x = d[64 * k:64 * k + 64]
        tv += (1 << 40) if (x >= (1 << 25)).any() else int(np.minimum(x, 1 << 25).sum())
        if tv >= (1 << 30):
            return k
    return None


WICK_BARS = 20_000


def _wick_series():
    """prices near 2^31, closes moving a few hundred ticks a bar (TV ~ 4e6,
    narrow by the closes alone), and wicks deep enough that every trade stops out at its level:
    each stop loses ~1e7-2e7 ticks, thousands of them push gap and mdd past 2^31. Series: both
    sides stopped on every bar; only longs stopped (shorts take normal wicks); deep wicks only
    from bar 12,000 on (narrow, then wide part-way); invalid bars (low above the close) that
    stop shorts a bar late."""
    rng = np.random.default_rng(99)
    B = WICK_BARS
    out = []
    base = (2_000_000_000 + np.cumsum(rng.integers(-400, 401, B))).astype(np.int64)
    deep_h = np.full(B, 2**31 - 1, np.int64)
    deep_l = np.full(B, 10_000, np.int64)
    near_h = base + rng.integers(0, 200, B)
    near_l = base - rng.integers(0, 200, B)
    out.append((deep_h, deep_l, base))
    out.append((near_h, deep_l, base))
    h3, l3 = near_h.copy(), near_l.copy()
    h3[12_000:], l3[12_000:] = deep_h[12_000:], deep_l[12_000:]
    out.append((h3, l3, base))
    l4 = deep_l.copy()
    l4[::7] = base[::7] + 3_000_000                      # l > c: the parser does not order OHLC
    out.append((deep_h, l4, base))
    return [tuple(x.astype(np.int32) for x in s) for s in out]


def test_wick_series_overflow_int32_without_the_level_slack():
    import orc_ffi as F
    grid = D.config4_grid()
    for i, (h, lo, c) in enumerate(_wick_series()):
        assert _first_wide_tile(c) is None, i           # the closes alone: narrow throughout
        k = _first_wide_tile_hl(h, lo, c)
        assert k is not None, i
        if i == 2:
            assert 12_000 // 64 <= k < WICK_BARS // 64 - 1, k
        # the busiest threshold (smallest k, the accountant's wave) runs past 2^31
        kw = grid.param(0)
        s, _ = F.boll(h, lo, c, kw["w"], kw["k_num"], kw["k_den"], kw["sl"], kw["tp"], 98280)
        assert int(s["mdd"]) > (2**29 if i == 1 else 2**31), (i, s)  # 1: short take-profits offset


@pytest.mark.gpu
@pytest.mark.parametrize("parity", [False, True])
def test_boll_level_fills_keep_wide_accounts(parity):
    """Stops filled at their levels move equity by ~ce·bps/1e4 however flat the closes are: the
    narrow flag must count the bars' wicks (tile_common.h level_fill_slack), else the int32
    accountant overflows. Every field vs the C oracle."""
    grid = D.config4_grid()
    series = _wick_series()
    kw = dict(parity=True, trade_cap=CAP) if parity else {}
    with D.Engine(grid, **kw) as e:
        e.set_segments(1)
        e.load_ohlc([s[2] for s in series], [s[0] for s in series], [s[1] for s in series])
        e.run()
        got = e.summaries()
        tr = e.trades() if parity else None
    for i, (h, lo, c) in enumerate(series):
        orc, otr = oracle_row("boll", grid, (c, h, lo, c), 98280, CAP if parity else 0)
        for p in range(grid.n_params):
            where = f"wick series {i} {grid.param(p)}"
            compare_summary(got[i, p], orc[p], where)
            if parity:
                compare_trades(tr[i, p], otr[p], min(int(orc[p]["n_trades"]), CAP), where)


@pytest.mark.gpu
@pytest.mark.parametrize("parity", [False, True])
def test_boll_narrow_to_wide_accounts_match_oracle(parity):
    """The Bollinger kernel's accountant (the split walk of the busiest z threshold) keeps gap and
    mdd in int32 on the same total-variation bound (tile_common.h Acct32); the same series, with
    highs and lows around the closes, through the config-4 grid."""
    grid = D.config4_grid()
    rng = np.random.default_rng(7)
    closes = _series()
    highs = [np.clip(c.astype(np.int64) + rng.integers(0, 1 << 16, len(c)), 1, 2**31 - 1).astype(np.int32)
             for c in closes]
    lows = [np.clip(c.astype(np.int64) - rng.integers(0, 1 << 16, len(c)), 1, 2**31 - 1).astype(np.int32)
            for c in closes]
    kw = dict(parity=True, trade_cap=CAP) if parity else {}
    with D.Engine(grid, **kw) as e:
        e.set_segments(1)                     # whole-series walks: the narrow path is SEG-free
        e.load_ohlc(closes, highs, lows)
        e.run()
        assert e.last_segments() == 1
        got = e.summaries()
        tr = e.trades() if parity else None
    for s, cl in enumerate(closes):
        orc, otr = oracle_row("boll", grid, (cl, highs[s], lows[s], cl), 98280, CAP if parity else 0)
        for p in range(grid.n_params):
            where = f"boll series {s} (first wide tile {_first_wide_tile(cl)}) {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            if parity:
                compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


EMA_BARS = 20_000


def _ema_series():
    """1-minute-like walks whose total variation crosses 2^30 at different tiles after the
    config-3 grid's 1,560-bar warm-up, one narrow throughout and one wide from its first tile."""
    rng = np.random.default_rng(31)
    out = [_walk(rng, 1 << 28, step, bars=EMA_BARS) for step in (120_000, 160_000, 230_000, 400_000)]
    out.append(_walk(rng, 5_000_000, 2_000, bars=EMA_BARS))           # TV ~ 2e7: narrow
    out.append(_walk(rng, 1 << 30, 1 << 26, bars=EMA_BARS, lo=1 << 28))  # wide at once
    return [x.astype(np.int32) for x in out]


def test_ema_series_cross_the_narrow_bound_after_warm_up():
    ks = [_first_wide_tile(c) for c in _ema_series()]
    assert all(k is not None and 1560 // 64 < k < EMA_BARS // 64 - 1 for k in ks[:4]), ks
    assert len(set(ks[:4])) == 4 and ks[4] is None and ks[5] == 0, ks


@pytest.mark.gpu
@pytest.mark.parametrize("parity", [False, True])
def test_ema_narrow_to_wide_accounts_match_oracle(parity):
    """The EMA+OLS walk keeps gap and mdd in int32 while the closes' total variation is below
    2^30 (k_tile.hip kEmaNarrow; fills are at closes, so the closes' TV bounds them), unsplit
    runs only: every field and trade vs the C oracle across the crossing tiles."""
    grid = D.config3_grid()
    closes = _ema_series()
    kw = dict(parity=True, trade_cap=CAP) if parity else {}
    with D.Engine(grid, **kw) as e:
        e.set_segments(1)
        e.load_ohlc(closes)
        e.run()
        assert e.last_segments() == 1
        got = e.summaries()
        tr = e.trades() if parity else None
    for s, cl in enumerate(closes):
        orc, otr = oracle_row("ema_ols", grid, (cl, cl, cl, cl), 98280, CAP if parity else 0)
        for p in range(grid.n_params):
            where = f"ema series {s} (first wide tile {_first_wide_tile(cl)}) {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            if parity:
                compare_trades(tr[s, p], otr[p], min(int(orc[p]["n_trades"]), CAP), where)
