"""Randomised GPU parity sweep: seeded random grids, ragged series lengths and tie-prone price
paths for all three strategies, every result field and every trade bit-exact vs the C oracle.

The price paths are chosen to reach the kernels' rare branches: narrow integer walks (equal SMA
floor keys, exact SMA ties, flat stretches), plateaus, spikes near the 2^31-tick ceiling, and
lengths that end mid-tile, exactly on a tile edge or before the longest window fills.
"""
import os

import numpy as np
import pytest

import dbx_amd as D
from helpers import compare_summary, compare_trades, ema_stage_tiles, oracle_row

pytestmark = pytest.mark.gpu

CAP = 4096
# seeds per sweep (BT_RANDOM_SEEDS widens a sweep for a one-off deep run); the defaults are
# sized so the driver's round-end `-m gpu` run carries a few hundred random cases (~10 s)
NS = int(os.environ.get("BT_RANDOM_SEEDS", "0"))
S0 = int(os.environ.get("BT_RANDOM_SEED0", "0"))  # first seed of a deep run (fresh seeds)


def _series(rng, n, kind):
    if kind == "walk":          # ordinary tick walk around $100
        x = 1_000_000 + np.cumsum(rng.integers(-4000, 4001, n))
    elif kind == "narrow":      # a few ticks wide: floor keys and exact SMAs collide often
        x = 10_000 + np.cumsum(rng.integers(-1, 2, n))
        x = np.clip(x, 10_000, 10_004)
    elif kind == "plateau":     # long flat stretches with rare jumps
        x = 20_000 + 50 * np.cumsum(rng.random(n) < 0.03)
    else:                       # "spiky": near the int32 price ceiling with large moves
        x = 2_000_000_000 + np.cumsum(rng.integers(-3_000_000, 3_000_001, n))
    return np.clip(x, 10_000, 2**31 - 1).astype(np.int32)


def _ohlc(rng, c):
    hi = c + rng.integers(0, 3000, len(c)).astype(np.int64)
    lo = c - rng.integers(0, 3000, len(c)).astype(np.int64)
    return np.clip(hi, 1, 2**31 - 1).astype(np.int32), np.clip(lo, 1, 2**31 - 1).astype(np.int32)


def _windows(rng, k, top):
    return sorted(set(int(x) for x in rng.integers(1, top, k)))


@pytest.mark.parametrize("seed", range(S0, S0 + (NS or 120)))
def test_random_sma(seed):
    rng = np.random.default_rng(1000 + seed)
    grid = D.Grid.sma(_windows(rng, 7, 40), _windows(rng, 6, 300), annualization=252)
    kinds = ["walk", "narrow", "plateau", "spiky"]
    closes = [_series(rng, int(n), kinds[i % 4])
              for i, n in enumerate(rng.choice([1, 2, 63, 64, 65, 127, 128, 300, 777, 1500], 8))]
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_ohlc(closes)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s, cl in enumerate(closes):
        orc, otr = oracle_row("sma", grid, (cl, cl, cl, cl), 252, CAP)
        for p in range(grid.n_params):
            where = f"seed {seed} sym {s} len {len(cl)} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


@pytest.mark.parametrize("strategy,seed", [(st, s) for st in ("ema_ols", "boll") for s in range(S0, S0 + (NS or 40))])
def test_random_tile_strategies(strategy, seed):
    rng = np.random.default_rng(2000 + seed + (100 if strategy == "boll" else 0))
    if strategy == "ema_ols":
        grid = D.Grid.ema_ols(_windows(rng, 4, 200), _windows(rng, 4, 400),
                              band_bps=int(rng.integers(0, 60)))
    else:
        grid = D.Grid.boll(_windows(rng, 3, 120), sorted(set(int(x) for x in rng.integers(1, 7, 3))),
                           [int(x) for x in rng.integers(10, 300, 2)],
                           [int(x) for x in rng.integers(10, 500, 2)], k_den=2)
    kinds = ["walk", "narrow", "plateau", "spiky"]
    closes = [_series(rng, int(n), kinds[i % 4])
              for i, n in enumerate(rng.choice([1, 2, 64, 65, 129, 500, 2000], 6))]
    highs, lows = zip(*[_ohlc(rng, c) for c in closes])
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_ohlc(closes, list(highs), list(lows))
        e.run()
        got, tr = e.summaries(), e.trades()
    for s, cl in enumerate(closes):
        orc, otr = oracle_row(strategy, grid, (cl, highs[s], lows[s], cl), 98280, CAP)
        for p in range(grid.n_params):
            where = f"{strategy} seed {seed} sym {s} len {len(cl)} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


@pytest.mark.parametrize("strategy,seed", [(st, s) for st in ("sma", "ema_ols", "boll")
                                           for s in range(S0, S0 + (NS or 40))])
def test_random_product_kernels(strategy, seed):
    """The release instantiations (no trade lists: the split Bollinger walk, the SMA kernel's
    fast paths) on the same kinds of random grids and paths, every summary field vs the oracle."""
    rng = np.random.default_rng(3000 + seed + 100 * ("sma", "ema_ols", "boll").index(strategy))
    if strategy == "sma":
        grid = D.Grid.sma(_windows(rng, 7, 40), _windows(rng, 6, 300), annualization=252)
    elif strategy == "ema_ols":
        grid = D.Grid.ema_ols(_windows(rng, 4, 200), _windows(rng, 4, 400),
                              band_bps=int(rng.integers(0, 60)))
    else:
        # 64 lanes per k value (8 windows x 2 x 4 levels), as config 4: the launcher splits the
        # walk of the smallest k's wave into a finder and an accountant
        pick = lambda lo, hi, k: sorted(int(x) for x in rng.choice(np.arange(lo, hi), k, replace=False))
        grid = D.Grid.boll(pick(2, 121, 8), pick(1, 9, 4), pick(10, 300, 2), pick(10, 500, 4), k_den=2)
    kinds = ["walk", "narrow", "plateau", "spiky"]
    closes = [_series(rng, int(n), kinds[i % 4])
              for i, n in enumerate(rng.choice([1, 2, 64, 65, 129, 500, 2000, 3000], 8))]
    highs, lows = zip(*[_ohlc(rng, c) for c in closes])
    ann = 252 if strategy == "sma" else 98280
    with D.Engine(grid) as e:
        e.load_ohlc(closes, list(highs), list(lows))
        e.run()
        got = e.summaries()
    for s, cl in enumerate(closes):
        ohlc = (cl, cl, cl, cl) if strategy == "sma" else (cl, highs[s], lows[s], cl)
        orc, _ = oracle_row(strategy, grid, ohlc, ann, CAP)
        for p in range(grid.n_params):
            compare_summary(got[s, p], orc[p], f"{strategy} seed {seed} sym {s} len {len(cl)} {grid.param(p)}")


def _ema_grid_128(rng):
    """A random EMA+OLS grid that the launcher runs in 128-bar stages (helpers.ema_stage_tiles):
    short random spans and windows plus one OLS window long enough (1,300-2,600 bars) that
    64-bar stages would not fit more blocks per CU."""
    for _ in range(64):
        spans = _windows(rng, int(rng.integers(2, 9)), 800)
        wins = sorted(set(_windows(rng, 3, 400) + [int(rng.integers(1300, 2600))]))
        if ema_stage_tiles(spans, wins)[0] == 2:
            return D.Grid.ema_ols(spans, wins, band_bps=int(rng.integers(0, 60)))
    raise AssertionError("no 128-bar-stage grid drawn")


@pytest.mark.parametrize("parity,seed", [(p, s) for p in (True, False) for s in range(S0, S0 + (NS or 16))])
def test_random_ema_128bar_stages(parity, seed):
    """The 128-bar-stage EMA+OLS kernel (config 3's shape) on random grids and ragged paths: with
    trade lists (parity instantiation) and the release instantiation, every field vs the oracle."""
    rng = np.random.default_rng(4000 + seed + (500 if parity else 0))
    grid = _ema_grid_128(rng)
    kinds = ["walk", "narrow", "plateau", "spiky"]
    closes = [_series(rng, int(n), kinds[i % 4])
              for i, n in enumerate(rng.choice([1, 65, 129, 640, 2000, 3000, 4500], 6))]
    with D.Engine(grid, parity=parity, trade_cap=CAP if parity else 0) as e:
        e.load_ohlc(closes)
        e.run()
        got = e.summaries()
        tr = e.trades() if parity else None
    for s, cl in enumerate(closes):
        orc, otr = oracle_row("ema_ols", grid, (cl, cl, cl, cl), 98280, CAP)
        for p in range(grid.n_params):
            where = f"ema 128 seed {seed} sym {s} len {len(cl)} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            if parity:
                compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)
