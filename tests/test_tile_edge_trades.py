"""Trades at 64-bar tile edges: the walks peel the first trade of every tile (only it can start
with a position carried in from earlier tiles; later trades of the tile open inside it), so the
parity cases must hold both shapes often:

* a carried Bollinger position filled by SL/TP on the FIRST bar of a tile (the one fill whose
  path before the fill bar is empty in this tile: `k_tile.hip` boll walk, `qi < a.sb`);
* a carried position closed in a tile and further trades (or reversals) after it in the same
  tile (the non-first, merge-free walk iterations).

EMA+OLS runs 128-bar stages (two tiles per barrier) when they keep as many blocks per CU as
64-bar ones (`k_tile.hip ema_stage_tiles`): a long OLS window (1,560 bars, config 3's) puts the
`ema_ols_128` grid there, and its cases must also hold trades carried across a stage edge, exits
on a stage's first bar, entries on a stage's last bar and trades across the edge between a
stage's two tiles.

The CPU tests check that the seeded cases below contain these shapes (oracle trade lists); the
GPU test checks every field and trade of them bit-exact against the C oracle (oracle/oracle.c
orc_boll / orc_ema_ols / orc_sma, docs/oracle_spec.md §4).
"""
import numpy as np
import pytest

import dbx_amd as D
from helpers import compare_summary, compare_trades, ema_stage_tiles, oracle_row

CAP = 8192
T = 64


def _case(seed):
    rng = np.random.default_rng(7000 + seed)
    n = 3000 + int(rng.integers(0, 64))
    c = 1_000_000 + np.cumsum(rng.integers(-6000, 6001, n))
    c = np.clip(c, 10_000, 2**31 - 1).astype(np.int32)
    hi = np.clip(c + rng.integers(0, 9000, n), 1, 2**31 - 1).astype(np.int32)
    lo = np.clip(c - rng.integers(0, 9000, n), 1, 2**31 - 1).astype(np.int32)
    return c, hi, lo


GRIDS = {
    "boll": lambda: D.Grid.boll([4, 9, 30], [1, 2, 4], [5, 25], [5, 40], k_den=2),
    # more than one parameter wave: the launcher splits the walk of the busiest wave into a
    # finder and an accountant (k_tile.hip), so these shapes run through the trade records
    "boll_split": lambda: D.Grid.boll([4, 9, 30, 60], [1, 2, 4], [5, 25], [5, 40, 80], k_den=2),
    "ema_ols": lambda: D.Grid.ema_ols([3, 8, 40], [4, 16], band_bps=0),
    # 128-bar stages: the 1,560-bar window's prefix ring makes 64-bar stages no denser in LDS
    "ema_ols_128": lambda: D.Grid.ema_ols([3, 8, 40], [4, 16, 1560], band_bps=0),
    "sma": lambda: D.Grid.sma([2, 3, 7], [4, 11, 50]),
}
ANN = {"boll": 98280, "boll_split": 98280, "ema_ols": 98280, "ema_ols_128": 98280, "sma": 252}
STRATEGY = {"boll_split": "boll", "ema_ols_128": "ema_ols"}


def _shapes(trades, n, close):
    """(carried positions filled by SL/TP on a tile's first bar, tiles where a carried position
    closes and another trade then opens in the same tile)."""
    edge_fill = carried_then_more = 0
    tr = [(int(t["entry_bar"]), int(t["exit_bar"]), int(t["exit_px"])) for t in trades[:n]]
    for i, (e, x, px) in enumerate(tr):
        carried = e // T < x // T
        if carried and x % T == 0 and px != int(close[x]):
            edge_fill += 1
        if carried and i + 1 < len(tr) and tr[i + 1][0] // T == x // T:
            carried_then_more += 1
    return edge_fill, carried_then_more


def _stage_shapes(trades, n, S=2 * T):
    """Trades against S-bar stage edges: (carried across a stage edge, exits on a stage's first
    bar, entries on a stage's last bar, trades across the edge between a stage's two tiles)."""
    cross = first = last = mid = 0
    for t in trades[:n]:
        e, x = int(t["entry_bar"]), int(t["exit_bar"])
        cross += e // S < x // S
        first += x % S == 0 and e < x
        last += e % S == S - 1
        mid += e // S == x // S and e % S < T <= x % S
    return cross, first, last, mid


def test_stage_model_picks_the_kernels_shapes():
    """helpers.ema_stage_tiles mirrors the launcher's rule: config 3's block is 61,120 B at 64-bar
    and 80,208 B at 128-bar stages (k_tile.hip ema_stage_tiles), two per CU either way."""
    g3 = D.config3_grid()
    assert ema_stage_tiles(g3.axes[0], g3.axes[1]) == (2, 61120, 80208)
    # test_ema_stage_shapes' two cases: one of each shape
    assert ema_stage_tiles([10, 780], [1560, 15]) == (1, 54288, 66560)
    assert ema_stage_tiles([10, 780], [1700, 30]) == (2, 56336, 68608)
    assert ema_stage_tiles(*GRIDS["ema_ols_128"]().axes[:2])[0] == 2
    assert ema_stage_tiles(*GRIDS["ema_ols"]().axes[:2])[0] == 1


def test_cases_hold_stage_edge_shapes():
    grid = GRIDS["ema_ols_128"]()
    tot = np.zeros(4, np.int64)
    for seed in range(2):
        c, hi, lo = _case(seed)
        orc, otr = oracle_row("ema_ols", grid, (c, hi, lo, c), ANN["ema_ols_128"], CAP)
        for p in range(grid.n_params):
            tot += _stage_shapes(otr[p], int(orc[p]["n_trades"]))
    cross, first, last, mid = tot.tolist()
    assert cross >= 50 and mid >= 50, (cross, mid)
    assert first >= 10 and last >= 10, (first, last)


@pytest.mark.parametrize("strategy", ["boll", "boll_split", "ema_ols", "ema_ols_128", "sma"])
def test_cases_hold_tile_edge_shapes(strategy):
    grid = GRIDS[strategy]()
    edge = more = 0
    for seed in range(2):
        c, hi, lo = _case(seed)
        orc, otr = oracle_row(STRATEGY.get(strategy, strategy), grid, (c, hi, lo, c), ANN[strategy], CAP)
        for p in range(grid.n_params):
            assert int(orc[p]["n_trades"]) <= CAP
            a, b = _shapes(otr[p], int(orc[p]["n_trades"]), c)
            edge += a
            more += b
    if strategy.startswith("boll"):
        assert edge >= 5, f"only {edge} SL/TP fills on a tile's first bar"
    assert more >= 20, f"only {more} tiles with a carried close followed by another trade"


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["boll", "boll_split", "ema_ols", "ema_ols_128", "sma"])
def test_tile_edge_trades_gpu(strategy):
    grid = GRIDS[strategy]()
    cases = [_case(seed) for seed in range(2)]
    closes = [x[0] for x in cases]
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        if strategy == "sma":
            e.load_ohlc(closes)
        else:
            e.load_ohlc(closes, [x[1] for x in cases], [x[2] for x in cases])
        e.run()
        got, tr = e.summaries(), e.trades()
    for s, (c, hi, lo) in enumerate(cases):
        orc, otr = oracle_row(STRATEGY.get(strategy, strategy), grid, (c, hi, lo, c), ANN[strategy], CAP)
        for p in range(grid.n_params):
            where = f"{strategy} case {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)
