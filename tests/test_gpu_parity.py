"""GPU parity: the HIP engine (through the C ABI) vs the C oracle, bit-exact.

North_star bar: trade counts and entry/exit bars bit-exact; PnL/Sharpe/MDD within 1e-9
relative in fp64 (here every field is bit-exact, Sharpe included — see docs/oracle_spec.md §3).
"""
import os

import numpy as np
import pytest

import dbx_amd as D
from dbx_amd import engine as E
import orc_ffi as F
from helpers import compare_summaries, compare_summary, compare_trades, oracle_row

pytestmark = pytest.mark.gpu

CAP = 4096


def _gen(seed, syms, bars, freq):
    cols = [F.gen(seed, s, bars, freq) for s in syms]
    o = [c[0] for c in cols]
    h = [c[1] for c in cols]
    lo = [c[2] for c in cols]
    c = [c[3] for c in cols]
    return o, h, lo, c


def test_synthetic_generator_matches_oracle():
    g = D.config2_grid()
    with D.Engine(g) as e:
        e.load_synthetic(0x5EED, 4990, 10, 2520, D.BT_DAILY)
        for i in (0, 3, 9):
            got = e.close_column(i, 2520)
            exp = F.gen(0x5EED, 4990 + i, 2520, 0)[3]
            assert np.array_equal(got, exp)
    with D.Engine(D.config4_grid()) as e:  # minute bars, high/low columns generated too
        e.load_synthetic(7, 3, 2, 5000, D.BT_MINUTE)
        assert np.array_equal(e.close_column(1, 5000), F.gen(7, 4, 5000, 1)[3])


@pytest.mark.parametrize("bars", [700, 64, 65, 1, 2, 130])
def test_sma_parity_synthetic(bars):
    grid = D.Grid.sma([2, 4, 6, 10, 42], [3, 50, 120, 240, 600], annualization=252)
    syms = list(range(5))
    o, h, lo, c = _gen(0x5EED, syms, bars, 0)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(0x5EED, 0, len(syms), bars, D.BT_DAILY)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s in syms:
        orc, otr = oracle_row("sma", grid, (o[s], h[s], lo[s], c[s]), 252, CAP)
        for p in range(grid.n_params):
            where = f"sym {s} param {grid.param(p)} bars {bars}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


def test_sma_parity_ragged_and_edges(golden_dir):
    import json, os
    edge = json.load(open(os.path.join(golden_dir, "edge.json")))
    closes = [np.array(x["c"], np.int32) for x in edge]
    grid = D.Grid.sma([2, 3, 4], [3, 5, 50], annualization=252)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_ohlc(closes)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s, cl in enumerate(closes):
        orc, otr = oracle_row("sma", grid, (cl, cl, cl, cl), 252, CAP)
        for p in range(grid.n_params):
            where = f"{edge[s]['name']} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


def test_sma_sums_exact():
    grid = D.Grid.sma([4, 10], [50, 60], annualization=252)
    o, h, lo, c = _gen(11, [0, 1], 900, 0)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(11, 0, 2, 900, D.BT_DAILY)
        e.run()
        sums = e.sums()
    for s in range(2):
        orc, _ = oracle_row("sma", grid, (o[s], h[s], lo[s], c[s]), 252)
        for p in range(grid.n_params):
            assert F.i128(sums[s, p]["s1_lo"], sums[s, p]["s1_hi"]) == F.i128(orc[p]["s1_lo"], orc[p]["s1_hi"])
            assert F.i128(sums[s, p]["s2_lo"], sums[s, p]["s2_hi"]) == F.i128(orc[p]["s2_lo"], orc[p]["s2_hi"])


@pytest.mark.parametrize("strategy", ["ema_ols", "boll"])
def test_lane_strategies_parity(strategy):
    if strategy == "ema_ols":
        grid = D.Grid.ema_ols([3, 10, 60, 390], [4, 15, 120, 780], band_bps=20)
    else:
        grid = D.Grid.boll([3, 10, 45, 240], [1, 3, 6], [50, 100], [50, 400], k_den=2)
    bars = 3000
    o, h, lo, c = _gen(0x5EED, [0, 1, 2], bars, 1)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(0x5EED, 0, 3, bars, D.BT_MINUTE)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s in range(3):
        orc, otr = oracle_row(strategy, grid, (o[s], h[s], lo[s], c[s]), 98280, CAP)
        for p in range(grid.n_params):
            where = f"{strategy} sym {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


def test_topk_exact_order():
    grid = D.Grid.sma([4, 6, 10], [50, 60, 120], annualization=252)
    S, bars, k = 40, 800, 25
    with D.Engine(grid, topk=k) as e:
        e.load_synthetic(3, 100, S, bars, D.BT_DAILY)
        e.run()
        top = e.read_topk()
        allr = e.summaries()
    recs = [(-float(allr[s, p]["sharpe"]), 100 + s, p) for s in range(S) for p in range(grid.n_params)]
    recs.sort()
    exp = [(r[1], r[2]) for r in recs[:k]]
    assert [(int(t["sym"]), int(t["param"])) for t in top] == exp
    assert all(float(top[i]["sharpe"]) >= float(top[i + 1]["sharpe"]) for i in range(k - 1))


def test_run_batch_csv_jobs():
    import oracle_np as N
    grid = D.Grid.sma([4, 10], [50, 120], annualization=252)
    jobs, series = [], []
    for s, bars in [(0, 300), (1, 451), (2, 64)]:
        o, h, lo, c, v = N.gen(0x5EED, [s], bars, 0)
        jobs.append((f"job-{s}", N.csv_bytes(o[0], h[0], lo[0], c[0], v[0], 0)))
        series.append(c[0].astype(np.int32))
    jobs.insert(1, ("bad", b"2010-01-04,1,2,1\n"))
    with D.Engine(grid) as e:
        res = e.run_batch(jobs)
    assert res[1][0] < 0 and '"error"' in res[1][1]
    good = [r for i, r in enumerate(res) if i != 1]
    for (status, data), cl in zip(good, series):
        assert status == 0
        lines = data.strip().split("\n")
        assert len(lines) == grid.n_params
        orc, _ = oracle_row("sma", grid, (cl, cl, cl, cl), 252)
        import json
        for p, line in enumerate(lines):
            j = json.loads(line)
            assert j["param"] == p and j["n"] == int(orc[p]["n_trades"])
            assert j["pnl"] == int(orc[p]["pnl"]) and j["mdd"] == int(orc[p]["mdd"])
            assert float(j["sharpe"]) == float(orc[p]["sharpe"])
            assert int(j["h"], 16) == int(orc[p]["hash"])


def test_config2_full_shape_parity():
    """BASELINE config 2 at full size on the GPU; every symbol and parameter (2M lanes) checked
    against the multithreaded C oracle, plus the exact top-100 order over all of them."""
    grid = D.config2_grid()
    S, bars = 5000, 2520
    with D.Engine(grid, topk=100) as e:
        e.load_synthetic(0x5EED, 0, S, bars, D.BT_DAILY)
        e.run()
        allr = e.summaries()
        st = e.stats()
        top = e.read_topk()
    assert st["bar_evals"] == S * bars * grid.n_params
    assert st["trades"] == int(allr["n_trades"].sum())
    closes = np.stack([F.gen(0x5EED, s, bars, 0)[3] for s in range(S)])
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    orc = F.sma_grid_mt(closes, np.arange(4, 43, 2), np.arange(50, 241, 10), 252, threads)
    compare_summaries(allr, orc, lambda i: f"config2 sym {i[0]} param {i[1]}")
    flat = allr.reshape(-1)
    order = np.lexsort((np.tile(np.arange(grid.n_params), S), np.repeat(np.arange(S), grid.n_params),
                        -flat["sharpe"]))
    exp = [(int(i // grid.n_params), int(i % grid.n_params)) for i in order[:100]]
    assert [(int(t["sym"]), int(t["param"])) for t in top] == exp


def _expected_topk(allr, sym_ids, k):
    P = allr.shape[1]
    flat = allr.reshape(-1)
    ids = np.repeat(np.asarray(sym_ids, np.int64), P)
    order = np.lexsort((np.tile(np.arange(P), len(sym_ids)), ids, -flat["sharpe"]))
    return [(int(ids[i]), int(i % P)) for i in order[:k]]


def test_topk_massive_ties_device_finish():
    """More records tie on the selected key prefix than the finish block's sort holds: every
    Sharpe is 0 on flat prices, so the order is (sym asc, param asc). The device completes the
    selection itself (k_topk.hip topk_finish_ties): the synchronous read, the pipelined fetch and
    the C-ABI RCCL exchange (world 1) all return the same 50 records."""
    grid = D.Grid.sma([2, 3, 4], [5, 6, 7], annualization=252)
    closes = [np.full(200, 1_000_000, np.int32) for _ in range(300)]   # 2,700 records
    exp = [(1000 + i // 9, i % 9) for i in range(50)]
    comm = E.Comm(E.Comm.unique_id(), 0, 1, 0, 50)
    try:
        with D.Engine(grid, topk=50) as e:
            e.load_ohlc(closes, sym_ids=np.arange(1000, 1300))
            e.run()
            top = e.read_topk()
            e.topk_fetch_async(0)
            fetched, trades = e.topk_fetch_wait(0)
            comm.exchange_async(e, 1)
            gathered, cnt = comm.exchange_wait(1)
    finally:
        comm.close()
    for recs in (top, fetched, gathered):
        assert [(int(t["sym"]), int(t["param"])) for t in recs] == exp
        assert all(float(t["sharpe"]) == 0.0 for t in recs)
    assert trades == 0 and cnt == [300 * 200 * 9, 0]


@pytest.mark.parametrize("k", [1, 50, 1024])
def test_topk_ties_mixed_with_winners(k):
    """Tie-heavy grid with real winners and losers around the tied value, symbol ids not in
    index order: records above the tied Sharpe come first, then the ties by (sym id, param);
    up to the largest k the engine accepts."""
    grid = D.Grid.sma([2, 3, 4, 5], [8, 9, 11], annualization=252)
    rng = np.random.default_rng(7)
    closes = []
    for s in range(900):
        if s % 30 == 0:  # a trending or noisy series: non-zero Sharpes on both sides of 0
            c = np.clip(1_000_000 + np.cumsum(rng.integers(-4000, 4400, 400)), 10_000, 2**31 - 1)
            closes.append(c.astype(np.int32))
        else:
            closes.append(np.full(400, 2_000_000, np.int32))
    ids = rng.permutation(np.arange(5000, 5900))
    with D.Engine(grid, topk=k) as e:
        e.load_ohlc(closes, sym_ids=ids)
        e.run()
        allr = e.summaries().copy()
        top = e.read_topk()
    assert (allr["sharpe"] == 0).sum() > 2048  # the tie path really runs
    assert [(int(t["sym"]), int(t["param"])) for t in top] == _expected_topk(allr, ids, k)


TILE_GRIDS = {
    "ema_ols": lambda: D.Grid.ema_ols([2, 3, 10, 100], [2, 4, 70, 200], band_bps=20),
    "boll": lambda: D.Grid.boll([2, 3, 20, 70, 130], [1, 4], [50, 100], [50, 400], k_den=2),
}


@pytest.mark.parametrize("bars", [1, 2, 63, 64, 65, 130, 1000])
@pytest.mark.parametrize("strategy", ["ema_ols", "boll"])
def test_tile_strategies_ragged(strategy, bars):
    """Tile kernels on every tile-boundary case, windows shorter and longer than a tile."""
    grid = TILE_GRIDS[strategy]()
    o, h, lo, c = _gen(0x5EED, [5, 6], bars, 1)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(0x5EED, 5, 2, bars, D.BT_MINUTE)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s in range(2):
        orc, otr = oracle_row(strategy, grid, (o[s], h[s], lo[s], c[s]), 98280, CAP)
        for p in range(grid.n_params):
            where = f"{strategy} bars {bars} sym {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


@pytest.mark.parametrize("strategy", ["ema_ols", "boll"])
def test_tile_strategies_edges(strategy, golden_dir):
    """Golden edge series (flat, near 2^31 ticks, saw-tooth, 1-2 tick moves, 1-2 bars) with
    their own highs and lows, loaded as ragged rows in one batch."""
    import json, os
    edge = json.load(open(os.path.join(golden_dir, "edge.json")))
    cols = [[np.array(x[k], np.int32) for x in edge] for k in ("c", "h", "l")]
    grid = TILE_GRIDS[strategy]()
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_ohlc(cols[0], cols[1], cols[2])
        e.run()
        got, tr = e.summaries(), e.trades()
    for s, x in enumerate(edge):
        orc, otr = oracle_row(strategy, grid, (cols[0][s], cols[1][s], cols[2][s], cols[0][s]), 98280, CAP)
        for p in range(grid.n_params):
            where = f"{strategy} {x['name']} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


@pytest.mark.parametrize("config", [3, 4])
def test_config34_grids_long_series(config):
    """BASELINE config 3 / 4 grids (all 64 / 256 params) on 1-min series of 20,000 bars."""
    grid = D.config3_grid() if config == 3 else D.config4_grid()
    strategy = "ema_ols" if config == 3 else "boll"
    bars, syms = 20000, [0, 1]
    o, h, lo, c = _gen(0x5EED, syms, bars, 1)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(0x5EED, 0, len(syms), bars, D.BT_MINUTE)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s in range(len(syms)):
        orc, otr = oracle_row(strategy, grid, (o[s], h[s], lo[s], c[s]), 98280, CAP)
        for p in range(grid.n_params):
            where = f"config {config} sym {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


@pytest.mark.parametrize("nf,ns", [(32, 32), (20, 30), (44, 25), (7, 3)])
def test_sma_block_shapes(nf, ns):
    """Every SMA launch shape: 16 waves with the scan folded into a parameter wave (P = 1024,
    the config-5 grid), a 10-wave block plus helper (600), two equal y-blocks (1100) and a
    partial single wave (21); long windows (config 5's slow axis reaches 6,400 bars)."""
    fast = np.arange(1, nf + 1) * 5
    slow = np.arange(1, ns + 1) * 200
    grid = D.Grid.sma(fast, slow, annualization=98280)
    S, bars = 3, 15000
    with D.Engine(grid) as e:
        e.load_synthetic(0x5EED, 40, S, bars, D.BT_MINUTE)
        e.run()
        got = e.summaries()
    closes = np.stack([F.gen(0x5EED, 40 + s, bars, 1)[3] for s in range(S)])
    orc = F.sma_grid_mt(closes, fast, slow, 98280, 8)
    for s in range(S):
        for p in range(grid.n_params):
            compare_summary(got[s, p], orc[s, p], f"shape {nf}x{ns} sym {s} param {p}")


def test_sma_large_block_trades_parity():
    """Blocks of more than 8 waves take the one-round-trip reversal loop (k_sma.hip ONE_TRIP):
    its trade lists in parity mode, a 16-wave grid (P = 1,024) and a 10-wave one (P = 600)."""
    for nf, ns in ((32, 32), (20, 30)):
        grid = D.Grid.sma(np.arange(1, nf + 1) * 2, np.arange(1, ns + 1) * 7 + 3,
                          annualization=252)
        syms, bars = [11, 12], 900
        o, h, lo, c = _gen(0x5EED, syms, bars, 0)
        with D.Engine(grid, parity=True, trade_cap=CAP) as e:
            e.load_synthetic(0x5EED, syms[0], len(syms), bars, D.BT_DAILY)
            e.run()
            got, tr = e.summaries(), e.trades()
        for i in range(len(syms)):
            orc, otr = oracle_row("sma", grid, (o[i], h[i], lo[i], c[i]), 252, CAP)
            for p in range(grid.n_params):
                where = f"{nf}x{ns} sym {syms[i]} param {grid.param(p)}"
                compare_summary(got[i, p], orc[p], where)
                compare_trades(tr[i, p], otr[p], int(orc[p]["n_trades"]), where)


@pytest.mark.parametrize("strategy", ["sma", "ema_ols", "boll"])
def test_spec_maximum_windows(strategy):
    """Windows up to the spec's 4,096 bars (docs/oracle_spec.md §3: w <= 4096 keeps window
    sums < 2^43), beside short ones, on 12,000-bar series: prefix rings of ~4.3k entries."""
    if strategy == "sma":
        grid = D.Grid.sma([3, 500], [4096, 700], annualization=98280)
    elif strategy == "ema_ols":
        grid = D.Grid.ema_ols([5, 4000], [4096, 16], band_bps=20)
    else:
        grid = D.Grid.boll([4096, 12], [2, 5], [50], [100, 400], k_den=2)
    bars = 12000
    o, h, lo, c = _gen(0x5EED, [8, 9], bars, 1)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(0x5EED, 8, 2, bars, D.BT_MINUTE)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s in range(2):
        orc, otr = oracle_row(strategy, grid, (o[s], h[s], lo[s], c[s]), 98280, CAP)
        for p in range(grid.n_params):
            where = f"{strategy} max windows sym {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


@pytest.mark.parametrize("ols", [[1560, 15], [1700, 30]])
def test_ema_stage_shapes(ols):
    """EMA+OLS launches run 128-bar stages when they keep as many blocks per CU as 64-bar ones
    (k_tile.hip ema_stage_tiles) and 64-bar stages otherwise. With two spans, a 1,560-bar OLS
    window gives 54.3 KB at 64-bar stages (three blocks per CU) and 66.6 KB at 128-bar (two):
    64-bar stages; a 1,700-bar window 56.3 / 68.6 KB (two either way): 128-bar stages
    (tests/helpers.py ema_stage_tiles, pinned in test_tile_edge_trades.py). Both shapes, with
    windows that reach back across stages and a ragged last stage, against the oracle."""
    grid = D.Grid.ema_ols([10, 780], ols, band_bps=20)
    bars = 5000 + 64 * 3 + 17
    o, h, lo, c = _gen(0x5EED, [4, 5], bars, 1)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(0x5EED, 4, 2, bars, D.BT_MINUTE)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s in range(2):
        orc, otr = oracle_row("ema_ols", grid, (o[s], h[s], lo[s], c[s]), 98280, CAP)
        for p in range(grid.n_params):
            where = f"ema stages ols {ols} sym {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


def test_pipelined_topk_fetch():
    """bench.py's pipelining: runs i+1 .. i+depth are enqueued before run i's top-k is read;
    each slot must hold its own run's records and trade count (same as the synchronous read of
    that run), with every slot in flight at once (runs i and i+2 share a summary buffer, which
    the engine orders behind run i's read-back). Reloading the data between the runs must not
    race the previous run's top-k chain, which reads the symbol descriptors on the second
    stream (round 2: a reload overwrote them first and slot 0 reported symbol 305 for 5);
    repeated, since a race shows only sometimes."""
    grid = D.Grid.sma([4, 6, 10], [50, 60, 120], annualization=252)
    firsts = [300 * i for i in range(D.PIPE_SLOTS)]
    with D.Engine(grid, topk=20) as e:
        refs = []
        for first in firsts:
            e.load_synthetic(9, first, 40, 700, D.BT_DAILY)
            e.run()
            refs.append((e.read_topk(), e.stats()["trades"]))
        for _ in range(4):
            for slot, first in enumerate(firsts):
                e.load_synthetic(9, first, 40, 700, D.BT_DAILY)  # drains the earlier top-k chains
                e.run()
                e.topk_fetch_async(slot)
            for slot, (top, trades) in enumerate(refs):
                got, n = e.topk_fetch_wait(slot)
                assert got.tolist() == top.tolist() and n == trades
        # the same data, no reload: PIPE_SLOTS runs back to back, as bench.py issues them
        e.load_synthetic(9, 0, 40, 700, D.BT_DAILY)
        for slot in range(D.PIPE_SLOTS):
            e.run()
            e.topk_fetch_async(slot)
        for slot in range(D.PIPE_SLOTS):
            got, n = e.topk_fetch_wait(slot)
            assert got.tolist() == refs[0][0].tolist() and n == refs[0][1]


@pytest.mark.parametrize("hi_prices", [False, True])
def test_sma_large_window_products(hi_prices):
    """SMA grids whose window products f*s pass 2^53 (600 x 4096, 4096 x 4000): equal floor keys
    are settled with F*s vs L*f in int64 (k_sma.hip), so every grid the LDS ring holds is exact.
    hi_prices: prices just below 2^31 with 0-3 tick noise, where keys tie on most bars and the
    products (~2^55) are beyond fp64's exact range."""
    grid = D.Grid.sma([600, 4096, 37], [4096, 4000, 5000], annualization=98280)
    bars = 9000
    if hi_prices:
        rng = np.random.default_rng(4)
        closes = [(2**31 - 2**20 - 1 - rng.integers(0, 4, bars)).astype(np.int32) for _ in range(2)]
    else:
        closes = [F.gen(0x5EED, s, bars, 1)[3] for s in (3, 4)]
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_ohlc(closes)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s, cl in enumerate(closes):
        orc, otr = oracle_row("sma", grid, (cl, cl, cl, cl), 98280, CAP)
        for p in range(grid.n_params):
            where = f"large windows hi={hi_prices} sym {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


def test_release_library_ignores_ablate_env(monkeypatch):
    """BT_ABLATE in the environment (a profiling switch of dev/prof.so) must not change a
    release-library result: bit-identical summaries with and without it."""
    grid = D.Grid.boll([10, 45], [3, 5], [50], [100, 400], k_den=2)
    res = []
    for env in (None, "15"):
        if env:
            monkeypatch.setenv("BT_ABLATE", env)
        with D.Engine(grid) as e:
            e.load_synthetic(0x5EED, 0, 4, 3000, D.BT_MINUTE)
            e.run()
            res.append(e.summaries().copy())
    assert res[0].tobytes() == res[1].tobytes() and int(res[0]["n_trades"].sum()) > 0


def test_boll_many_k_values():
    """Bollinger grids with more than 8 z thresholds per window (condition words in passes of
    8 k values, k_tile.hip): 12 k values x 3 windows, bit-exact trades vs the oracle."""
    grid = D.Grid.boll([5, 20, 90], list(range(1, 13)), [50], [100], k_den=4)
    bars = 4000
    o, h, lo, c = _gen(0x5EED, [21, 22], bars, 1)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(0x5EED, 21, 2, bars, D.BT_MINUTE)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s in range(2):
        orc, otr = oracle_row("boll", grid, (o[s], h[s], lo[s], c[s]), 98280, CAP)
        for p in range(grid.n_params):
            where = f"boll 12 k sym {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


@pytest.mark.parametrize("sl,tp", [
    ([25, 50, 75, 100, 150], [50, 100, 200, 300, 400, 75]),   # 3 shared: 8 distinct levels
    ([30, 9999, 120], [45, 9999]),                            # 4 distinct (odd pairs), extreme bps
    ([60], [60]),                                             # one level for all four sides
])
def test_boll_sltp_level_sharing(sl, tp):
    """SL/TP level tables built per *distinct* bps (a level 1e4 -+ bps serves every SL and TP of
    that bps) and searched two per level task: grids with shared, odd-count and extreme
    (9,999 bps) distances, bit-exact trades vs the oracle."""
    grid = D.Grid.boll([10, 45], [3, 5], sl, tp, k_den=2)
    bars = 3000
    o, h, lo, c = _gen(0x5EED, [31, 32], bars, 1)
    with D.Engine(grid, parity=True, trade_cap=CAP) as e:
        e.load_synthetic(0x5EED, 31, 2, bars, D.BT_MINUTE)
        e.run()
        got, tr = e.summaries(), e.trades()
    for s in range(2):
        orc, otr = oracle_row("boll", grid, (o[s], h[s], lo[s], c[s]), 98280, CAP)
        for p in range(grid.n_params):
            where = f"boll levels sym {s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            compare_trades(tr[s, p], otr[p], int(orc[p]["n_trades"]), where)


def _zigzag(bars, seed):
    """Closes alternating by ~0.1 % with wide wicks: with k = 0 and zero-bps stops every lane
    trades every other bar (~21 trades per lane and tile)."""
    rng = np.random.default_rng(seed)
    base = 1_000_000 + np.cumsum(rng.integers(-50, 51, bars))
    c = (base + np.where(np.arange(bars) % 2 == 0, 0, 1000)).astype(np.int64)
    h = c + rng.integers(0, 3000, bars)
    lo = c - rng.integers(0, 3000, bars)
    return [x.astype(np.int32) for x in (h, lo, c)]


@pytest.mark.parametrize("segments", [1, 3])
def test_boll_trade_flood(segments):
    """A grid and series that trade every other bar on every lane (~21 trades per lane and tile,
    ~8,000 per block-tile: the finder's record buffer and the walkers' loops near their per-tile
    maximum; split into bar segments too); every field vs the oracle."""
    grid = D.Grid.boll([2, 3, 4, 5, 6, 7, 8, 9], [0, 1, 2, 3], [0, 1], [0, 1, 2, 3], k_den=4)
    series = [_zigzag(3000, 1), _zigzag(2500, 2)]
    with D.Engine(grid, parity=segments == 1, trade_cap=CAP if segments == 1 else 0) as e:
        e.set_segments(segments)
        e.load_ohlc([s[2] for s in series], [s[0] for s in series], [s[1] for s in series])
        e.run()
        got = e.summaries()
        tr = e.trades() if segments == 1 else None
        if segments > 1:
            assert e.last_segments() == segments
    for i, (h, lo, c) in enumerate(series):
        orc, otr = oracle_row("boll", grid, (c, h, lo, c), 98280, CAP if segments == 1 else 0)
        assert int(orc[0]["n_trades"]) > 600, orc[0]
        for p in range(grid.n_params):
            where = f"zigzag {i} {grid.param(p)}"
            compare_summary(got[i, p], orc[p], where)
            if tr is not None:
                compare_trades(tr[i, p], otr[p], min(int(orc[p]["n_trades"]), CAP), where)


def test_run_batch_binary_and_csv_mixed():
    """bt_run_batch on one JobsReply mixing DBXCOL1 payloads (decoded straight into the pinned
    staging rows), CSV text, and malformed payloads of every kind: good jobs bit-exact vs the
    oracle (Bollinger: high/low columns too), bad jobs answered with the same message the
    standalone parser gives, and the batch profile accounts for every job."""
    import json
    import oracle_np as N
    from dbx_amd import payload as PL
    grid = D.Grid.boll([10, 45], [3, 5], [50, 100], [100, 400], k_den=2)
    o, h, lo, c, v = N.gen(0x5EED, [0, 1, 2], 3000, 1)
    good = {0: PL.encode_columns(o[0], h[0], lo[0], c[0], v[0]),
            2: N.csv_bytes(o[1], h[1], lo[1], c[1], v[1], 1),
            4: PL.encode_columns(o[2], h[2], lo[2], c[2])}
    base = PL.encode_columns(o[0][:100], h[0][:100], lo[0][:100], c[0][:100])
    bad = {1: base[:-1],                                                          # length
           3: base[:16 + 4 * 300 + 8] + (0).to_bytes(4, "little") + base[16 + 4 * 300 + 12:],  # price
           5: base[:16 + 4 * 300 + 40] + (2**31 - 1).to_bytes(4, "little") + base[16 + 4 * 300 + 44:]}  # 100%
    jobs = [(f"j{i}", good[i] if i in good else bad[i]) for i in range(6)]
    with D.Engine(grid) as e:
        res = e.run_batch(jobs)
        prof = e.batch_profile()
        st = e.stats()
    assert prof["n_jobs"] == 6 and prof["n_failed"] == 3 and st["errors"] == 3
    assert prof["bars"] == 9000 and prof["payload_bytes"] == sum(len(b) for _, b in jobs)
    # bytes ingest reads: job 0's volume column is skipped; job 1 fails its header check unread;
    # jobs 3 and 5 are read whole before their validation fails
    assert prof["payload_bytes_read"] == (16 + 16 * len(o[0])) + len(good[2]) + len(good[4]) \
        + len(bad[3]) + len(bad[5])
    for i, b in bad.items():
        assert res[i][0] < 0
        with pytest.raises(ValueError) as why:
            E.parse_csv(b)
        assert json.loads(res[i][1])["error"] == str(why.value)
    for i, s in ((0, 0), (2, 1), (4, 2)):
        status, data = res[i]
        assert status == 0
        lines = data.strip().split("\n")
        orc, _ = oracle_row("boll", grid, (o[s], h[s], lo[s], c[s]), 98280)
        for p, line in enumerate(lines):
            j = json.loads(line)
            assert j["n"] == int(orc[p]["n_trades"]) and j["pnl"] == int(orc[p]["pnl"])
            assert j["mdd"] == int(orc[p]["mdd"]) and j["exp"] == int(orc[p]["exposure"])
            assert float(j["sharpe"]) == float(orc[p]["sharpe"]) and int(j["h"], 16) == int(orc[p]["hash"])


def test_rccl_exchange_world1_matches_local_topk():
    """The C-ABI RCCL exchange (bt_comm_*, comm.cpp) at world size 1 on the MI355X: an
    all-gather from the engine's device top-k, pipelined over every slot (BT_PIPE_SLOTS runs in
    flight before the first wait, as bench.py's two-deep N > 1 loop needs three), returns each
    run's top-k and counters exactly."""
    grid = D.Grid.sma([4, 6, 10], [50, 60, 120], annualization=252)
    comm = E.Comm(E.Comm.unique_id(), 0, 1, 0, 20)
    firsts = [300 * i for i in range(D.PIPE_SLOTS)]
    try:
        with D.Engine(grid, topk=20) as e:
            refs = []
            for first in firsts:
                e.load_synthetic(9, first, 40, 700, D.BT_DAILY)
                e.run()
                refs.append((e.read_topk(), e.stats()))
            for slot, first in enumerate(firsts):
                e.load_synthetic(9, first, 40, 700, D.BT_DAILY)
                e.run()
                comm.exchange_async(e, slot)
            for slot, (top, st) in enumerate(refs):
                got, cnt = comm.exchange_wait(slot)
                assert got.tolist() == top.tolist()
                assert cnt == [st["bar_evals"], st["trades"]]
            with pytest.raises(D.BtError, match="bad arguments"):
                comm.exchange_async(e, D.PIPE_SLOTS)
    finally:
        comm.close()


def test_torch_nccl_backend_exchange_world1():
    """parallel.exchange over torch.distributed's "nccl" backend (RCCL) with device tensors, at
    world size 1: the branch bench.py takes on multi-GPU nodes has run on an MI355X."""
    import os
    import torch
    import torch.distributed as dist
    from dbx_amd import parallel as PAR
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        recs = np.zeros(5, D.TOPK_DTYPE)
        recs["sharpe"] = [3.0, 2.0, 2.0, 1.0, 0.5]
        recs["sym"] = [4, 1, 2, 9, 9]
        recs["param"] = [0, 7, 3, 1, 2]
        top, cnt = PAR.exchange(recs, 5, [123, 45], dist)
        assert top.tolist() == recs.tolist() and cnt == [123, 45]
        comm = PAR.make_comm(dist, 0, 5)
        comm.close()
    finally:
        dist.destroy_process_group()


def test_run_batch_empty_all_failed_then_good():
    """An empty JobsReply, then one whose every job is malformed (no kernel launch, every job
    answered with an error), then a good one on the same engine: results stay exact."""
    import json
    import oracle_np as N
    grid = D.Grid.sma([4, 10], [50, 120], annualization=252)
    o, h, lo, c, v = N.gen(0x5EED, [5], 700, 0)
    good = N.csv_bytes(o[0], h[0], lo[0], c[0], v[0], 0)
    with D.Engine(grid) as e:
        assert e.run_batch([]) == []
        bad = e.run_batch([("a", b""), ("b", b"not,a,csv\n"), ("c", b"DBXCOL1\n\x00\x00")])
        assert all(st < 0 and "error" in json.loads(d) for st, d in bad)
        (st, data), = e.run_batch([("g", good)])
    assert st == 0
    orc, _ = oracle_row("sma", grid, (c[0], c[0], c[0], c[0]), 252)
    for p, line in enumerate(data.strip().split("\n")):
        j = json.loads(line)
        assert j["n"] == int(orc[p]["n_trades"]) and j["pnl"] == int(orc[p]["pnl"])
        assert int(j["h"], 16) == int(orc[p]["hash"])
