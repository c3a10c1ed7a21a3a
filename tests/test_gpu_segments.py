"""Bar-axis split of the Bollinger walk (k_tile.hip SEG; include/bt.h bt_set_segments): every
summary field of a split run must equal the unsplit run and the C oracle bit for bit, whatever
the segment count and burn-in — including burn-ins too short for the speculative walk to meet
the true one (the fix pass re-walks those boundaries) and segments with no bars at all."""
import numpy as np
import pytest

import dbx_amd as D
import orc_ffi as F
from helpers import compare_summary, ema_stage_tiles, oracle_row

pytestmark = pytest.mark.gpu


def _run(grid, sym0, n_sym, bars, segments, burn=0):
    with D.Engine(grid) as e:
        e.set_segments(segments, burn)
        e.load_synthetic(0x5EED, sym0, n_sym, bars, D.BT_MINUTE)
        e.run()
        got = e.summaries().copy()
        used, refixed = e.last_segments(with_refixed=True)
        st = e.stats()
    _run.refixed = refixed
    return got, used, st


@pytest.mark.parametrize("segments,burn", [(2, 64), (2, 1), (3, 2), (4, 1), (5, 3)])
def test_split_equals_unsplit_and_oracle(segments, burn):
    grid = D.Grid.boll([10, 45, 240], [3, 5], [50, 100], [100, 400], k_den=2)
    bars = 20000
    ref, used1, st1 = _run(grid, 0, 3, bars, 1)
    got, used, st = _run(grid, 0, 3, bars, segments, burn)
    assert used1 == 1 and used == segments
    if burn <= 2:  # one or two tiles of burn-in rarely reach the true state: the fix pass ran
        assert _run.refixed > 0
    assert got.tobytes() == ref.tobytes(), "split run differs from the unsplit run"
    assert st["trades"] == st1["trades"] == int(ref["n_trades"].sum())
    for s in range(3):
        o, h, lo, c = F.gen(0x5EED, s, bars, 1)[:4]
        orc, _ = oracle_row("boll", grid, (o, h, lo, c), 98280)
        for p in range(grid.n_params):
            compare_summary(got[s, p], orc[p], f"G={segments} burn={burn} sym {s} {grid.param(p)}")


def test_split_config4_grid_short_burn_in():
    """All 256 config-4 parameters, burn-in of one tile: many boundaries need the fix pass."""
    grid = D.config4_grid()
    ref, _, _ = _run(grid, 7, 4, 30000, 1)
    got, used, _ = _run(grid, 7, 4, 30000, 2, 1)
    assert used == 2 and got.tobytes() == ref.tobytes()


def test_split_ragged_and_empty_segments():
    """Ragged series (1 bar to a few tiles) cut into more segments than they have tiles."""
    grid = D.Grid.boll([2, 3, 20, 70], [1, 4], [50, 100], [50, 400], k_den=2)
    lengths = [1, 2, 63, 64, 65, 130, 700, 3000]
    cols = [F.gen(0x5EED, 30 + i, n, 1) for i, n in enumerate(lengths)]
    outs = []
    for segments in (1, 4, 9):
        with D.Engine(grid) as e:
            e.set_segments(segments, 1)
            e.load_ohlc([x[3] for x in cols], [x[1] for x in cols], [x[2] for x in cols])
            e.run()
            outs.append(e.summaries().copy())
            assert e.last_segments() == segments
    assert outs[1].tobytes() == outs[0].tobytes() and outs[2].tobytes() == outs[0].tobytes()
    for i, x in enumerate(cols):
        orc, _ = oracle_row("boll", grid, (x[0], x[1], x[2], x[3]), 98280)
        for p in range(grid.n_params):
            compare_summary(outs[1][i, p], orc[p], f"ragged {lengths[i]} bars {grid.param(p)}")


def test_auto_split_on_small_shard_matches_oracle():
    """Automatic mode on a shard with fewer symbols than CUs (the 8-GPU config-4 shard is 250):
    the engine splits, and sampled symbols match the oracle."""
    grid = D.config4_grid()
    got, used, _ = _run(grid, 100, 120, 40000, 0)
    assert used >= 2
    for s in (0, 77, 119):
        o, h, lo, c = F.gen(0x5EED, 100 + s, 40000, 1)[:4]
        orc, _ = oracle_row("boll", grid, (o, h, lo, c), 98280)
        for p in range(0, grid.n_params, 5):
            compare_summary(got[s, p], orc[p], f"auto split sym {100 + s} {grid.param(p)}")


def test_parity_mode_never_splits():
    grid = D.Grid.boll([10, 45], [3, 5], [50], [100], k_den=2)
    with D.Engine(grid, parity=True, trade_cap=4096) as e:
        e.set_segments(4, 1)
        e.load_synthetic(0x5EED, 0, 2, 5000, D.BT_MINUTE)
        e.run()
        assert e.last_segments() == 1


def _run_grid(grid, cols, segments, burn=0):
    with D.Engine(grid) as e:
        e.set_segments(segments, burn)
        e.load_ohlc([x[3] for x in cols], [x[1] for x in cols], [x[2] for x in cols])
        e.run()
        got = e.summaries().copy()
        used, refixed = e.last_segments(with_refixed=True)
    return got, used, refixed


@pytest.mark.parametrize("segments,burn", [(2, 0), (3, 0), (2, 1), (4, 2)])
@pytest.mark.parametrize("long_window,stage", [(780, 1), (1560, 2)])
def test_ema_split_equals_unsplit_and_oracle(segments, burn, long_window, stage):
    """EMA+OLS segments must also agree on the fp64 EMA chains at every boundary: with the
    default burn-in (6 x the longest span, the chains starting from the weighted-sum estimate)
    the speculative chains meet the true ones; with a 1-2 tile burn-in the lanes' trade states
    (and the longest span's chain) mostly do not, and the fix pass re-walks from the true values.
    The 1,560-bar OLS window puts the split kernel in 128-bar stages (config 3's 250-symbol
    shard runs so), the 780-bar one in 64-bar stages (tests/helpers.py ema_stage_tiles)."""
    grid = D.Grid.ema_ols([10, 60, 390], [15, 120, long_window], band_bps=20)
    assert ema_stage_tiles(*grid.axes[:2])[0] == stage
    cols = [F.gen(0x5EED, 60 + i, 40000, 1) for i in range(3)]
    ref, used1, _ = _run_grid(grid, cols, 1)
    got, used, refixed = _run_grid(grid, cols, segments, burn)
    assert used1 == 1 and used == segments
    if burn and burn <= 2:
        assert refixed > 0
    assert got.tobytes() == ref.tobytes(), "split run differs from the unsplit run"
    for i, x in enumerate(cols):
        orc, _ = oracle_row("ema_ols", grid, (x[0], x[1], x[2], x[3]), 98280)
        for p in range(grid.n_params):
            compare_summary(got[i, p], orc[p], f"ema G={segments} burn={burn} sym {i} {grid.param(p)}")


@pytest.mark.parametrize("long_window,stage", [(200, 1), (1700, 2)])
def test_ema_split_ragged_and_empty_segments(long_window, stage):
    grid = D.Grid.ema_ols([2, 3, 10, 100], [2, 4, 70, long_window], band_bps=20)
    assert ema_stage_tiles(*grid.axes[:2])[0] == stage
    lengths = [1, 2, 63, 64, 65, 130, 700, 5000]
    cols = [F.gen(0x5EED, 80 + i, n, 1) for i, n in enumerate(lengths)]
    ref, _, _ = _run_grid(grid, cols, 1)
    for segments, burn in ((4, 1), (9, 1), (3, 0)):
        got, used, _ = _run_grid(grid, cols, segments, burn)
        assert used == segments and got.tobytes() == ref.tobytes(), (segments, burn)
    for i, x in enumerate(cols):
        orc, _ = oracle_row("ema_ols", grid, (x[0], x[1], x[2], x[3]), 98280)
        for p in range(grid.n_params):
            compare_summary(ref[i, p], orc[p], f"ema ragged {lengths[i]} bars {grid.param(p)}")


@pytest.mark.parametrize("segments,burn", [(3, 1), (2, 2)])
def test_ema_split_many_param_blocks(segments, burn):
    """EMA+OLS grid of more than 896 params (64 lanes x 14 parameter waves), so each symbol's
    parameters span several blockIdx.y blocks that share the per-(segment, symbol) chain record:
    with a burn-in too short for the chains to meet, the fix pass must re-walk every y-block of
    a boundary (a fix pass that rewrote the shared start record would let later y-blocks keep
    results built on the wrong chain). The 3,000-bar span keeps its chain from meeting the true
    one within the short burn-in even from the weighted-sum start estimate."""
    spans = list(range(3, 3 + 2 * 29, 2)) + [3000]  # 30 spans
    wins = list(range(4, 4 + 5 * 32, 5))           # 32 OLS windows -> 960 params
    grid = D.Grid.ema_ols(spans, wins, band_bps=15)
    assert grid.n_params > 896
    cols = [F.gen(0x5EED, 400 + i, 12000 + 3000 * i, 1) for i in range(3)]
    ref, used1, _ = _run_grid(grid, cols, 1)
    got, used, refixed = _run_grid(grid, cols, segments, burn)
    assert used1 == 1 and used == segments and refixed > 0
    assert got.tobytes() == ref.tobytes(), "split run differs from the unsplit run"
    for i, x in enumerate(cols):
        orc, _ = oracle_row("ema_ols", grid, (x[0], x[1], x[2], x[3]), 98280)
        for p in range(0, grid.n_params, 7):
            compare_summary(got[i, p], orc[p], f"ema y-blocks G={segments} sym {i} {grid.param(p)}")


def test_ema_auto_split_config3_grid_small_shard():
    """Config-3 grid on a small shard (automatic split) against the oracle on sampled symbols."""
    grid = D.config3_grid()
    with D.Engine(grid) as e:
        e.load_synthetic(0x5EED, 200, 100, 98280, D.BT_MINUTE)
        e.run()
        got = e.summaries().copy()
        used, refixed = e.last_segments(with_refixed=True)
    assert used >= 2
    print(f"config-3 grid, 100 symbols: {used} segments, {refixed} boundary blocks re-walked")
    for s in (0, 63, 99):
        o, h, lo, c = F.gen(0x5EED, 200 + s, 98280, 1)[:4]
        orc, _ = oracle_row("ema_ols", grid, (o, h, lo, c), 98280)
        for p in range(0, grid.n_params, 3):
            compare_summary(got[s, p], orc[p], f"ema auto split sym {200 + s} {grid.param(p)}")


SMA_SEG_GRID = lambda: D.Grid.sma([5, 20, 60, 150], [200, 900, 3000], annualization=98280)


@pytest.mark.parametrize("segments,burn", [(2, 2), (3, 1), (4, 1), (6, 3)])
def test_sma_split_equals_unsplit_and_oracle(segments, burn):
    """SMA bar segments (k_sma.hip SEG): positions are held for thousands of bars, so the trade
    open at a boundary is carried symbolically and closed by the combine pass. Every summary
    field equals the unsplit kernel and the oracle bit for bit."""
    grid = SMA_SEG_GRID()
    cols = [F.gen(0x5EED, 500 + i, 30000 + 7000 * i, 1) for i in range(3)]
    ref, used1, _ = _run_grid(grid, cols, 1)
    got, used, _ = _run_grid(grid, cols, segments, burn)
    assert used1 == 1 and used == segments
    assert got.tobytes() == ref.tobytes(), "split run differs from the unsplit run"
    for i, x in enumerate(cols):
        orc, _ = oracle_row("sma", grid, (x[0], x[1], x[2], x[3]), 98280)
        for p in range(grid.n_params):
            compare_summary(got[i, p], orc[p], f"sma G={segments} burn={burn} sym {i} {grid.param(p)}")


def test_sma_split_ragged_and_empty_segments():
    grid = D.Grid.sma([2, 3, 10], [4, 70, 200], annualization=98280)
    lengths = [1, 2, 63, 64, 65, 130, 700, 5000]
    cols = [F.gen(0x5EED, 90 + i, n, 1) for i, n in enumerate(lengths)]
    ref, _, _ = _run_grid(grid, cols, 1)
    for segments, burn in ((4, 1), (9, 1), (3, 2)):
        got, used, _ = _run_grid(grid, cols, segments, burn)
        assert used == segments and got.tobytes() == ref.tobytes(), (segments, burn)
    for i, x in enumerate(cols):
        orc, _ = oracle_row("sma", grid, (x[0], x[1], x[2], x[3]), 98280)
        for p in range(grid.n_params):
            compare_summary(ref[i, p], orc[p], f"sma ragged {lengths[i]} bars {grid.param(p)}")


def test_sma_split_tied_burn_in_takes_the_fix_pass():
    """Flat prices across the boundaries: every comparison of the burn-in ties, so a speculative
    segment starts flat while the true position (set before the flat stretch) is held; the fix
    pass re-walks those segments from the true position."""
    grid = D.Grid.sma([3, 8, 20], [40, 90], annualization=98280)
    rng = np.random.default_rng(11)
    walk = lambda n, c0: np.clip(c0 + np.cumsum(rng.integers(-3000, 3001, n)), 10_000, 2**31 - 1)
    a = walk(5000, 1_000_000)
    c = np.concatenate([a, np.full(10000, a[-1]), walk(5000, a[-1])]).astype(np.int32)
    # a second symbol without flat stretches: its boundaries agree while the first symbol's
    # re-walk, so the fix pass must leave the agreeing symbol's segments as they are
    c2 = walk(20000, 2_000_000).astype(np.int32)
    cols = [(c, c, c, c), (c2, c2, c2, c2)]
    ref, _, _ = _run_grid(grid, cols, 1)
    got, used, refixed = _run_grid(grid, cols, 3, 1)   # boundaries at bars 6,720 and 13,376
    assert used == 3 and refixed > 0
    assert got.tobytes() == ref.tobytes()
    for i, x in enumerate((c, c2)):
        orc, _ = oracle_row("sma", grid, (x, x, x, x), 98280)
        for p in range(grid.n_params):
            compare_summary(got[i, p], orc[p], f"sma flat boundary sym {i} {grid.param(p)}")


def test_sma_auto_segments_only_for_few_long_blocks():
    """Automatic mode splits the config-5 shape (16-wave blocks, a shard filling the GPU a few
    times) and leaves config 2 (several 8-wave blocks per CU) alone."""
    with D.Engine(D.config2_grid()) as e:
        e.load_synthetic(0x5EED, 0, 600, 2520, D.BT_DAILY)
        e.run()
        assert e.last_segments() == 1
    with D.Engine(D.config5_grid()) as e:
        e.load_synthetic(0x5EED, 0, 300, 60000, D.BT_MINUTE)
        e.run()
        assert e.last_segments() > 1
        got = e.summaries().copy()
    closes = np.stack([F.gen(0x5EED, s, 60000, 1)[3] for s in (0, 299)])
    grid = D.config5_grid()
    orc = F.sma_grid_mt(closes, np.asarray(grid.axes[0]), np.asarray(grid.axes[1]), 98280, 8)
    for i, s in enumerate((0, 299)):
        for p in range(grid.n_params):
            compare_summary(got[s, p], orc[i, p], f"config-5 grid auto split sym {s} param {p}")


_NS = int(__import__("os").environ.get("BT_RANDOM_SEEDS", "0"))


@pytest.mark.parametrize("strategy,seed", [(st, s) for st in ("boll", "ema_ols", "sma") for s in range(_NS or 3)])
def test_random_splits_equal_unsplit(strategy, seed):
    """Random grids, segment counts (2-6), burn-ins (1-6 tiles) and ragged random-walk series
    (SMA's symbolic carried trades included):
    the split run equals the unsplit one bit for bit (the unsplit kernels are oracle-checked by
    the parity sweeps), whether or not the fix pass re-walks boundaries."""
    rng = np.random.default_rng(4000 + seed + (500 if strategy == "ema_ols" else 0))
    pick = lambda lo, hi, k: sorted(int(x) for x in rng.choice(np.arange(lo, hi), k, replace=False))
    if strategy == "boll":
        grid = D.Grid.boll(pick(2, 121, 8), pick(1, 9, 4), pick(10, 300, 2), pick(10, 500, 4), k_den=2)
    elif strategy == "sma":
        grid = D.Grid.sma(pick(2, 60, 4), pick(20, 2000, 4), annualization=98280)
    else:
        grid = D.Grid.ema_ols(pick(2, 200, 4), pick(2, 400, 4), band_bps=int(rng.integers(0, 60)))
    n = int(rng.integers(2, 6))
    closes, highs, lows = [], [], []
    for i in range(n):
        bars = int(rng.integers(1, 16000))
        c = np.clip(1_000_000 + np.cumsum(rng.integers(-3000, 3001, bars)), 10_000, 2**31 - 1)
        closes.append(c.astype(np.int32))
        highs.append(np.clip(c + rng.integers(0, 2000, bars), 1, 2**31 - 1).astype(np.int32))
        lows.append(np.clip(c - rng.integers(0, 2000, bars), 1, 2**31 - 1).astype(np.int32))
    G, burn = int(rng.integers(2, 7)), int(rng.integers(1, 7))
    outs = []
    for segments, b in ((1, 0), (G, burn)):
        with D.Engine(grid) as e:
            e.set_segments(segments, b)
            e.load_ohlc(closes, highs, lows)
            e.run()
            outs.append(e.summaries().copy())
            assert e.last_segments() == segments
    assert outs[1].tobytes() == outs[0].tobytes(), f"{strategy} G={G} burn={burn}"
