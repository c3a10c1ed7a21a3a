"""Shared test helpers: oracle-vs-engine comparison (tests only)."""
import numpy as np

import orc_ffi as F


def oracle_row(strategy, grid, ohlc, ann, cap=0):
    """Run the C oracle for every param of `grid` on one symbol; returns (summaries, trades)."""
    o, h, lo, c = ohlc
    out, trades = [], []
    for p in range(grid.n_params):
        kw = grid.param(p)
        if strategy == "sma":
            s, tr = F.sma(c, kw["f"], kw["s"], ann, cap)
        elif strategy == "ema_ols":
            s, tr = F.ema_ols(c, kw["n"], kw["w"], kw["band_bps"], ann, cap)
        else:
            s, tr = F.boll(h, lo, c, kw["w"], kw["k_num"], kw["k_den"], kw["sl"], kw["tp"], ann, cap)
        out.append(s)
        trades.append(tr)
    return out, trades


FIELDS = ("n_trades", "pnl", "mdd", "exposure", "hash")


def compare_summary(gpu, orc, where=""):
    """Bit-exact comparison of one engine summary vs one oracle summary."""
    for f in FIELDS:
        assert int(gpu[f]) == int(orc[f]), f"{where}: {f} gpu={gpu[f]} oracle={orc[f]}"
    # Sharpe: bit-exact by construction (exact int128 sums, fixed op sequence); the north_star
    # tolerance (1e-9 relative) is asserted as well so a failure message shows the size.
    g, o = float(gpu["sharpe"]), float(orc["sharpe"])
    assert abs(g - o) <= 1e-9 * max(abs(o), 1e-300), f"{where}: sharpe {g!r} vs {o!r}"
    assert g == o, f"{where}: sharpe not bit-exact {g!r} vs {o!r}"


def compare_summaries(gpu, orc, where):
    """Bit-exact comparison of two equal-shape summary arrays (every field, Sharpe by bits);
    the first mismatch is reported through compare_summary with where(index)."""
    assert gpu.shape == orc.shape, f"shapes {gpu.shape} vs {orc.shape}"
    bad = np.zeros(gpu.shape, dtype=bool)
    for f in FIELDS:
        bad |= gpu[f].astype(np.int64) != orc[f].astype(np.int64)
    bad |= gpu["sharpe"].astype(np.float64).view(np.uint64) != orc["sharpe"].astype(np.float64).view(np.uint64)
    if bad.any():
        i = tuple(int(x) for x in np.argwhere(bad)[0])
        compare_summary(gpu[i], orc[i], where(i))
        raise AssertionError(f"{where(i)}: summaries differ")


def compare_trades(gpu_tr, orc_tr, n, where=""):
    got = [tuple(int(x) for x in (t["entry_bar"], t["exit_bar"], t["side"], t["entry_px"], t["exit_px"]))
           for t in gpu_tr[:n]]
    exp = [tuple(int(x) for x in (t["entry_bar"], t["exit_bar"], t["side"], t["entry_px"], t["exit_px"]))
           for t in orc_tr[:n]]
    assert got == exp, f"{where}: trade lists differ (first diff at {next((i for i,(a,b) in enumerate(zip(got,exp)) if a!=b), None)})"


def ema_stage_tiles(spans, windows):
    """Model of k_tile.hip ema_stage_tiles / tile_lds_layout(kind 0): the EMA+OLS block's LDS bytes
    at 64-bar (TS 1) and 128-bar (TS 2) stages and the stage the launcher picks (TS 2 when it keeps
    as many blocks per CU). Used only to choose test grids that reach each shape; pinned to the
    kernel's own figures for config 3 (61,120 / 80,208 B) in test_tile_edge_trades.py."""
    T, cu = 64, 160 * 1024
    ring = (max(windows) + 5 * T - 1) // T * T
    na, nb = len(spans), len(windows)

    def lds(ts):
        ns, nd, sl = 3 * ts, 3 if ts == 1 else 2 * ts, 2 * ts
        parts = [ring * 8, ring * 8, ns * T * 4, ns * 2 * T * 8, nd * 6 * T * 16,
                 sl * na * (T + 1) * 8, sl * (4 * na + 2 * nb) * 8, nb * 4, ns * 4, 4]
        return sum((p + 15) & ~15 for p in parts)

    l1, l2 = lds(1), lds(2)
    return (2 if l2 <= cu and cu // l2 >= cu // l1 else 1), l1, l2
