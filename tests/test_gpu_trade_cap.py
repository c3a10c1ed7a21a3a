"""Parity-mode trade lists shorter than the trade count (bt_config.trade_cap, include/bt.h): each
(symbol, parameter) keeps its first trade_cap trades and the rest are dropped, never written
past its slot range, and the summaries (every field, the trade hash included) still cover every
trade. Caps of 1-3 against walks of hundreds of trades, all three strategies, compared with the
C oracle's full lists; the Bollinger lists come from the split walk's accountant wave."""
import numpy as np
import pytest

import dbx_amd as D
import orc_ffi as F
from helpers import compare_summary, compare_trades, oracle_row

pytestmark = pytest.mark.gpu

GRIDS = {
    "sma": lambda: D.Grid.sma([3, 5, 9, 14], [20, 31, 50], annualization=98280),
    "ema_ols": lambda: D.Grid.ema_ols([5, 20, 60], [10, 40, 150], band_bps=10, annualization=98280),
    "boll": lambda: D.Grid.boll([10, 30, 90], [2, 4, 6], [50], [50, 200], k_den=2, annualization=98280),
}


@pytest.mark.parametrize("strategy", list(GRIDS))
@pytest.mark.parametrize("cap", [1, 3])
def test_trade_lists_truncate_at_cap(strategy, cap):
    grid = GRIDS[strategy]()
    n_sym, bars = 3, 6000
    with D.Engine(grid, parity=True, trade_cap=cap) as e:
        e.load_synthetic(0x5EED, 40, n_sym, bars, D.BT_MINUTE)
        e.run()
        got = e.summaries().copy()
        trades = e.trades().copy()
        total = e.stats()["trades"]
    assert trades.shape == (n_sym, grid.n_params, cap)
    assert total == int(got["n_trades"].sum())
    many = 0
    for s in range(n_sym):
        o, h, lo, c = F.gen(0x5EED, 40 + s, bars, 1)[:4]
        orc, orc_tr = oracle_row(strategy, grid, (o, h, lo, c), 98280, cap=4096)
        for p in range(grid.n_params):
            where = f"{strategy} cap={cap} sym {40 + s} {grid.param(p)}"
            compare_summary(got[s, p], orc[p], where)
            n = int(orc[p]["n_trades"])
            many += n > cap
            compare_trades(trades[s, p], orc_tr[p], min(n, cap), where)
    assert many >= grid.n_params, "too few lanes overflow the cap to test truncation"
