"""Pin the C oracle (oracle/oracle.c) to the committed golden vectors (tests/golden/), which
oracle/make_golden.py produced from the independent numpy restatement (oracle/oracle_np.py).

The reference has no fixtures for this path (its job function sleeps), so
these vectors pin docs/oracle_spec.md, not reference outputs ("parity unpinned" vs the
reference; see oracle/oracle.h)."""
import json
import os

import numpy as np
import pytest

import orc_ffi as F


def _load(golden_dir, name):
    return json.load(open(os.path.join(golden_dir, name)))


def test_generator_known_answers(golden_dir):
    g = _load(golden_dir, "gen.json")
    for k in g["known"]:
        o, h, lo, c, v = F.gen(int(k["seed"], 16), k["sym"], k["bars"], k["freq"])
        for name, arr in (("o", o), ("h", h), ("l", lo), ("c", c), ("v", v)):
            assert arr.tolist() == k[name], (k["sym"], name)
    for k in g["checksums"]:
        o, h, lo, c, v = F.gen(int(k["seed"], 16), k["sym"], k["bars"], k["freq"])
        assert int(o.astype(np.int64).sum()) == k["sum_o"]
        assert int(h.astype(np.int64).sum()) == k["sum_h"]
        assert int(lo.astype(np.int64).sum()) == k["sum_l"]
        assert int(c.astype(np.int64).sum()) == k["sum_c"]
        assert int(v.astype(np.int64).sum()) == k["sum_v"]
        assert int(c[-1]) == k["c_last"]
        assert int(sum(int(x) * int(x) for x in c) % (1 << 61)) == k["sum_c_sq_mod"]


def test_csv_parse_golden(golden_dir):
    g = _load(golden_dir, "csv.json")
    for key in ("daily", "minute"):
        o, h, lo, c, v = F.parse_csv(g[key]["text"].encode())
        assert c.tolist() == g[key]["c"] and h.tolist() == g[key]["h"]
        assert lo.tolist() == g[key]["l"] and o.tolist() == g[key]["o"]
    for name, case in g["good"].items():
        o, h, lo, c, v = F.parse_csv(case["text"].encode())
        assert c.tolist() == case["c"], name
        assert h.tolist() == case["h"] and lo.tolist() == case["l"] and o.tolist() == case["o"]
    for name, text in g["bad"].items():
        with pytest.raises(ValueError):
            F.parse_csv(text.encode())


def _check_case(strategy, ohlc, case, ann, where):
    p = case["params"]
    o, h, lo, c = (np.asarray(x, np.int32) for x in ohlc)
    if strategy == "sma":
        s, tr = F.sma(c, p["f"], p["s"], ann, 5000)
    elif strategy == "ema_ols":
        s, tr = F.ema_ols(c, p["n"], p["w"], p["band_bps"], ann, 5000)
    else:
        s, tr = F.boll(h, lo, c, p["w"], p["k_num"], p["k_den"], p["sl"], p["tp"], ann, 5000)
    e = case["summary"]
    assert int(s["n_trades"]) == e["n"], where
    assert int(s["pnl"]) == e["pnl"] and int(s["mdd"]) == e["mdd"], where
    assert int(s["exposure"]) == e["exposure"], where
    assert F.i128(s["s1_lo"], s["s1_hi"]) == int(e["s1"]), where
    assert F.i128(s["s2_lo"], s["s2_hi"]) == int(e["s2"]), where
    assert float(s["sharpe"]) == float.fromhex(e["sharpe"]), where
    assert f"{int(s['hash']):016x}" == e["h"], where
    got = [[int(t[k]) for k in ("entry_bar", "exit_bar", "side", "entry_px", "exit_px")] for t in tr]
    assert got == case["trades"], where


@pytest.mark.parametrize("name", ["sma_daily", "ema_ols_minute", "boll_minute"])
def test_strategy_golden(golden_dir, name):
    fx = _load(golden_dir, f"{name}.json")
    for sym in fx["symbols"]:
        o, h, lo, c, v = F.gen(int(sym["seed"], 16), sym["sym"], sym["bars"], sym["freq"])
        for case in sym["cases"]:
            _check_case(fx["strategy"], (o, h, lo, c), case, fx["ann"],
                        f"{name} sym {sym['sym']} {case['params']}")


def test_edge_golden(golden_dir):
    for series in _load(golden_dir, "edge.json"):
        ohlc = (series["o"], series["h"], series["l"], series["c"])
        for strategy in ("sma", "ema_ols", "boll"):
            ann = 252 if strategy == "sma" else 98280
            for case in series[strategy]:
                _check_case(strategy, ohlc, case, ann, f"edge {series['name']} {strategy}")


def test_fixed_point_sharpe_close_to_naive_fp64():
    """Spec §3: the exact fixed-point Sharpe agrees with a naive fp64 sequential-sum Sharpe
    far inside north_star's 1e-9 relative tolerance on well-conditioned lanes."""
    worst = 0.0
    for sym in range(4):
        o, h, lo, c, v = F.gen(0x5EED, sym, 2520, 0)
        for f, s in [(4, 50), (10, 120), (42, 240)]:
            r, _ = F.sma(c, f, s, 252)
            if abs(r["sharpe_f64"]) > 1e-3:
                worst = max(worst, abs(r["sharpe"] / r["sharpe_f64"] - 1))
    assert worst < 1e-11


def test_numpy_restatement_matches_c_fresh():
    """Fresh random cases (not in the fixtures): both restatements agree bit-for-bit."""
    import oracle_np as N
    rng = np.random.default_rng(2024)
    for _ in range(6):
        seed = int(rng.integers(0, 2**63))
        sym = int(rng.integers(0, 10**6))
        bars = int(rng.integers(1, 400))
        o, h, lo, c, v = F.gen(seed, sym, bars, 1)
        no, nh, nl, nc, nv = N.gen(seed, [sym], bars, 1)
        assert np.array_equal(c, nc[0]) and np.array_equal(h, nh[0]) and np.array_equal(lo, nl[0])
        f, s = int(rng.integers(1, 30)), int(rng.integers(1, 60))
        r, _ = F.sma(c, f, s, 252, 0)
        e, _ = N.run("sma", (o, h, lo, c), {"f": f, "s": s}, 252)
        assert int(r["pnl"]) == e["pnl"] and float(r["sharpe"]) == e["sharpe"] and int(r["hash"]) == e["h"]
        w = int(rng.integers(2, 40))
        r, _ = F.boll(h, lo, c, w, 3, 2, 50, 100, 98280, 0)
        e, _ = N.run("boll", (o, h, lo, c), {"w": w, "k_num": 3, "k_den": 2, "sl": 50, "tp": 100}, 98280)
        assert int(r["pnl"]) == e["pnl"] and int(r["mdd"]) == e["mdd"] and int(r["hash"]) == e["h"]


def test_sltp_level_floor():
    """k_tile.hip level_y: trunc(fl(ce * fl(f * fl(1e-4))) + 2^-16) == floor(ce * f / 10000) (the
    oracle's integer SL/TP levels, oracle/oracle.c orc_boll) for every factor f = 10000 -+ bps,
    bps in [0, 9999], at random prices and at prices whose product leaves remainder 0, 1 or 9999
    (the only places a rounding error could move the truncation) near 2^31."""
    rng = np.random.default_rng(12)
    f = np.concatenate([10000 - np.arange(10000), 10000 + np.arange(10000)]).astype(np.int64)
    g = f.astype(np.float64) * 1e-4
    ce = np.concatenate([[1, 2, 9999, 10000, 10001, 2 ** 30, 2 ** 31 - 2, 2 ** 31 - 1],
                         rng.integers(1, 2 ** 31, 40)]).astype(np.int64)
    y = ce[None, :].astype(np.float64) * g[:, None] + 2.0 ** -16
    assert np.array_equal(np.trunc(y).astype(np.int64), (ce[None, :] * f[:, None]) // 10000)
    # adversarial remainders: prices ce = 2^31 - k with ce * f % 10000 in {0, 1, 9999}
    c = (2 ** 31 - 1 - np.arange(10000, dtype=np.int64))
    for fi, gi in zip(f[::3], g[::3]):
        r = (c * fi) % 10000
        sel = c[(r == 0) | (r == 1) | (r == 9999)]
        got = np.trunc(sel.astype(np.float64) * gi + 2.0 ** -16).astype(np.int64)
        assert np.array_equal(got, (sel * fi) // 10000), f"level mismatch f={fi}"


def test_biased_reciprocal_floor():
    """k_sma.hip floor_key: trunc(F * key_recip(W)) == floor(F / W) for every window length the
    SMA kernel can hold (W <= 16,384; its LDS ring caps windows near 16,000) and F/W < 2^31,
    checked at and around every tested multiple of W (the only places a rounding error could
    move the truncation)."""
    rng = np.random.default_rng(11)
    W = np.arange(1, 16385, dtype=np.int64)[:, None]
    iw = (1.0 / W.astype(np.float64)) * (1.0 + 2.0 ** -47)   # device_common.h key_recip
    n = np.concatenate([[0, 1, 2, 10_000, 2 ** 31 - 2, 2 ** 31 - 1],
                        rng.integers(1, 2 ** 31 - 1, 120)]).astype(np.int64)[None, :]
    for r in (lambda w: 0 * w, lambda w: np.minimum(1, w - 1), lambda w: w - 1, lambda w: w // 2,
              lambda w: rng.integers(0, 1 << 20, w.shape) % w):
        rem = r(W)
        F = n * W + rem                                  # < 2^43: exact as float64
        got = np.trunc(F.astype(np.float64) * iw).astype(np.int64)
        assert np.array_equal(got, np.broadcast_to(n, got.shape)), "floor key mismatch"
