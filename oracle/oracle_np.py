"""oracle_np.py — numpy / pure-Python restatement of the backtest hot path.

TEST INFRASTRUCTURE ONLY: used by oracle/make_golden.py to write tests/golden/ and by tests.
It is deliberately written differently from oracle/oracle.c (vectorised generator, direct
window formulas instead of running sums, Python big ints instead of int64/int128) so that the
two restatements of docs/oracle_spec.md cross-check each other.

Reference anchors: the job function replaced is /root/reference/src/worker/process.rs:13-29
(a 1000 ms sleep per job, process.rs:23); Job.File bytes come from
/root/reference/src/server/main.rs:164-180. Parity unpinned against the reference (it has no
arithmetic and no tests: SURVEY.md §4, §8(c)); pinned to the authored spec only.
"""
from __future__ import annotations

import datetime as _dt
import math

import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
MASK = (1 << 64) - 1
MIX_K = 0xBF58476D1CE4E5B9  # trade hash (spec §4): h = sum of mix(w) mod 2^64
DAILY, MINUTE = 0, 1


# --------------------------------------------------------------------------- spec §1
def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def draws(seed: int, syms: np.ndarray, k: np.ndarray) -> np.ndarray:
    """u[s, j] = SplitMix64 draw number k[j] of symbol syms[s] (counter form)."""
    s0 = np.uint64(seed & MASK) ^ (syms.astype(np.uint64) * np.uint64(GOLDEN))
    with np.errstate(over="ignore"):
        z = s0[:, None] + (k.astype(np.uint64)[None, :] + np.uint64(1)) * np.uint64(GOLDEN)
        return _mix(z)


def _tdiv(a: np.ndarray, b: int) -> np.ndarray:
    """C-style truncating division of int64 by a positive int."""
    return np.sign(a) * (np.abs(a) // b)


def gen(seed: int, syms, bars: int, freq: int = DAILY):
    """Return (o, h, l, c, v) int64 arrays of shape [len(syms), bars]."""
    syms = np.asarray(syms, dtype=np.int64)
    m = 17320 if freq == DAILY else 866
    r = m // 4 + 1
    u = draws(seed, syms, np.arange(1 + 7 * bars, dtype=np.uint64))
    c0 = 1_000_000 + (u[:, 0] % np.uint64(9_000_001)).astype(np.int64)
    body = u[:, 1:].reshape(len(syms), bars, 7)
    walk = (body[:, :, 0:4] % np.uint64(2 * m + 1)).astype(np.int64).sum(axis=2) - 4 * m
    hoff = (body[:, :, 4] % np.uint64(r)).astype(np.int64)
    loff = (body[:, :, 5] % np.uint64(r)).astype(np.int64)
    vol = 1000 + (body[:, :, 6] % np.uint64(100_000)).astype(np.int64)
    c = np.empty((len(syms), bars), np.int64)
    o = np.empty_like(c)
    c[:, 0] = c0
    o[:, 0] = c0
    for t in range(1, bars):
        prev = c[:, t - 1]
        nxt = prev + _tdiv(walk[:, t] * prev, 1_000_000)
        c[:, t] = np.clip(nxt, 10_000, 2**31 - 2**20)
        o[:, t] = prev
    h = np.maximum(o, c) + hoff
    lo = np.maximum(np.minimum(o, c) - loff, 10_000)
    return o, h, lo, c, vol


def csv_bytes(o, h, l, c, v, freq: int = DAILY) -> bytes:
    """One symbol's bars as the spec §1 CSV."""
    out = ["timestamp,open,high,low,close,volume"]
    day0 = _dt.date(2010, 1, 4)

    def bday(i):
        return day0 + _dt.timedelta(days=7 * (i // 5) + i % 5)

    def px(x):
        x = int(x)
        return f"{x // 10000}.{x % 10000:04d}"

    for t in range(len(c)):
        if freq == DAILY:
            ts = bday(t).isoformat()
        else:
            d, mnt = divmod(t, 390)
            hh, mm = divmod(9 * 60 + 30 + mnt, 60)
            ts = f"{bday(d).isoformat()} {hh:02d}:{mm:02d}:00"
        out.append(f"{ts},{px(o[t])},{px(h[t])},{px(l[t])},{px(c[t])},{int(v[t])}")
    return ("\n".join(out) + "\n").encode()


# --------------------------------------------------------------------------- spec §3-4
def fixed_returns(c):
    """q_t, q2_t (spec §3) as Python ints; index 0 unused (0)."""
    q = [0] * len(c)
    q2 = [0] * len(c)
    for t in range(1, len(c)):
        ret = float(int(c[t]) - int(c[t - 1])) / float(int(c[t - 1]))
        q[t] = int(round(ret * 2.0**56))          # round(): half to even, like rint
        q2[t] = int(round((ret * ret) * 2.0**56))
    return q, q2


def _sharpe(s1, s2, bars, ann):
    if bars < 2:
        return 0.0
    n = float(bars - 1)
    m = math.ldexp(float(s1), -56) / n            # float(int): round to nearest even
    v = math.ldexp(float(s2), -56) / n - m * m
    return (m / math.sqrt(v)) * math.sqrt(float(ann)) if v > 0 else 0.0


def account(c, positions, exits, ann):
    """Score a position path.

    positions[t] = position after bar t; exits[t] = fill price of a close at bar t (None =
    close). Returns (summary dict, trades list)."""
    q, q2 = fixed_returns(c)
    trades = []
    pos = 0
    entry_bar = entry_px = 0
    realized = peak = mdd = 0
    s1 = s2 = expo = 0
    h = 0
    for t in range(len(c)):
        if t >= 1 and pos:
            s1 += pos * q[t]
            s2 += q2[t]
            expo += 1
        np_ = positions[t]
        if np_ != pos:
            if pos:
                px = exits[t] if exits[t] is not None else int(c[t])
                realized += pos * (px - entry_px)
                w = entry_bar | (t << 31) | ((1 if pos > 0 else 0) << 62)
                z = ((w ^ (w >> 29)) * MIX_K) & MASK
                h = (h + (z ^ (z >> 32))) & MASK
                trades.append((entry_bar, t, pos, entry_px, px))
            if np_:
                entry_bar, entry_px = t, int(c[t])
            pos = np_
        eq = realized + pos * (int(c[t]) - entry_px) if pos else realized
        peak = max(peak, eq)
        mdd = max(mdd, peak - eq)
    summ = dict(n=len(trades), pnl=realized, mdd=mdd, exposure=expo, s1=s1, s2=s2,
                sharpe=_sharpe(s1, s2, len(c), ann), h=h)
    return summ, trades


# --------------------------------------------------------------------------- spec §5
def sma_positions(c, f, s):
    c = [int(x) for x in c]
    bars = len(c)
    pos, out = 0, []
    for t in range(bars):
        if t == bars - 1:
            pos = 0
        elif t >= max(f, s) - 1:
            F = sum(c[t - f + 1:t + 1])
            L = sum(c[t - s + 1:t + 1])
            if F * s > L * f:
                pos = 1
            elif F * s < L * f:
                pos = -1
        out.append(pos)
    return out, [None] * bars


def ema_ols_positions(c, n, w, band_bps=20):
    c = [int(x) for x in c]
    bars = len(c)
    alpha = 2.0 / (float(n) + 1.0)
    e = 0.0
    coef = np.arange(w, dtype=np.int64) * 2 - (w - 1)
    pos, out = 0, []
    for t in range(bars):
        e = float(c[0]) if t == 0 else e + alpha * (float(c[t]) - e)
        if t == bars - 1:
            pos = 0
        elif t >= max(n, w) - 1:
            N = int(sum(int(k) * x for k, x in zip(coef, c[t - w + 1:t + 1])))
            cd = float(c[t])
            if pos == 1:
                if cd >= e:
                    pos = 0
            elif pos == -1:
                if cd <= e:
                    pos = 0
            else:
                lhs = cd * 10000.0
                if lhs < e * float(10000 - band_bps) and N >= 0:
                    pos = 1
                elif lhs > e * float(10000 + band_bps) and N <= 0:
                    pos = -1
        out.append(pos)
    return out, [None] * bars


def boll_positions(h, lo, c, w, k_num, k_den, sl, tp):
    h = [int(x) for x in h]
    lo = [int(x) for x in lo]
    c = [int(x) for x in c]
    bars = len(c)
    pos = entry = 0
    sl_l = tp_l = 0
    out, exits = [], []
    for t in range(bars):
        exit_px = None
        exited = False
        if pos and t >= entry + 1:
            if pos == 1:
                if lo[t] <= sl_l:
                    exit_px = sl_l
                elif h[t] >= tp_l:
                    exit_px = tp_l
            else:
                if h[t] >= sl_l:
                    exit_px = sl_l
                elif lo[t] <= tp_l:
                    exit_px = tp_l
            if exit_px is not None:
                pos, exited = 0, True
        if t == bars - 1:
            pos = 0
        elif t >= w - 1:
            win = c[t - w + 1:t + 1]
            sc = sum(win)
            D = w * c[t] - sc
            Q = w * sum(x * x for x in win) - sc * sc
            if pos == 1 and D >= 0:
                pos = 0
            elif pos == -1 and D <= 0:
                pos = 0
            elif pos == 0 and not exited:
                big = D * D * k_den * k_den > k_num * k_num * Q
                if D < 0 and big:
                    pos, entry = 1, t
                    sl_l = c[t] * (10000 - sl) // 10000
                    tp_l = c[t] * (10000 + tp) // 10000
                elif D > 0 and big:
                    pos, entry = -1, t
                    sl_l = c[t] * (10000 + sl) // 10000
                    tp_l = c[t] * (10000 - tp) // 10000
        out.append(pos)
        exits.append(exit_px)
    return out, exits


def run(strategy: str, ohlc, params: dict, ann: int):
    o, h, lo, c = ohlc
    if strategy == "sma":
        p, e = sma_positions(c, params["f"], params["s"])
    elif strategy == "ema_ols":
        p, e = ema_ols_positions(c, params["n"], params["w"], params.get("band_bps", 20))
    elif strategy == "boll":
        p, e = boll_positions(h, lo, c, params["w"], params["k_num"], params["k_den"],
                              params["sl"], params["tp"])
    else:
        raise ValueError(strategy)
    return account(c, p, e, ann)
