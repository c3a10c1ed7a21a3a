"""ctypes binding to oracle/liborc.so (the C oracle). TEST INFRASTRUCTURE ONLY.

Callers allowed by the build contract: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg — as the checker / CPU baseline, never as the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liborc.so")

SUMMARY_DTYPE = np.dtype([
    ("n_trades", "<i4"), ("status", "<i4"), ("pnl", "<i8"), ("mdd", "<i8"),
    ("exposure", "<i8"), ("sharpe", "<f8"), ("hash", "<u8"),
    ("s1_lo", "<u8"), ("s1_hi", "<i8"), ("s2_lo", "<u8"), ("s2_hi", "<i8"),
    ("sharpe_f64", "<f8"), ("pad", "<i8"),
])


def i128(lo, hi):
    """Python int from an int128 stored as (uint64 lo, int64 hi)."""
    return (int(hi) << 64) | int(lo)


TRADE_DTYPE = np.dtype([
    ("entry_bar", "<i4"), ("exit_bar", "<i4"), ("side", "<i4"), ("pad", "<i4"),
    ("entry_px", "<i8"), ("exit_px", "<i8"),
])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C")
        i64p = np.ctypeslib.ndpointer(np.int64, flags="C")
        sp = np.ctypeslib.ndpointer(SUMMARY_DTYPE, flags="C")
        L.orc_gen.argtypes = [C.c_uint64, C.c_int64, C.c_int32, C.c_int32] + [i32p] * 5
        L.orc_gen.restype = None
        L.orc_parse_csv.argtypes = [C.c_char_p, C.c_size_t, C.c_int32, i32p, i32p, i32p, i32p,
                                    i64p, C.c_char_p, C.c_size_t]
        L.orc_parse_csv.restype = C.c_int32
        L.orc_sma.argtypes = [i32p, C.c_int32, C.c_int32, C.c_int32, C.c_int64, sp,
                              C.c_void_p, C.c_int32]
        L.orc_ema_ols.argtypes = [i32p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int64,
                                  sp, C.c_void_p, C.c_int32]
        L.orc_boll.argtypes = [i32p, i32p, i32p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                               C.c_int32, C.c_int32, C.c_int64, sp, C.c_void_p, C.c_int32]
        L.orc_sma_grid_mt.argtypes = [i32p, C.c_int32, C.c_int32, i32p, C.c_int32, i32p,
                                      C.c_int32, C.c_int64, sp, C.c_int32]
        L.orc_ema_grid_mt.argtypes = [i32p, C.c_int32, C.c_int32, i32p, C.c_int32, i32p,
                                      C.c_int32, C.c_int32, C.c_int64, sp, C.c_int32]
        L.orc_boll_grid_mt.argtypes = [i32p, i32p, i32p, C.c_int32, C.c_int32, i32p, C.c_int32,
                                       i32p, C.c_int32, C.c_int32, i32p, C.c_int32, i32p,
                                       C.c_int32, C.c_int64, sp, C.c_int32]
        for f in (L.orc_sma, L.orc_ema_ols, L.orc_boll, L.orc_sma_grid_mt, L.orc_ema_grid_mt,
                  L.orc_boll_grid_mt):
            f.restype = None
        _lib = L
    return _lib


def gen(seed, sym, bars, freq=0):
    cols = [np.empty(bars, np.int32) for _ in range(5)]
    lib().orc_gen(seed & ((1 << 64) - 1), sym, bars, freq, *cols)
    return tuple(cols)  # o, h, l, c, v


def parse_csv(data: bytes, cap=1 << 22):
    cap = int(cap)
    o, h, lo, c = (np.empty(cap, np.int32) for _ in range(4))
    v = np.empty(cap, np.int64)
    err = C.create_string_buffer(256)
    n = lib().orc_parse_csv(data, len(data), cap, o, h, lo, c, v, err, 256)
    if n < 0:
        raise ValueError(err.value.decode())
    return o[:n].copy(), h[:n].copy(), lo[:n].copy(), c[:n].copy(), v[:n].copy()


def _run(fn, args, cap):
    out = np.zeros(1, SUMMARY_DTYPE)
    if cap:
        tr = np.zeros(cap, TRADE_DTYPE)
        fn(*args, out, tr.ctypes.data, cap)
        n = int(out["n_trades"][0])
        return out[0], tr[:min(n, cap)]
    fn(*args, out, None, 0)
    return out[0], None


def sma(c, f, s, ann, trades_cap=0):
    c = np.ascontiguousarray(c, np.int32)
    return _run(lib().orc_sma, (c, len(c), f, s, ann), trades_cap)


def ema_ols(c, n, w, band_bps, ann, trades_cap=0):
    c = np.ascontiguousarray(c, np.int32)
    return _run(lib().orc_ema_ols, (c, len(c), n, w, band_bps, ann), trades_cap)


def boll(h, lo, c, w, k_num, k_den, sl, tp, ann, trades_cap=0):
    h, lo, c = (np.ascontiguousarray(x, np.int32) for x in (h, lo, c))
    return _run(lib().orc_boll, (h, lo, c, len(c), w, k_num, k_den, sl, tp, ann), trades_cap)


def sma_grid_mt(closes, fast, slow, ann, nthreads):
    closes = np.ascontiguousarray(closes, np.int32)
    S, B = closes.shape
    fast = np.ascontiguousarray(fast, np.int32)
    slow = np.ascontiguousarray(slow, np.int32)
    out = np.zeros(S * len(fast) * len(slow), SUMMARY_DTYPE)
    lib().orc_sma_grid_mt(closes, S, B, fast, len(fast), slow, len(slow), ann, out, nthreads)
    return out.reshape(S, len(fast) * len(slow))


def ema_grid_mt(closes, span, ols, band_bps, ann, nthreads):
    closes = np.ascontiguousarray(closes, np.int32)
    S, B = closes.shape
    span, ols = (np.ascontiguousarray(x, np.int32) for x in (span, ols))
    out = np.zeros(S * len(span) * len(ols), SUMMARY_DTYPE)
    lib().orc_ema_grid_mt(closes, S, B, span, len(span), ols, len(ols), band_bps, ann, out, nthreads)
    return out.reshape(S, len(span) * len(ols))


def boll_grid_mt(highs, lows, closes, win, k_num, k_den, sl, tp, ann, nthreads):
    h, lo, c = (np.ascontiguousarray(x, np.int32) for x in (highs, lows, closes))
    S, B = c.shape
    win, k_num, sl, tp = (np.ascontiguousarray(x, np.int32) for x in (win, k_num, sl, tp))
    P = len(win) * len(k_num) * len(sl) * len(tp)
    out = np.zeros(S * P, SUMMARY_DTYPE)
    lib().orc_boll_grid_mt(h, lo, c, S, B, win, len(win), k_num, len(k_num), k_den, sl, len(sl),
                           tp, len(tp), ann, out, nthreads)
    return out.reshape(S, P)
