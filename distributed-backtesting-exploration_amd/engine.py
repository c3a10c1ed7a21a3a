"""ctypes binding of libbt.so (include/bt.h) — the MI355X backtest engine.

This is the Python face of the C ABI that replaces the reference worker's job function
(/root/reference/src/worker/process.rs:13-29). Every result comes from the HIP kernels;
there is no CPU fallback: if libbt.so or a GPU is missing, constructing an Engine raises.
"""
from __future__ import annotations

import ctypes as C
import importlib.util
import os
import subprocess
import sys
from dataclasses import dataclass, field
from typing import Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# BT_LIB (tuning aid): another in-tree build of the library under dev/, e.g. dev/prof.so (the
# profiling build, `make PROFILING=1`) or dev/base.so for an A/B; nothing outside the package
_bt_lib = os.path.normpath(os.environ.get("BT_LIB", "libbt.so"))
if _bt_lib.startswith("..") or os.path.isabs(_bt_lib):
    raise ImportError(f"BT_LIB={_bt_lib}: a path inside {PKG_DIR} (libbt.so or dev/NAME.so)")
LIB_PATH = os.path.join(PKG_DIR, _bt_lib)
CSRC = os.path.join(PKG_DIR, "csrc")
# include/bt.h BT_ABI_VERSION this wrapper is written against (build() checks the built library)
ABI_VERSION = 3
PIPE_SLOTS = 4  # include/bt.h BT_PIPE_SLOTS: pinned read-back / exchange slots

BT_SMA_CROSS, BT_EMA_OLS, BT_BOLL = 1, 2, 3
BT_FLAG_PARITY, BT_FLAG_TIMING = 1, 2
BT_DAILY, BT_MINUTE = 0, 1

SUMMARY_DTYPE = np.dtype([
    ("n_trades", "<i4"), ("status", "<i4"), ("pnl", "<i8"), ("mdd", "<i8"),
    ("exposure", "<i8"), ("sharpe", "<f8"), ("hash", "<u8"),
])
SUMS_DTYPE = np.dtype([("s1_lo", "<u8"), ("s1_hi", "<i8"), ("s2_lo", "<u8"), ("s2_hi", "<i8")])
TRADE_DTYPE = np.dtype([
    ("entry_bar", "<i4"), ("exit_bar", "<i4"), ("side", "<i4"), ("pad", "<i4"),
    ("entry_px", "<i8"), ("exit_px", "<i8"),
])
TOPK_DTYPE = np.dtype([("sharpe", "<f8"), ("sym", "<i4"), ("param", "<i4"), ("pnl", "<i8")])
assert SUMMARY_DTYPE.itemsize == 48 and TOPK_DTYPE.itemsize == 24 and TRADE_DTYPE.itemsize == 32


class BtError(RuntimeError):
    pass


class _Config(C.Structure):
    _fields_ = [
        ("strategy", C.c_int32),
        ("n_fast", C.c_int32), ("n_slow", C.c_int32),
        ("fast", C.POINTER(C.c_int32)), ("slow", C.POINTER(C.c_int32)),
        ("n_span", C.c_int32), ("n_ols", C.c_int32),
        ("span", C.POINTER(C.c_int32)), ("ols", C.POINTER(C.c_int32)),
        ("band_bps", C.c_int32),
        ("n_bwin", C.c_int32), ("n_k", C.c_int32), ("n_sl", C.c_int32), ("n_tp", C.c_int32),
        ("bwin", C.POINTER(C.c_int32)), ("k_num", C.POINTER(C.c_int32)),
        ("k_den", C.c_int32),
        ("sl_bps", C.POINTER(C.c_int32)), ("tp_bps", C.POINTER(C.c_int32)),
        ("annualization", C.c_int64),
        ("device", C.c_int32), ("topk", C.c_int32), ("flags", C.c_int32),
        ("host_threads", C.c_int32), ("trade_cap", C.c_int32),
        ("stream", C.c_void_p),
    ]


class _JobIn(C.Structure):
    _fields_ = [("id", C.c_char_p), ("file", C.c_void_p), ("len", C.c_size_t)]


class _JobOut(C.Structure):
    _fields_ = [("data", C.c_void_p), ("len", C.c_size_t), ("status", C.c_int32),
                ("n_bars", C.c_int32)]


class _BatchProfile(C.Structure):
    _fields_ = [("n_jobs", C.c_int64), ("n_failed", C.c_int64), ("payload_bytes", C.c_int64),
                ("payload_bytes_read", C.c_int64), ("bars", C.c_int64),
                ("host_ingest_ms", C.c_double), ("upload_ms", C.c_double),
                ("compute_ms", C.c_double), ("readback_ms", C.c_double),
                ("format_ms", C.c_double), ("total_ms", C.c_double)]


class _Stats(C.Structure):
    _fields_ = [("n_symbols", C.c_int64), ("n_params", C.c_int64), ("bar_evals", C.c_int64),
                ("trades", C.c_int64), ("errors", C.c_int64)]


_lib = None


def build(force: bool = False) -> str:
    """Compile libbt.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-j8", "-C", CSRC], check=True)
    return LIB_PATH


def _one_hip_runtime():
    """libbt.so needs libamdhip64.so.7 by SONAME. PyTorch-ROCm loads its bundled HIP and HSA
    runtimes by path, so a process that loads libbt.so first and torch afterwards holds two HSA
    runtimes, and torch then finds no GPU ("No HIP GPUs are available"; measured on the MI355X,
    scripts/dev/torch_after_libbt.py). With torch installed, importing it first lets libbt.so bind
    torch's copy: one runtime per process, whatever the caller imports later."""
    if "torch" in sys.modules:
        return
    if importlib.util.find_spec("torch") is not None:
        import torch  # noqa: F401


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BtError(f"{LIB_PATH} missing: run __graft_entry__.build() (no CPU fallback)")
    _one_hip_runtime()
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    L.bt_engine_create.argtypes = [C.POINTER(_Config), C.c_char_p, C.c_size_t]
    L.bt_engine_create.restype = P
    L.bt_engine_destroy.argtypes = [P]
    L.bt_engine_destroy.restype = None
    L.bt_last_error.restype = C.c_char_p
    L.bt_abi_version.restype = C.c_int32
    L.bt_num_params.argtypes = [P]
    L.bt_set_segments.argtypes = [P, C.c_int32, C.c_int32]
    L.bt_last_segments.argtypes = [P, C.POINTER(C.c_int64)]
    L.bt_run_batch.argtypes = [P, C.c_size_t, C.POINTER(_JobIn), C.POINTER(_JobOut)]
    L.bt_job_out_free.argtypes = [C.POINTER(_JobOut), C.c_size_t]
    L.bt_job_out_free.restype = None
    L.bt_load_synthetic.argtypes = [P, C.c_uint64, C.c_int64, C.c_int32, C.c_int32, C.c_int32]
    L.bt_load_ohlc.argtypes = [P, C.c_int32, P, P, P, P, P, P]
    for f in ("bt_run", "bt_sync", "bt_reset_timing"):
        getattr(L, f).argtypes = [P]
    L.bt_read_summaries.argtypes = [P, P, C.c_size_t]
    L.bt_read_sums.argtypes = [P, P, C.c_size_t]
    L.bt_read_trades.argtypes = [P, P, C.c_size_t]
    L.bt_read_topk.argtypes = [P, P, C.c_int32]
    L.bt_read_stats.argtypes = [P, C.POINTER(_Stats)]
    L.bt_topk_fetch_async.argtypes = [P, C.c_int32]
    L.bt_topk_fetch_wait.argtypes = [P, C.c_int32, P, C.c_int32, C.POINTER(C.c_int64)]
    L.bt_read_close.argtypes = [P, C.c_int32, P, C.c_int32]
    L.bt_kernel_timing.argtypes = [P, C.POINTER(C.c_double), C.POINTER(C.c_int64),
                                   C.POINTER(C.c_char_p)]
    L.bt_merge_topk.argtypes = [P, C.c_size_t, C.c_int32, P]
    L.bt_i128_to_double.argtypes = [C.c_uint64, C.c_int64]
    L.bt_i128_to_double.restype = C.c_double
    L.bt_parse_csv.argtypes = [C.c_char_p, C.c_size_t, C.c_int32, P, P, P, C.c_char_p,
                               C.c_size_t]
    L.bt_parse_job.argtypes = L.bt_parse_csv.argtypes
    L.bt_encode_columns.argtypes = [P, P, P, P, P, C.c_int32, P, C.c_size_t]
    L.bt_encode_columns.restype = C.c_int64
    L.bt_gen_payload.argtypes = [C.c_uint64, C.c_int64, C.c_int32, C.c_int32, P, C.c_size_t]
    L.bt_gen_payload.restype = C.c_int64
    L.bt_last_batch_profile.argtypes = [P, C.POINTER(_BatchProfile)]
    L.bt_format_summaries.argtypes = [P, C.c_int32, P, C.c_size_t]
    L.bt_format_summaries.restype = C.c_int64
    _lib = L
    return L


# Entry points added after ABI version 2 (the multi-GPU exchange), bound on first use: an older
# library (e.g. a previous round's build, loaded with BT_LIB for a regression check) then still
# loads and runs everything else. Each carries the first ABI version whose signature it matches:
# a symbol whose signature changed (bt_exchange_merge gained block_bytes in ABI 3) must not be
# bound with the new argument list on a library that exports the old one.
_LATE_SYMBOLS = {
    "bt_comm_unique_id": (2, [C.c_void_p], C.c_int32),
    "bt_comm_create": (2, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_char_p,
                           C.c_size_t], C.c_void_p),
    "bt_comm_destroy": (2, [C.c_void_p], None),
    "bt_exchange_async": (2, [C.c_void_p, C.c_void_p, C.c_int32], C.c_int32),
    "bt_exchange_wait": (2, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p], C.c_int32),
    "bt_exchange_message_bytes": (2, [C.c_int32], C.c_int64),
    "bt_exchange_merge": (3, [C.c_void_p, C.c_size_t, C.c_int32, C.c_int32, C.c_void_p, C.c_int32,
                              C.c_void_p], C.c_int32),
}
_late = {}


def sym(name: str):
    """A late (post-v2) entry point of libbt.so, typed on first use. BtError if the loaded
    library's ABI predates the signature bound here (or AttributeError if it lacks the symbol)."""
    f = _late.get(name)
    if f is None:
        min_abi, argtypes, restype = _LATE_SYMBOLS[name]
        have = lib().bt_abi_version()
        if have < min_abi:
            raise BtError(f"{name}: {LIB_PATH} has ABI {have}, this binding needs ABI >= {min_abi}")
        f = getattr(lib(), name)
        f.argtypes, f.restype = argtypes, restype
        _late[name] = f
    return f


def _check(rc):
    if rc < 0:
        raise BtError(lib().bt_last_error().decode())
    return rc


def _arr(v) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(v, dtype=np.int32))


@dataclass
class Grid:
    """Worker-side parameter grid (the proto carries none: SURVEY.md §7 hard part 5)."""
    strategy: int
    axes: Sequence[Sequence[int]]
    band_bps: int = 20
    k_den: int = 2
    annualization: int = 252
    _keep: list = field(default_factory=list, repr=False)

    @property
    def n_params(self) -> int:
        n = 1
        for a in self.axes:
            n *= len(a)
        return n

    @staticmethod
    def sma(fast, slow, annualization=252):
        return Grid(BT_SMA_CROSS, [list(fast), list(slow)], annualization=annualization)

    @staticmethod
    def ema_ols(span, ols, band_bps=20, annualization=98280):
        return Grid(BT_EMA_OLS, [list(span), list(ols)], band_bps=band_bps,
                    annualization=annualization)

    @staticmethod
    def boll(win, k_num, sl_bps, tp_bps, k_den=2, annualization=98280):
        return Grid(BT_BOLL, [list(win), list(k_num), list(sl_bps), list(tp_bps)], k_den=k_den,
                    annualization=annualization)

    def param(self, p: int) -> dict:
        """Decode a param index (include/bt.h ordering) into named values."""
        if self.strategy == BT_SMA_CROSS:
            return {"f": self.axes[0][p // len(self.axes[1])], "s": self.axes[1][p % len(self.axes[1])]}
        if self.strategy == BT_EMA_OLS:
            return {"n": self.axes[0][p // len(self.axes[1])], "w": self.axes[1][p % len(self.axes[1])],
                    "band_bps": self.band_bps}
        nk, nsl, ntp = (len(a) for a in self.axes[1:])
        return {"w": self.axes[0][p // (ntp * nsl * nk)], "k_num": self.axes[1][(p // (ntp * nsl)) % nk],
                "k_den": self.k_den, "sl": self.axes[2][(p // ntp) % nsl], "tp": self.axes[3][p % ntp]}

    def to_c(self, device=0, topk=0, flags=0, host_threads=0, trade_cap=0, stream=None) -> _Config:
        cfg = _Config()
        cfg.strategy = self.strategy
        arrs = [_arr(a) for a in self.axes]
        self._keep = arrs
        ptr = [a.ctypes.data_as(C.POINTER(C.c_int32)) for a in arrs]
        if self.strategy == BT_SMA_CROSS:
            cfg.n_fast, cfg.n_slow = len(arrs[0]), len(arrs[1])
            cfg.fast, cfg.slow = ptr
        elif self.strategy == BT_EMA_OLS:
            cfg.n_span, cfg.n_ols = len(arrs[0]), len(arrs[1])
            cfg.span, cfg.ols = ptr
            cfg.band_bps = self.band_bps
        else:
            cfg.n_bwin, cfg.n_k, cfg.n_sl, cfg.n_tp = (len(a) for a in arrs)
            cfg.bwin, cfg.k_num, cfg.sl_bps, cfg.tp_bps = ptr
            cfg.k_den = self.k_den
        cfg.annualization = self.annualization
        cfg.device, cfg.topk, cfg.flags = device, topk, flags
        cfg.host_threads, cfg.trade_cap = host_threads, trade_cap
        cfg.stream = stream
        return cfg


# Pinned grids of BASELINE.json configs.
def config2_grid():
    return Grid.sma(range(4, 43, 2), range(50, 241, 10), annualization=252)


def config3_grid():
    return Grid.ema_ols([10, 20, 30, 60, 120, 240, 390, 780],
                        [15, 30, 60, 120, 240, 390, 780, 1560], band_bps=20, annualization=98280)


def config4_grid():
    return Grid.boll([10, 20, 30, 45, 60, 90, 120, 240], [3, 4, 5, 6], [50, 100],
                     [50, 100, 200, 400], k_den=2, annualization=98280)


def config5_grid():
    # SMA fast 32 x slow 32 on 1-min bars
    return Grid.sma(range(5, 161, 5), range(200, 6401, 200), annualization=98280)


class Engine:
    """One engine per GPU (one process per GPU)."""

    def __init__(self, grid: Grid, device=0, topk=0, parity=False, timing=False,
                 trade_cap=0, host_threads=0, stream=None):
        self.grid = grid
        flags = (BT_FLAG_PARITY if parity else 0) | (BT_FLAG_TIMING if timing else 0)
        cfg = grid.to_c(device, topk, flags, host_threads, trade_cap, stream)
        err = C.create_string_buffer(512)
        h = lib().bt_engine_create(C.byref(cfg), err, 512)
        if not h:
            raise BtError(err.value.decode())
        self._h = h
        self.n_params = lib().bt_num_params(h)
        self.trade_cap = trade_cap
        self.n_symbols = 0
        self.topk = topk

    def close(self):
        if getattr(self, "_h", None):
            lib().bt_engine_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- HBM-resident path
    def load_synthetic(self, seed, sym_begin, n_sym, n_bars, freq=BT_DAILY):
        _check(lib().bt_load_synthetic(self._h, seed & ((1 << 64) - 1), sym_begin, n_sym, n_bars, freq))
        self.n_symbols = n_sym

    def load_ohlc(self, closes, highs=None, lows=None, sym_ids=None):
        """closes: list of 1-D int arrays (ragged allowed)."""
        bars = np.array([len(c) for c in closes], np.int32)
        offs = np.zeros(len(closes), np.int64)
        if len(closes):
            offs[1:] = np.cumsum(bars[:-1])
        cat = lambda xs: np.ascontiguousarray(np.concatenate([np.asarray(x, np.int32) for x in xs])) if len(xs) else np.zeros(1, np.int32)
        c = cat(closes)
        h = cat(highs) if highs is not None else None
        lo = cat(lows) if lows is not None else None
        ids = np.ascontiguousarray(np.arange(len(closes), dtype=np.int64) if sym_ids is None
                                   else np.asarray(sym_ids, np.int64))
        ptr = lambda a: None if a is None else a.ctypes.data
        _check(lib().bt_load_ohlc(self._h, len(closes), ids.ctypes.data, bars.ctypes.data,
                                  offs.ctypes.data, ptr(h), ptr(lo), c.ctypes.data))
        self.n_symbols = len(closes)

    def run(self):
        _check(lib().bt_run(self._h))

    def set_segments(self, segments: int, burn_tiles: int = 0) -> None:
        """Bar-axis split of the EMA+OLS / Bollinger walks: 0 = automatic, 1 = off, n = n
        segments per symbol; burn_tiles 0 = the strategy's default burn-in."""
        _check(lib().bt_set_segments(self._h, segments, burn_tiles))

    def last_segments(self, with_refixed: bool = False):
        """Segments per symbol of the last run (and, with_refixed, the fix pass's re-walks)."""
        n = C.c_int64(0)
        g = _check(lib().bt_last_segments(self._h, C.byref(n)))
        return (g, int(n.value)) if with_refixed else g

    def sync(self):
        _check(lib().bt_sync(self._h))

    def summaries(self) -> np.ndarray:
        n = self.n_symbols * self.n_params
        out = np.zeros(max(n, 1), SUMMARY_DTYPE)
        _check(lib().bt_read_summaries(self._h, out.ctypes.data, n))
        return out[:n].reshape(self.n_symbols, self.n_params)

    def sums(self) -> np.ndarray:
        n = self.n_symbols * self.n_params
        out = np.zeros(max(n, 1), SUMS_DTYPE)
        _check(lib().bt_read_sums(self._h, out.ctypes.data, n))
        return out[:n].reshape(self.n_symbols, self.n_params)

    def trades(self) -> np.ndarray:
        n = self.n_symbols * self.n_params * self.trade_cap
        out = np.zeros(max(n, 1), TRADE_DTYPE)
        _check(lib().bt_read_trades(self._h, out.ctypes.data, n))
        return out[:n].reshape(self.n_symbols, self.n_params, self.trade_cap)

    def read_topk(self, k=None) -> np.ndarray:
        k = k or self.topk
        out = np.zeros(k, TOPK_DTYPE)
        m = _check(lib().bt_read_topk(self._h, out.ctypes.data, k))
        return out[:m]

    def topk_fetch_async(self, slot: int) -> None:
        """Enqueue the read-back of the last run's top-k and trade count into pinned slot
        0 .. PIPE_SLOTS-1 (no host wait): later runs can be enqueued before these records are
        consumed."""
        _check(lib().bt_topk_fetch_async(self._h, slot))

    def topk_fetch_wait(self, slot: int, k=None) -> tuple:
        """Wait for the slot's read-back; returns (top-k records, trades of that run)."""
        k = k or self.topk
        out = np.zeros(k, TOPK_DTYPE)
        n = C.c_int64(0)
        m = _check(lib().bt_topk_fetch_wait(self._h, slot, out.ctypes.data, k, C.byref(n)))
        return out[:m], int(n.value)

    def stats(self) -> dict:
        st = _Stats()
        _check(lib().bt_read_stats(self._h, C.byref(st)))
        return {f: getattr(st, f) for f, _ in _Stats._fields_}

    def close_column(self, sym_index, n) -> np.ndarray:
        out = np.zeros(n, np.int32)
        _check(lib().bt_read_close(self._h, sym_index, out.ctypes.data, n))
        return out

    def kernel_timing(self):
        ms, n, name = C.c_double(), C.c_int64(), C.c_char_p()
        _check(lib().bt_kernel_timing(self._h, C.byref(ms), C.byref(n), C.byref(name)))
        return ms.value, n.value, name.value.decode()

    def reset_timing(self):
        _check(lib().bt_reset_timing(self._h))

    # ---- the JobsReply batch (drop-in for process_incoming_job)
    def run_batch(self, jobs: Sequence[tuple]) -> list:
        """jobs: [(id: str, file: bytes)] -> [(status, data: str)] in job order."""
        n = len(jobs)
        jin = (_JobIn * max(n, 1))()
        keep = []
        for i, (jid, data) in enumerate(jobs):
            b = bytes(data)
            idb = jid.encode() if isinstance(jid, str) else bytes(jid)
            keep += [b, idb]
            jin[i].id = idb
            jin[i].file = C.cast(C.c_char_p(b), C.c_void_p)
            jin[i].len = len(b)
        jout = (_JobOut * max(n, 1))()
        try:
            _check(lib().bt_run_batch(self._h, n, jin, jout))
            res = [(jout[i].status, C.string_at(jout[i].data, jout[i].len).decode()) for i in range(n)]
        finally:
            lib().bt_job_out_free(jout, n)  # safe on NULL entries, also after a failure
        return res

    def batch_profile(self) -> dict:
        """Phase times of the last run_batch (bt_last_batch_profile)."""
        pr = _BatchProfile()
        _check(lib().bt_last_batch_profile(self._h, C.byref(pr)))
        return {f: getattr(pr, f) for f, _ in _BatchProfile._fields_}


class Comm:
    """The multi-GPU exchange behind the C ABI (bt_comm_*, csrc/comm.cpp): one RCCL all-gather
    per run of every rank's top-k records and counters, from the engine's device buffers."""

    ID_BYTES = 128

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(Comm.ID_BYTES)
        _check(sym("bt_comm_unique_id")(buf))
        return buf.raw

    def __init__(self, uid: bytes, rank: int, world: int, device: int, k: int):
        if len(uid) != Comm.ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        err = C.create_string_buffer(512)
        self._uid = C.create_string_buffer(bytes(uid), Comm.ID_BYTES)
        h = sym("bt_comm_create")(self._uid, rank, world, device, k, err, 512)
        if not h:
            raise BtError(err.value.decode())
        self._h, self.k, self.world = h, k, world

    def exchange_async(self, engine: "Engine", slot: int) -> None:
        _check(sym("bt_exchange_async")(self._h, engine._h, slot))

    def exchange_wait(self, slot: int, k=None) -> tuple:
        """Merged global top-k and [bar-evals, trades] summed over ranks."""
        k = k or self.k
        out = np.zeros(k, TOPK_DTYPE)
        cnt = np.zeros(2, np.int64)
        m = _check(sym("bt_exchange_wait")(self._h, slot, out.ctypes.data, k, cnt.ctypes.data))
        return out[:m], [int(cnt[0]), int(cnt[1])]

    def close(self):
        if getattr(self, "_h", None):
            sym("bt_comm_destroy")(self._h)
            self._h = None

    __del__ = close


def merge_topk(records: np.ndarray, k: int) -> np.ndarray:
    """Host merge of shard top-k lists (same order as the device: sharpe desc, sym, param)."""
    recs = np.ascontiguousarray(records, TOPK_DTYPE)
    out = np.zeros(max(k, 1), TOPK_DTYPE)
    m = _check(lib().bt_merge_topk(recs.ctypes.data if len(recs) else None, len(recs), k,
                                   out.ctypes.data))
    return out[:m]


def exchange_message(records: np.ndarray, k_msg: int, bar_evals: int, trades: int) -> bytes:
    """One rank's exchange message as bt_exchange_async sends it (comm.cpp): a header record whose
    first int32 is the record count, k_msg record slots (the first n used), bar-evals, trades."""
    n = len(records)
    size = _check(sym("bt_exchange_message_bytes")(k_msg))
    buf = np.zeros(size, np.uint8)
    buf[:4] = np.frombuffer(np.int32(n).tobytes(), np.uint8)
    rec = TOPK_DTYPE.itemsize
    if n:
        buf[rec:rec * (1 + n)] = np.frombuffer(np.ascontiguousarray(records, TOPK_DTYPE).tobytes(), np.uint8)
    buf[rec * (k_msg + 1):] = np.frombuffer(np.array([bar_evals, trades], np.int64).tobytes(), np.uint8)
    return buf.tobytes()


def exchange_merge(block: bytes, world: int, k_msg: int, k: int) -> tuple:
    """The host half of Comm.exchange_wait (bt_exchange_merge) on a gathered block of `world`
    messages: the merged top-k and [bar-evals, trades] summed over ranks."""
    raw = np.frombuffer(block, np.uint8)
    need = world * _check(sym("bt_exchange_message_bytes")(k_msg))
    if len(raw) != need:  # the C side checks the same; fail before handing it a short buffer
        raise BtError(f"exchange block holds {len(raw)} bytes, expected {need} "
                      f"(world {world} x message of k_msg {k_msg})")
    out = np.zeros(max(k, 1), TOPK_DTYPE)
    cnt = np.zeros(2, np.int64)
    m = _check(sym("bt_exchange_merge")(raw.ctypes.data, len(raw), world, k_msg, out.ctypes.data,
                                        k, cnt.ctypes.data))
    return out[:m], [int(cnt[0]), int(cnt[1])]


def format_summaries(rows: np.ndarray) -> str:
    """The CompleteRequest.data text bt_run_batch writes for these summaries (spec §6)."""
    rows = np.ascontiguousarray(rows, SUMMARY_DTYPE)
    cap = _check(lib().bt_format_summaries(None, len(rows), None, 0))
    buf = C.create_string_buffer(max(cap, 1))
    n = _check(lib().bt_format_summaries(rows.ctypes.data if len(rows) else None, len(rows), buf, cap))
    return buf.raw[:n].decode()


def i128_to_double(lo: int, hi: int) -> float:
    return lib().bt_i128_to_double(lo & ((1 << 64) - 1), hi)


def parse_csv(data: bytes, cap=1 << 22):
    """Host ingest of one Job.File (CSV or binary columns) -> (high, low, close) int32 ticks."""
    cap = int(cap)
    h, lo, c = (np.empty(cap, np.int32) for _ in range(3))
    err = C.create_string_buffer(256)
    n = lib().bt_parse_job(data, len(data), cap, h.ctypes.data, lo.ctypes.data, c.ctypes.data,
                           err, 256)
    if n < 0:
        raise ValueError(err.value.decode())
    return h[:n].copy(), lo[:n].copy(), c[:n].copy()
