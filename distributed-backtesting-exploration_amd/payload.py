"""Binary columnar Job.File payloads (format in csrc/payload.cpp).

The reference dispatcher sends each symbol as the whole file it read
(/root/reference/src/server/main.rs:164-180) in `Job.File` (proto/backtesting.proto:15). A
5-year 1-minute CSV is ~29 MiB (> grpc's 4 MiB default) and parsing it dominates a gRPC-fed run,
so files may instead hold "DBXCOL1" columns (16 B per bar): the worker's `bt_run_batch` accepts
either format per job, dispatched on the magic. The dispatcher is unchanged — it still reads
bytes from disk; these helpers write such files.

    python -m dbx_amd.payload gen OUTDIR --symbols 16 --bars 98280 --freq minute
    python -m dbx_amd.payload csv2bin IN.csv OUT.dbxcol
"""
from __future__ import annotations

import argparse
import ctypes as C
import os

import numpy as np

from .engine import BT_DAILY, BT_MINUTE, lib

MAGIC = b"DBXCOL1\n"


def encode_columns(o, h, lo, c, v=None) -> bytes:
    """int32 open/high/low/close ticks (+ optional int64 volume) -> payload bytes."""
    cols = [np.ascontiguousarray(x, np.int32) for x in (o, h, lo, c)]
    n = len(cols[3])
    if any(len(x) != n for x in cols):
        raise ValueError("columns differ in length")
    vv = None if v is None else np.ascontiguousarray(v, np.int64)
    if vv is not None and len(vv) != n:
        raise ValueError("volume column differs in length")
    L = lib()
    ptrs = [x.ctypes.data for x in cols] + [None if vv is None else vv.ctypes.data]
    need = L.bt_encode_columns(*ptrs, n, None, 0)
    if need < 0:
        raise ValueError(L.bt_last_error().decode())
    buf = C.create_string_buffer(int(need))
    got = L.bt_encode_columns(*ptrs, n, buf, need)
    if got != need:
        raise ValueError(L.bt_last_error().decode())
    return buf.raw


def gen_payload(seed: int, sym: int, bars: int, freq: int = BT_DAILY) -> bytes:
    """Spec §1 synthetic symbol as a payload, generated on the host (bit-identical to
    Engine.load_synthetic)."""
    L = lib()
    need = L.bt_gen_payload(seed, sym, bars, freq, None, 0)
    if need < 0:
        raise ValueError(L.bt_last_error().decode())
    buf = C.create_string_buffer(int(need))
    if L.bt_gen_payload(seed, sym, bars, freq, buf, need) != need:
        raise ValueError(L.bt_last_error().decode())
    return buf.raw


def decode_columns(data: bytes):
    """Payload bytes -> (open, high, low, close, volume or None) numpy views (no validation;
    the engine's bt_parse_job validates)."""
    if data[:8] != MAGIC:
        raise ValueError("not a DBXCOL1 payload")
    n, flags = np.frombuffer(data, np.uint32, 2, 8)
    n = int(n)
    cols = np.frombuffer(data, np.int32, 4 * n, 16).reshape(4, n)
    v = np.frombuffer(data, np.int64, n, 16 + 16 * n) if flags & 1 else None
    return cols[0], cols[1], cols[2], cols[3], v


def _parse_csv_full(text: bytes):
    """CSV -> int32 open/high/low/close ticks (exact decimal parse, spec §2) and int64 volume."""
    o, h, lo, c, v = [], [], [], [], []
    lines = text.split(b"\n")
    start = 1 if lines and lines[0][:1] and not lines[0][:1].isdigit() else 0
    for ln in lines[start:]:
        ln = ln.strip(b"\r")
        if not ln:
            continue
        f = ln.split(b",")
        px = []
        for x in f[1:5]:
            w, _, fr = x.partition(b".")
            if len(fr) > 4:
                raise ValueError("more than 4 decimals")
            px.append(int(w) * 10000 + int((fr + b"0000")[:4]))
        o.append(px[0]); h.append(px[1]); lo.append(px[2]); c.append(px[3])
        v.append(int(float(f[5])) if len(f) > 5 else 0)
    return o, h, lo, c, v


def csv_to_payload(text: bytes) -> bytes:
    o, h, lo, c, v = _parse_csv_full(text)
    return encode_columns(o, h, lo, c, v)


def main(argv=None):
    ap = argparse.ArgumentParser(description="binary columnar Job.File payloads")
    sub = ap.add_subparsers(dest="cmd", required=True)
    g = sub.add_parser("gen", help="write synthetic symbols (spec §1) as payload files")
    g.add_argument("outdir")
    g.add_argument("--symbols", type=int, default=16)
    g.add_argument("--first", type=int, default=0)
    g.add_argument("--bars", type=int, default=2520)
    g.add_argument("--freq", choices=["daily", "minute"], default="daily")
    g.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED)
    cv = sub.add_parser("csv2bin", help="convert one CSV file")
    cv.add_argument("src")
    cv.add_argument("dst")
    a = ap.parse_args(argv)
    if a.cmd == "gen":
        os.makedirs(a.outdir, exist_ok=True)
        freq = BT_DAILY if a.freq == "daily" else BT_MINUTE
        for s in range(a.first, a.first + a.symbols):
            with open(os.path.join(a.outdir, f"SYM{s:05d}.dbxcol"), "wb") as f:
                f.write(gen_payload(a.seed, s, a.bars, freq))
    else:
        with open(a.src, "rb") as f:
            data = csv_to_payload(f.read())
        with open(a.dst, "wb") as f:
            f.write(data)


if __name__ == "__main__":
    main()
