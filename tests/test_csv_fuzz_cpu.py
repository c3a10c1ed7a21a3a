"""Property tests of the host ingest (docs/oracle_spec.md §2) on the CPU:
the engine's CSV / DBXCOL1 parser (csv.cpp, payload.cpp through bt_parse_job) against a plain
Python statement of the same grammar on generated files mixing valid and malformed rows, and
random corruption of valid payloads (the parser must reject cleanly, never crash)."""
import re

import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import oracle_np as N
from dbx_amd import engine as E
from dbx_amd import payload as PL

_PRICE = re.compile(rb"^([0-9]+)(?:\.([0-9]*))?$")
_TS = re.compile(rb"^[0-9]{4}-[0-9]{2}-[0-9]{2}(?:[ T][0-9:.+\-Z]+)?$")
_VOL = re.compile(rb"^[0-9]+(?:\.[0-9]*)?$")


def ref_parse(buf: bytes):
    """Spec §2 grammar: optional header (first byte not a digit), LF or CRLF rows, blank rows
    skipped, `ts,o,h,l,c[,v]`, prices digits[.digits] with <= 4 fraction digits as exact ticks in
    [1, 2^31), at least one row, |c_t - c_(t-1)| <= c_(t-1). Returns (h, l, c) or None."""
    lines = buf.split(b"\n")
    if buf and not buf[:1].isdigit():
        lines = lines[1:]
    h, lo, c = [], [], []
    for ln in lines:
        if ln.endswith(b"\r"):
            ln = ln[:-1]
        if not ln:
            continue
        f = ln.split(b",")
        if len(f) not in (5, 6) or not _TS.match(f[0]):
            return None
        px = []
        for tok in f[1:5]:
            m = _PRICE.match(tok)
            if not m or len(m.group(2) or b"") > 4:
                return None
            t = int(m.group(1)) * 10000 + int((m.group(2) or b"").ljust(4, b"0") or b"0")
            if t < 1 or t >= 2 ** 31:
                return None
            px.append(t)
        if len(f) == 6 and not _VOL.match(f[5]):
            return None
        h.append(px[1])
        lo.append(px[2])
        c.append(px[3])
    if not c:
        return None
    for a, b in zip(c, c[1:]):
        if abs(b - a) > a:
            return None
    return h, lo, c


def _px(t: int, style: int) -> str:
    whole, frac = divmod(t, 10000)
    s = f"{frac:04d}"
    if style == 0:
        return f"{whole}.{s}"
    s = s.rstrip("0")
    if style == 1 and s:
        return f"{whole}.{s}"
    return f"{whole}.{s}" if s else (f"{whole}" if style == 2 else f"{whole}.")


_good_price = st.integers(1, 2 ** 31 - 1)
_bad_token = st.sampled_from(["", "-1", "1e3", "12.34567", "0", "0.0000", "214748.3648", "abc",
                              " 12", "12 ", "1,2", "999999999"])
_ts = st.sampled_from(["2010-01-04", "2010-01-04 09:30:00", "2010-01-04T09:30:00Z", "2010-1-04",
                       "20100104", "2010-01-04 ", "2010-01-04 x"])


@st.composite
def csv_files(draw):
    n = draw(st.integers(0, 12))
    base = draw(st.integers(2, 2 ** 30))
    rows = []
    for _ in range(n):
        step = draw(st.integers(-base // 2, base // 2))
        base = max(1, min(2 ** 31 - 1, base + step))
        vals = [draw(st.one_of(st.just(base), _good_price)) for _ in range(4)]
        vals[3] = base
        toks = [_px(v, draw(st.integers(0, 3))) for v in vals]
        if draw(st.integers(0, 9)) == 0:
            toks[draw(st.integers(0, 3))] = draw(_bad_token)
        ts = draw(_ts) if draw(st.integers(0, 7)) == 0 else "2011-02-03"
        fields = [ts] + toks
        if draw(st.booleans()):
            fields.append(draw(st.sampled_from(["1000", "12.5", "7.", "x", ""])))
        if draw(st.integers(0, 15)) == 0:
            fields = fields[:draw(st.integers(1, 4))]
        rows.append(",".join(fields))
        if draw(st.integers(0, 10)) == 0:
            rows.append("")
    eol = draw(st.sampled_from(["\n", "\r\n"]))
    head = draw(st.sampled_from(["", "timestamp,open,high,low,close,volume" + eol, "t,o,h,l,c" + eol]))
    tail = eol if draw(st.booleans()) else ""
    return (head + eol.join(rows) + tail).encode()


def _engine_parse(buf: bytes):
    try:
        h, lo, c = E.parse_csv(buf)
    except ValueError:
        return None
    return [[int(x) for x in col] for col in (h, lo, c)]


@settings(max_examples=400, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(csv_files())
def test_csv_parser_matches_grammar(buf):
    want = ref_parse(buf)
    got = _engine_parse(buf)
    assert (got is None) == (want is None), buf
    if want is not None:
        assert got == [list(x) for x in want]


@settings(max_examples=300, deadline=None)
@given(st.integers(0, 2 ** 32 - 1), st.lists(st.tuples(st.integers(0, 10 ** 6), st.integers(0, 255)),
                                               min_size=1, max_size=6),
       st.booleans(), st.integers(0, 40))
def test_corrupted_payloads_are_rejected_or_parsed_never_crash(seed, edits, binary, cut):
    o, h, lo, c, v = N.gen(seed % 1000, [seed % 97], 60, 0)
    blob = bytearray(PL.encode_columns(o[0], h[0], lo[0], c[0]) if binary else
                     N.csv_bytes(o[0], h[0], lo[0], c[0], v[0], 0))
    for pos, val in edits:
        blob[pos % len(blob)] = val
    if cut:
        del blob[len(blob) - cut:]
    got = _engine_parse(bytes(blob))
    if got is not None:  # whatever is accepted satisfies the spec's invariants
        hh, ll, cc = (np.asarray(x, np.int64) for x in got)
        assert len(cc) >= 1 and (cc >= 1).all() and (cc < 2 ** 31).all()
        assert (np.abs(np.diff(cc)) <= cc[:-1]).all()
        if not binary:
            assert ref_parse(bytes(blob)) is not None
