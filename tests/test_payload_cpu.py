"""Binary columnar Job.File payload: codec, host generator and the
engine's ingest, on the CPU (no GPU calls). The C oracle is the checker."""
import numpy as np
import pytest

import dbx_amd as D
import orc_ffi as F
import oracle_np as N
from dbx_amd import engine as E
from dbx_amd import payload as PL


@pytest.mark.parametrize("freq,bars", [(0, 2520), (1, 5000), (0, 1)])
def test_host_generator_matches_oracle(freq, bars):
    for sym in (0, 7, 4999):
        o, h, lo, c, v = PL.decode_columns(PL.gen_payload(0x5EED, sym, bars, freq))
        eo, eh, el, ec, ev = F.gen(0x5EED, sym, bars, freq)
        for got, exp in ((o, eo), (h, eh), (lo, el), (c, ec)):
            assert np.array_equal(got, exp)
        _, _, _, _, nv = N.gen(0x5EED, [sym], bars, freq)
        assert np.array_equal(v, nv[0])


def test_binary_and_csv_ingest_agree():
    o, h, lo, c, v = N.gen(0x5EED, [3], 3000, 1)
    text = N.csv_bytes(o[0], h[0], lo[0], c[0], v[0], 1)
    blob = PL.csv_to_payload(text)
    assert blob[:8] == PL.MAGIC and len(blob) == 16 + 3000 * 24
    a = E.parse_csv(text)
    b = E.parse_csv(blob)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert np.array_equal(b[2], c[0])
    # without the volume column
    blob2 = PL.encode_columns(o[0], h[0], lo[0], c[0])
    assert len(blob2) == 16 + 3000 * 16
    assert np.array_equal(E.parse_csv(blob2)[2], c[0])


@pytest.mark.parametrize("mutate,msg", [
    (lambda b: b[:-1], "length"),
    (lambda b: b[:8] + (0).to_bytes(4, "little") + b[12:], "bar count"),
    (lambda b: b[:12] + (6).to_bytes(4, "little") + b[16:], "flags"),
    (lambda b: b[:16 + 4 * 100 * 3 + 8] + (0).to_bytes(4, "little") + b[16 + 4 * 100 * 3 + 12:], "price"),
    (lambda b: b[:16 + 4 * 100 * 3 + 40] + (2 ** 31 - 1).to_bytes(4, "little") + b[16 + 4 * 100 * 3 + 44:], "100%"),
])
def test_binary_payload_rejects_malformed(mutate, msg):
    o, h, lo, c, _v = N.gen(1, [0], 100, 0)
    blob = PL.encode_columns(o[0], h[0], lo[0], c[0])
    with pytest.raises(ValueError, match=msg):
        E.parse_csv(mutate(blob))


def test_payload_cli_gen(tmp_path):
    PL.main(["gen", str(tmp_path), "--symbols", "3", "--first", "10", "--bars", "500",
             "--freq", "minute"])
    files = sorted(tmp_path.iterdir())
    assert [f.name for f in files] == ["SYM00010.dbxcol", "SYM00011.dbxcol", "SYM00012.dbxcol"]
    c = PL.decode_columns(files[1].read_bytes())[3]
    assert np.array_equal(c, F.gen(0x5EED, 11, 500, 1)[3])
