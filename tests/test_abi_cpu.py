"""CPU-side checks of the C ABI (include/bt.h): the library loads, exports every declared
symbol, its host helpers are right, and it fails loudly (no CPU fallback) without a GPU."""
import ctypes as C
import json
import os
import random
import re
import subprocess

import numpy as np
import pytest

import dbx_amd as D
from dbx_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    text = open(os.path.join(ROOT, "include", "bt.h")).read()
    return sorted(set(re.findall(r"\b(bt_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(E.LIB_PATH)
    names = _declared_symbols()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", E.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (bt_[a-z0-9_]+)$", out, re.M))
    assert set(names) <= exported


def test_library_targets_gfx950_only():
    blob = open(E.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}


def test_abi_version_and_no_gpu_failure():
    hdr = open(os.path.join(ROOT, "include", "bt.h")).read()
    want = int(re.search(r"#define BT_ABI_VERSION (\d+)", hdr).group(1))
    # the header, the wrapper (and so __graft_entry__.build()'s check) and the library agree
    assert D.lib().bt_abi_version() == D.ABI_VERSION == want
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(D.BtError, match="device|HIP"):
        D.Engine(D.config2_grid())
    # SMA grids of any window product are accepted (ties settle in int64, k_sma.hip): validation
    # passes and only the missing GPU stops engine creation
    with pytest.raises(D.BtError, match="device|HIP"):
        D.Engine(D.Grid.sma([600, 4096], [4096, 4000]))


def test_late_symbols_check_the_library_abi(monkeypatch):
    # every late entry point binds on the current library ...
    for name in E._LATE_SYMBOLS:
        assert E.sym(name) is not None
    # ... and a library older than a symbol's signature is refused, not bound with shifted
    # arguments (bt_exchange_merge gained block_bytes in ABI 3)
    monkeypatch.setattr(E, "_late", {})
    min_abi, args, res = E._LATE_SYMBOLS["bt_exchange_merge"]
    monkeypatch.setitem(E._LATE_SYMBOLS, "bt_exchange_merge", (D.ABI_VERSION + 1, args, res))
    with pytest.raises(D.BtError, match="needs ABI"):
        E.sym("bt_exchange_merge")


def test_config_validation():
    with pytest.raises(D.BtError, match="empty axis"):
        D.Engine(D.Grid.sma([], [10]))
    with pytest.raises(D.BtError, match="annualization"):
        D.Engine(D.Grid.sma([2], [10], annualization=0))
    # per-symbol prefix rings live in LDS: windows beyond a CU's 160 KB are refused up front
    with pytest.raises(D.BtError, match="LDS"):
        D.Engine(D.Grid.boll([8000], [2], [50], [50]))
    with pytest.raises(D.BtError, match="spans"):
        D.Engine(D.Grid.ema_ols(list(range(2, 70)), [10]))
    with pytest.raises(D.BtError, match="sl_bps"):
        D.Engine(D.Grid.boll([20], [2], [10000], [50]))


def test_i128_to_double_round_to_nearest_even():
    rng = random.Random(5)
    cases = [0, 1, -1, 2**53, 2**53 + 1, 2**53 + 3, -(2**53 + 1), 2**64 - 1, 2**100 + 2**47,
             2**100 + 2**47 + 1, -(2**127), 2**127 - 1, 3 << 70]
    cases += [rng.getrandbits(rng.randint(1, 126)) * rng.choice([1, -1]) for _ in range(2000)]
    for x in cases:
        lo, hi = x & (2**64 - 1), x >> 64
        assert E.i128_to_double(lo, hi) == float(x), x


def test_product_csv_parser_matches_golden(golden_dir):
    g = json.load(open(os.path.join(golden_dir, "csv.json")))
    for key in ("daily", "minute"):
        h, lo, c = E.parse_csv(g[key]["text"].encode())
        assert c.tolist() == g[key]["c"] and h.tolist() == g[key]["h"] and lo.tolist() == g[key]["l"]
    for name, case in g["good"].items():
        h, lo, c = E.parse_csv(case["text"].encode())
        assert c.tolist() == case["c"], name
    for name, text in g["bad"].items():
        with pytest.raises(ValueError):
            E.parse_csv(text.encode())


def test_product_csv_parser_matches_oracle_on_synthetic_files():
    import oracle_np as N
    import orc_ffi as F
    for sym, bars, freq in [(0, 300, 0), (5, 1000, 1)]:
        o, h, lo, c, v = N.gen(9, [sym], bars, freq)
        text = N.csv_bytes(o[0], h[0], lo[0], c[0], v[0], freq)
        ph, pl, pc = E.parse_csv(text)
        fo, fh, fl, fc, fv = F.parse_csv(text)
        assert np.array_equal(ph, fh) and np.array_equal(pl, fl) and np.array_equal(pc, fc)


def test_merge_topk_order():
    rng = np.random.default_rng(0)
    recs = np.zeros(500, D.TOPK_DTYPE)
    recs["sharpe"] = rng.choice([0.5, 1.0, -2.0, 3.25], 500)
    recs["sym"] = rng.integers(0, 50, 500)
    recs["param"] = rng.integers(0, 400, 500)
    got = D.merge_topk(recs, 40)
    exp = sorted(recs.tolist(), key=lambda r: (-r[0], r[1], r[2]))[:40]
    assert [tuple(r) for r in got.tolist()] == [tuple(r) for r in exp]
    assert len(D.merge_topk(recs[:0], 5)) == 0


def test_release_library_reads_no_environment():
    """The release libbt.so has no profiling switches: phase ablation (BT_ABLATE), s_memtime
    stamps and launch overrides exist only in dev/prof.so (`make PROFILING=1`), so no stray
    environment variable in a worker can change a backtest result."""
    blob = open(E.LIB_PATH, "rb").read()
    for name in (b"BT_ABLATE", b"BT_PW", b"BT_XW", b"BT_LPW", b"BT_ONE_TRIP"):
        assert name not in blob, name
    out = subprocess.run(["nm", "-D", "--undefined-only", E.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert not re.search(r"\bgetenv\b", out)


def test_result_lines_match_printf_format():
    """bt_run_batch's CompleteRequest.data lines (std::to_chars) are byte-identical to the spec §6
    printf format: "%.17g" Sharpe, "%016x" hash, decimal integers."""
    rng = np.random.default_rng(7)
    n = 3000
    rows = np.zeros(n, D.SUMMARY_DTYPE)
    rows["n_trades"] = rng.integers(0, 2**31 - 1, n)
    rows["pnl"] = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
    rows["mdd"] = rng.integers(0, 2**63 - 1, n, dtype=np.int64)
    rows["exposure"] = rng.integers(0, 2**22, n)
    sh = rng.standard_normal(n) * 10.0 ** rng.integers(-300, 300, n)
    sh[:8] = [0.0, -0.0, 1.0, -1.5, 1e-320, 5e-324, 1.7976931348623157e308, 0.1]
    rows["sharpe"] = sh
    rows["hash"] = rng.integers(0, 2**63, n, dtype=np.uint64) * 2 + rng.integers(0, 2, n).astype(np.uint64)
    rows["hash"][0] = 0
    got = E.format_summaries(rows).split("\n")
    assert got[-1] == "" and len(got) == n + 1
    for p, (r, line) in enumerate(zip(rows, got)):
        exp = ('{"param":%d,"n":%d,"pnl":%d,"mdd":%d,"exp":%d,"sharpe":"%.17g","h":"%016x"}'
               % (p, r["n_trades"], r["pnl"], r["mdd"], r["exposure"], r["sharpe"], r["hash"]))
        assert line == exp, (p, line, exp)
        assert json.loads(line)["param"] == p


def build_abi_host(tmpdir):
    """tests/abi_host.c — a compiled C99 host of include/bt.h (what a Rust / C worker links):
    built with -std=c99 -pedantic -Werror against the in-tree libbt.so."""
    exe = os.path.join(str(tmpdir), "abi_host")
    lib_dir = os.path.dirname(E.LIB_PATH)
    r = subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "abi_host.c"),
                        "-L", lib_dir, "-l:" + os.path.basename(E.LIB_PATH),
                        "-Wl,-rpath," + lib_dir, "-Wl,-rpath-link,/opt/rocm/lib", "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c99_host_compiles_and_struct_layouts_match_the_python_mirror(tmp_path):
    """bt.h is plain C99 (a Rust / C host binds it as is), and every struct the Python mirror
    (engine.py ctypes classes and numpy dtypes) reads has the header's size and offsets."""
    exe = build_abi_host(tmp_path)
    got = json.loads(subprocess.run([exe, "layout"], capture_output=True, text=True, check=True).stdout)
    assert got["abi_version"] == 3
    mirror = {"bt_config": E._Config, "bt_job_in": E._JobIn, "bt_job_out": E._JobOut,
              "bt_batch_profile": E._BatchProfile, "bt_stats": E._Stats}
    for cname, cls in mirror.items():
        assert got[cname] == C.sizeof(cls), cname
        for f, _ in cls._fields_:
            key = f"{cname}.{f}"
            if key in got:
                assert got[key] == getattr(cls, f).offset, key
    dtypes = {"bt_summary": E.SUMMARY_DTYPE, "bt_trade": E.TRADE_DTYPE, "bt_sums": E.SUMS_DTYPE,
              "bt_topk_rec": E.TOPK_DTYPE}
    for cname, dt in dtypes.items():
        assert got[cname] == dt.itemsize, cname
        for f in dt.names:
            key = f"{cname}.{f}"
            if key in got:
                assert got[key] == dt.fields[f][1], key
    checked = [k for k in got if "." in k]
    assert len(checked) >= 30
