"""Write tests/golden/*.json from the numpy restatement (oracle/oracle_np.py).

TEST INFRASTRUCTURE. Run: python oracle/make_golden.py   (takes ~1 minute, pure Python)

The reference has no fixtures or golden vectors for this path; these
vectors pin docs/oracle_spec.md. The C oracle and the HIP engine are both checked against
them. Wire-level vectors at the end are the proto pins SURVEY.md §8(c) captured with the
protobuf runtime against /root/reference/proto/backtesting.proto.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import oracle_np as N  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def summ_json(s):
    return {"n": s["n"], "pnl": s["pnl"], "mdd": s["mdd"], "exposure": s["exposure"],
            "s1": str(s["s1"]), "s2": str(s["s2"]), "sharpe": s["sharpe"].hex(),
            "h": f"{s['h']:016x}"}


def series(o, h, lo, c):
    return {"o": [int(x) for x in o], "h": [int(x) for x in h], "l": [int(x) for x in lo],
            "c": [int(x) for x in c]}


def run_cases(strategy, ohlc, plist, ann):
    cases = []
    for p in plist:
        s, tr = N.run(strategy, ohlc, p, ann)
        cases.append({"params": p, "summary": summ_json(s),
                      "trades": [list(map(int, t)) for t in tr]})
    return cases


def main():
    os.makedirs(OUT, exist_ok=True)
    # ---- generator known answers
    gen = []
    for seed, sym, bars, freq in [(0x5EED, 0, 64, 0), (0x5EED, 4999, 64, 0), (0, 1, 32, 1),
                                  (0xFFFFFFFFFFFFFFFF, 123456, 40, 1)]:
        o, h, lo, c, v = N.gen(seed, [sym], bars, freq)
        gen.append({"seed": f"{seed:#x}", "sym": sym, "bars": bars, "freq": freq,
                    **series(o[0], h[0], lo[0], c[0]), "v": [int(x) for x in v[0]]})
    # long-series checksums (whole config-2 row, 1-min row)
    sums = []
    for seed, sym, bars, freq in [(0x5EED, 7, 2520, 0), (0x5EED, 3, 98280, 1)]:
        o, h, lo, c, v = N.gen(seed, [sym], bars, freq)
        sums.append({"seed": f"{seed:#x}", "sym": sym, "bars": bars, "freq": freq,
                     "sum_o": int(o.sum()), "sum_h": int(h.sum()), "sum_l": int(lo.sum()),
                     "sum_c": int(c.sum()), "sum_v": int(v.sum()),
                     "c_last": int(c[0, -1]), "sum_c_sq_mod": int((c.astype(object) ** 2).sum() % (1 << 61))})
    json.dump({"known": gen, "checksums": sums}, open(os.path.join(OUT, "gen.json"), "w"))

    # ---- CSV: bytes -> ticks
    o, h, lo, c, v = N.gen(0x5EED, [42], 12, 0)
    daily = {"text": N.csv_bytes(o[0], h[0], lo[0], c[0], v[0], 0).decode(),
             **series(o[0], h[0], lo[0], c[0])}
    o, h, lo, c, v = N.gen(0x5EED, [43], 8, 1)
    minute = {"text": N.csv_bytes(o[0], h[0], lo[0], c[0], v[0], 1).decode(),
              **series(o[0], h[0], lo[0], c[0])}
    bad = {
        "bad_price_5dp": "timestamp,open,high,low,close,volume\n2010-01-04,1.00001,2,1,1,5\n",
        "bad_fields": "2010-01-04,1,2,1\n",
        "bad_ts": "2010/01/04,1,2,1,1,5\n",
        "zero_price": "2010-01-04,0,2,1,1,5\n",
        "too_big": "2010-01-04,214748.3648,214748.3648,1,1,5\n",
        "empty": "timestamp,open,high,low,close,volume\n",
        "jump": "2010-01-04,1,1,1,1.0000,1\n2010-01-05,3,3,3,3.0000,1\n",
    }
    good_extra = {
        "crlf_no_header_no_vol": ("2010-01-04,1.5,2.25,1.0001,2\r\n2010-01-05T09:30:00Z,2,2,2,2.5\r\n\r\n",
                                  {"o": [15000, 20000], "h": [22500, 20000], "l": [10001, 20000],
                                   "c": [20000, 25000]}),
        "max_price": ("2010-01-04,214748.3647,214748.3647,214748.3647,214748.3647,1\n",
                      {"o": [2147483647], "h": [2147483647], "l": [2147483647], "c": [2147483647]}),
    }
    json.dump({"daily": daily, "minute": minute, "bad": bad,
               "good": {k: {"text": t, **exp} for k, (t, exp) in good_extra.items()}},
              open(os.path.join(OUT, "csv.json"), "w"))

    # ---- strategies on synthetic series
    fixtures = {}
    o, h, lo, c, v = N.gen(0x5EED, [0, 1, 2], 600, 0)
    sma_params = [{"f": f, "s": s} for f in (4, 10, 42) for s in (50, 120, 240)]
    sma_params += [{"f": 20, "s": 20}, {"f": 60, "s": 50}, {"f": 4, "s": 600}, {"f": 4, "s": 601}]
    fixtures["sma_daily"] = {"strategy": "sma", "ann": 252, "symbols": [
        {"seed": "0x5eed", "sym": s, "bars": 600, "freq": 0,
         "cases": run_cases("sma", (o[s], h[s], lo[s], c[s]), sma_params, 252)} for s in range(3)]}

    o, h, lo, c, v = N.gen(0x5EED, [0, 1], 2500, 1)
    ema_params = [{"n": n, "w": w, "band_bps": 20} for n in (10, 60, 390) for w in (15, 120, 780)]
    fixtures["ema_ols_minute"] = {"strategy": "ema_ols", "ann": 98280, "symbols": [
        {"seed": "0x5eed", "sym": s, "bars": 2500, "freq": 1,
         "cases": run_cases("ema_ols", (o[s], h[s], lo[s], c[s]), ema_params, 98280)}
        for s in range(2)]}

    boll_params = [{"w": w, "k_num": k, "k_den": 2, "sl": sl, "tp": tp}
                   for w in (10, 45, 240) for k in (3, 6) for sl in (50, 100) for tp in (50, 400)]
    fixtures["boll_minute"] = {"strategy": "boll", "ann": 98280, "symbols": [
        {"seed": "0x5eed", "sym": s, "bars": 2500, "freq": 1,
         "cases": run_cases("boll", (o[s], h[s], lo[s], c[s]), boll_params, 98280)}
        for s in range(2)]}

    # ---- edge cases on explicit series
    flat = [1_000_000] * 300
    rng = np.random.default_rng(7)
    big = list(np.clip(2**31 - 1 - rng.integers(0, 4000, 300), 1, 2**31 - 1))
    saw = [1_000_000 + (50_000 if (t // 7) % 2 else -50_000) for t in range(300)]
    tiny = [1, 2, 1, 2, 2, 1, 1, 2, 1, 1, 2, 2, 2, 1]
    edge = []
    for name, cl in [("flat", flat), ("near_max", big), ("saw", saw), ("tiny", tiny),
                     ("one_bar", [5_000_000]), ("two_bars", [5_000_000, 5_100_000])]:
        cl = [int(x) for x in cl]
        hh = [min(x + 3, 2**31 - 1) for x in cl]
        ll = [max(x - 3, 1) for x in cl]
        ohlc = (cl, hh, ll, cl)
        edge.append({"name": name, **series(*ohlc),
                     "sma": run_cases("sma", ohlc, [{"f": 2, "s": 5}, {"f": 3, "s": 3},
                                                    {"f": 4, "s": 50}], 252),
                     "ema_ols": run_cases("ema_ols", ohlc, [{"n": 3, "w": 4, "band_bps": 20},
                                                            {"n": 10, "w": 15, "band_bps": 0}], 98280),
                     "boll": run_cases("boll", ohlc, [{"w": 3, "k_num": 1, "k_den": 2, "sl": 50, "tp": 50},
                                                      {"w": 10, "k_num": 3, "k_den": 2, "sl": 100, "tp": 400}],
                                       98280)})
    fixtures["edge"] = edge
    for k, val in fixtures.items():
        json.dump(val, open(os.path.join(OUT, f"{k}.json"), "w"))

    # ---- wire pins (captured with protobuf 7.35.1 runtime descriptors)
    json.dump({
        "JobsRequest{cores=4}": "0804",
        "StatusRequest{RUNNING}": "0801",
        "JobsReply{[Job{id:'abc', File:'t,o,h,l,c,v\\n'}]}":
            "0a130a03616263120c742c6f2c682c6c2c632c760a",
        "grpc_default_max_receive": 4194304,
    }, open(os.path.join(OUT, "wire.json"), "w"), indent=1)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
