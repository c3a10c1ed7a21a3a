"""Per-GPU throughput of the other BASELINE configs (3, 4, 5 shards) on HBM-resident synthetic
data — a development aid beside bench.py (which measures config 2, the headline metric).

  python scripts/bench_configs.py --config 3 [--symbols N --bars B --steps K]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbx_amd as D  # noqa: E402

CONFIGS = {  # per-GPU shard: (grid, symbols, bars, freq, seed)
    2: (D.config2_grid, 5000, 2520, D.BT_DAILY),
    3: (D.config3_grid, 500, 98280, D.BT_MINUTE),
    4: (D.config4_grid, 500, 98280, D.BT_MINUTE),      # 2,000 symbols over 4 GPUs
    5: (D.config5_grid, 1250, 491400, D.BT_MINUTE),    # 10,000 symbols over 8 GPUs
}


def cpu_baseline(config, grid, B, max_sym, target_thread_s=15.0):
    """The C oracle (oracle/oracle.c, -O2 -ffp-contract=off) on the first symbols of the same
    workload, one (symbol, param) task per call on a thread pool (ctypes drops the GIL);
    config 5 uses the oracle's pthread grid. Sized to ~target_thread_s thread-seconds."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import numpy as np
    import orc_ffi as F
    threads = min(16, os.cpu_count() or 1)
    freq = 1 if config != 2 else 0
    ann = 98280 if freq else 252

    def run(n_sym):
        cols = [F.gen(0x5EED, s, B, freq) for s in range(n_sym)]
        t0 = time.perf_counter()
        if grid.strategy == D.BT_SMA_CROSS:
            F.sma_grid_mt(np.stack([c[3] for c in cols]), np.asarray(grid.axes[0]),
                          np.asarray(grid.axes[1]), ann, threads)
        else:
            def one(sp):
                s, p = sp
                o, h, lo, c = cols[s][:4]
                kw = grid.param(p)
                if grid.strategy == D.BT_EMA_OLS:
                    F.ema_ols(c, kw["n"], kw["w"], kw["band_bps"], ann)
                else:
                    F.boll(h, lo, c, kw["w"], kw["k_num"], kw["k_den"], kw["sl"], kw["tp"], ann)
            with ThreadPoolExecutor(threads) as ex:
                list(ex.map(one, [(s, p) for s in range(n_sym) for p in range(grid.n_params)]))
        return time.perf_counter() - t0

    n = 1
    dt = run(n)
    # thread-seconds of the probe: the pthread SMA grid runs one symbol per thread, the pool
    # spreads one symbol's parameters over every thread
    probe_ts = dt if grid.strategy == D.BT_SMA_CROSS else dt * threads
    n = max(1, min(max_sym, int(target_thread_s / max(probe_ts, 1e-6))))
    if grid.strategy == D.BT_SMA_CROSS:
        n = max(n, min(max_sym, threads))
    if n > 1:
        dt = run(n)
    ev = n * B * grid.n_params
    return {"value": ev / dt, "unit": "bar-evals/s", "cores": threads, "kind": "port",
            "sample": f"first {n} symbols x {B} bars x {grid.n_params} params, {dt:.2f} s wall "
                      f"on {threads} threads (oracle/oracle.c)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--symbols", type=int, default=0)
    ap.add_argument("--bars", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-baseline", action="store_true",
                    help="also time the C oracle on a bounded sample (host threads)")
    a = ap.parse_args()
    gridf, S, B, freq = CONFIGS[a.config]
    S = a.symbols or S
    B = a.bars or B
    grid = gridf()
    eng = D.Engine(grid, topk=100, timing=True)
    t0 = time.perf_counter()
    eng.load_synthetic(0x5EED, 0, S, B, freq)
    eng.sync()
    tgen = time.perf_counter() - t0
    for _ in range(a.warmup):
        eng.run()
        eng.read_topk()
    eng.sync()
    eng.reset_timing()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.run()
        top = eng.read_topk()
    eng.sync()
    dt = (time.perf_counter() - t0) / a.steps
    kms, nl, kname = eng.kernel_timing()
    evals = S * B * grid.n_params
    cpu = cpu_baseline(a.config, grid, B, S) if a.cpu_baseline else None
    print(json.dumps({"cpu_baseline": cpu,"config": a.config, "symbols": S, "bars": B, "params": grid.n_params,
                      "bar_evals_per_s": evals / dt, "ms_per_step": dt * 1e3,
                      "kernel": kname, "kernel_ms": kms / max(nl, 1), "gen_s": tgen,
                      "trades": eng.stats()["trades"],
                      "top1_sharpe": float(top[0]["sharpe"]) if len(top) else None}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
