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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--symbols", type=int, default=0)
    ap.add_argument("--bars", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
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
    print(json.dumps({"config": a.config, "symbols": S, "bars": B, "params": grid.n_params,
                      "bar_evals_per_s": evals / dt, "ms_per_step": dt * 1e3,
                      "kernel": kname, "kernel_ms": kms / max(nl, 1), "gen_s": tgen,
                      "trades": eng.stats()["trades"],
                      "top1_sharpe": float(top[0]["sharpe"]) if len(top) else None}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
