"""bench.py — bar-evals/s of the backtest hot path on 1..N MI355X (BASELINE.json metric).

Default workload (N=1 and per GPU for N>1): BASELINE config 2 — SMA fast/slow crossover,
5,000 symbols x 2,520 daily bars x 400 param pairs, synthetic OHLC (docs/oracle_spec.md §1)
generated directly in HBM before timing. One step = one pass of the hot path over that batch:
the fused strategy kernel (indicators + signals + position/PnL/drawdown/Sharpe per lane), the
per-GPU top-k and its read-back; for N>1 also one RCCL all-gather of every rank's top-k records
and counters (the only exchange step). Step i+1 is enqueued before step i's
read-back/exchange is consumed, so host work and the collective overlap the next pass. Symbols
are sharded across ranks with no data-path collective (weak scaling: every rank runs its own
shard).

`--config 3|4|5` measures the per-GPU shard of the other BASELINE configs the same way (EMA+OLS
500 x 98,280 x 64; Bollinger 500 x 98,280 x 256, i.e. 2,000 symbols over 4 GPUs; SMA
1,250 x 491,400 x 1,024, i.e. 10,000 symbols over 8 GPUs); the driver runs the default.

Run: python bench.py [--gpus N --steps K --warmup W] [--config C]
     torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import dbx_amd as D  # noqa: E402
from dbx_amd import parallel as PAR  # noqa: E402

SEED, TOPK = 0x5EED, 100
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue ceiling: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction
# (MI355X_MICROARCH.md per-instruction constants: v_fma_f32 wave64 = 2 cycles on SIMD-32)
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2

# per-GPU shard of each BASELINE config: grid, symbols, bars, bar frequency, annualization,
# and the SURVEY.md §8(d) byte-model terms c (OHLC columns consumed) and W (indicator series)
CONFIGS = {
    2: dict(grid=D.config2_grid, S=5000, B=2520, freq=D.BT_DAILY, ann=252, c=1, W=40,
            name="BASELINE config 2: SMA fast/slow crossover"),
    3: dict(grid=D.config3_grid, S=500, B=98280, freq=D.BT_MINUTE, ann=98280, c=1, W=16,
            name="BASELINE config 3: EMA + rolling-OLS-slope mean reversion"),
    4: dict(grid=D.config4_grid, S=500, B=98280, freq=D.BT_MINUTE, ann=98280, c=3, W=16,
            name="BASELINE config 4: Bollinger z-score with SL/TP (2,000 symbols over 4 GPUs)"),
    5: dict(grid=D.config5_grid, S=1250, B=491400, freq=D.BT_MINUTE, ann=98280, c=1, W=64,
            name="BASELINE config 5: SMA 32x32 grid, 5y 1-min bars (10,000 symbols over 8 GPUs)"),
}


def algorithmic_bytes(S, B, P, c=1, W=40):
    """SURVEY.md §8(d) pinned byte model: B_alg = S*B*(8c + 16W) + 32*S*P."""
    return S * B * (8 * c + 16 * W) + 32 * S * P


def cpu_baseline(cfg, grid, threads=None, target_thread_s=25.0):
    """The C oracle (oracle/oracle.c, -O2 -ffp-contract=off) on the first symbols of
    the same workload, sized from a one-symbol probe to ~target_thread_s thread-seconds. SMA
    grids run on the oracle's pthread grid (one symbol per thread); EMA/Bollinger run one
    (symbol, param) call per task on a thread pool (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc_ffi as F
    threads = threads or min(16, os.cpu_count() or 1)
    B, freq, ann = cfg["B"], 1 if cfg["freq"] == D.BT_MINUTE else 0, cfg["ann"]

    def run(n):
        cols = [F.gen(SEED, s, B, freq) for s in range(n)]
        t0 = time.perf_counter()
        if grid.strategy == D.BT_SMA_CROSS:
            F.sma_grid_mt(np.stack([x[3] for x in cols]), np.asarray(grid.axes[0]),
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
                list(ex.map(one, [(s, p) for s in range(n) for p in range(grid.n_params)]))
        return time.perf_counter() - t0

    probe = min(threads, cfg["S"]) if grid.strategy == D.BT_SMA_CROSS else 1
    dt = run(probe)
    thread_s = dt * (threads if grid.strategy != D.BT_SMA_CROSS else min(threads, probe))
    per_sym = thread_s / probe
    n_sym = int(min(cfg["S"], max(probe, target_thread_s / max(per_sym, 1e-9))))
    if n_sym > probe:
        dt = run(n_sym)
    else:
        n_sym = probe
    evals = n_sym * B * grid.n_params
    return {"value": evals / dt, "unit": "bar-evals/s", "cores": threads, "kind": "port",
            "sample": f"first {n_sym} of the {cfg['S']} shard symbols x {B} bars x "
                      f"{grid.n_params} params ({evals:.3g} bar-evals, {dt:.2f} s wall = "
                      f"{dt * threads:.1f} thread-s on {threads} threads; oracle/oracle.c, gcc -O2 -ffp-contract=off)"}


def load_traffic(config):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summaries."""
    path = os.path.join(ROOT, "profiles", "pmc_sma_config2.json") if config == 2 else \
        os.path.join(ROOT, "profiles", "r01_configs", "configs.json")
    try:
        d = json.load(open(path))
        if config == 2:
            return float(d["hbm_bytes_per_launch"])
        v = d[f"config{config}"]
        return float(v["hbm_read_bytes"] + v["hbm_write_bytes"])
    except Exception:
        return None


def load_valu_insts(config):
    """VALU wave-instructions per launch of the dominant kernel (PMC SQ_INSTS_VALU) from the
    committed rocprofv3 summaries: the kernels are VALU-issue bound, not HBM bound."""
    try:
        if config == 2:
            d = json.load(open(os.path.join(ROOT, "profiles", "r01", "pmc_summary.json")))
            return float(d["sq"]["SQ_INSTS_VALU"])
        d = json.load(open(os.path.join(ROOT, "profiles", "r01_configs", "configs.json")))
        return float(d[f"config{config}"]["pmc"]["SQ_INSTS_VALU"])
    except Exception:
        return None


def valu_issue(insts, kernel_s):
    if insts is None:
        return None
    achieved = insts / kernel_s / 1e9
    return {"insts_per_launch": insts, "achieved": achieved, "peak": VALU_PEAK_GINST,
            "unit": "Ginst/s", "frac": achieved / VALU_PEAK_GINST}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    S_PER_GPU, BARS = cfg["S"], cfg["B"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local
    if world > 1:
        import torch
        import torch.distributed as dist
        # one process per GPU; ranks outnumbering the visible GPUs (a rehearsal on a 1-GPU box)
        # share devices, and RCCL needs distinct devices, so the k x 24 B exchange then uses gloo
        ndev = torch.cuda.device_count()
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        device = local % max(ndev, 1)
        torch.cuda.set_device(device)
        if ndev >= local_world:
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")

    grid = cfg["grid"]()
    P = grid.n_params
    eng = D.Engine(grid, device=device, topk=TOPK, timing=True)
    eng.load_synthetic(SEED, rank * S_PER_GPU, S_PER_GPU, BARS, cfg["freq"])

    def issue(i):
        eng.run()                      # kernels of step i, enqueued on the engine stream
        eng.topk_fetch_async(i & 1)    # its top-k + trade count into pinned slot i % 2

    def finish(i):
        top, trades = eng.topk_fetch_wait(i & 1)
        if dist is None:
            return top
        # the one exchange step: a single RCCL all-gather carrying each rank's k x 24 B top-k
        # records and its run counters (summed on the host)
        top, _ = PAR.exchange(top, TOPK, [S_PER_GPU * BARS * P, trades], dist)
        return top

    def steps(n):
        """n steps; step i+1 is enqueued before step i's read-back and exchange, so the GPU runs
        the next pass while the host consumes (and, for N > 1, exchanges) this one."""
        top = None
        if n > 0:
            issue(0)
        for i in range(n):
            if i + 1 < n:
                issue(i + 1)
            top = finish(i)
        return top

    steps(args.warmup)
    eng.sync()
    eng.reset_timing()
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    top = steps(args.steps)
    eng.sync()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64,
                          device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    kms, launches, kname = eng.kernel_timing()
    stats = eng.stats()

    if rank == 0:
        evals_per_step = S_PER_GPU * BARS * P * world
        value = evals_per_step * args.steps / elapsed
        kavg_s = kms / 1e3 / max(launches, 1)
        alg = algorithmic_bytes(S_PER_GPU, BARS, P, cfg["c"], cfg["W"])
        achieved = alg / kavg_s / 1e9
        traffic = load_traffic(args.config)
        line = {
            "metric": "bar-evals/sec (symbols x params x bars)",
            "value": value,
            "unit": "bar-evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64+int64",
            "data": "synthetic (SplitMix64 integer OHLC walk, docs/oracle_spec.md §1, generated in HBM)",
            "config": {"workload": cfg["name"],
                       "symbols_per_gpu": S_PER_GPU, "bars": BARS, "params": P,
                       "topk": TOPK, "parallelism": f"dp{world} (symbol shards, "
                       f"{'RCCL' if dist is None or dist.get_backend() == 'nccl' else 'gloo'} top-k gather)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel": kname, "kernel_avg_ms": kavg_s * 1e3,
                         "alg_bytes_per_launch": alg},
            # the bound that actually limits the fused kernels: VALU issue (PMC instruction
            # count per launch from profiles/, over the live kernel time)
            "valu_issue": valu_issue(load_valu_insts(args.config), kavg_s),
            "trades_per_step": stats["trades"],
            "top1": {"sharpe": float(top[0]["sharpe"]), "sym": int(top[0]["sym"]),
                     "param": int(top[0]["param"])} if len(top) else None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, grid)
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
