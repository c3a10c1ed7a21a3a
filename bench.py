"""bench.py — bar-evals/s of the backtest hot path on 1..N MI355X (BASELINE.json metric).

Workload (N=1 and per GPU for N>1): BASELINE config 2 — SMA fast/slow crossover,
5,000 symbols x 2,520 daily bars x 400 param pairs, synthetic OHLC (docs/oracle_spec.md §1)
generated directly in HBM before timing. One step = one pass of the hot path over that batch:
the fused SMA kernel (indicators + signals + position/PnL/drawdown/Sharpe per lane) and the
per-GPU top-k; for N>1 also the RCCL all-gather of the top-k records + all-reduce of counters
(the only exchange step). Symbols are sharded across ranks with no data-path
collective (weak scaling: every rank runs its own 5,000 symbols).

Run: python bench.py [--gpus N --steps K --warmup W]
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

S_PER_GPU, BARS, SEED, TOPK = 5000, 2520, 0x5EED, 100
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(S, B, P, c=1, W=40):
    """SURVEY.md §8(d) pinned byte model: B_alg = S*B*(8c + 16W) + 32*S*P."""
    return S * B * (8 * c + 16 * W) + 32 * S * P


def cpu_baseline(grid, threads=None, target_cpu_s=15.0):
    """The C oracle (scalar, multithreaded: SURVEY B4) on a bounded sample of the same workload:
    a 64-symbol probe sizes the sample to ~target_cpu_s thread-seconds (at most all 5,000)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc_ffi as F
    threads = threads or min(16, os.cpu_count() or 1)
    fast, slow = np.asarray(grid.axes[0]), np.asarray(grid.axes[1])

    def timed(n):
        closes = np.stack([F.gen(SEED, s, BARS, 0)[3] for s in range(n)])
        t0 = time.perf_counter()
        F.sma_grid_mt(closes, fast, slow, 252, threads)
        return time.perf_counter() - t0

    probe = 64
    dt = timed(probe)
    n_sym = int(min(S_PER_GPU, max(probe, probe * target_cpu_s / threads / max(dt, 1e-6))))
    if n_sym > probe:
        dt = timed(n_sym)
    else:
        n_sym = probe
    evals = n_sym * BARS * grid.n_params
    return {"value": evals / dt, "unit": "bar-evals/s", "cores": threads, "kind": "port",
            "sample": f"first {n_sym} of the 5000 config-2 symbols x {BARS} bars x "
                      f"{grid.n_params} params ({evals:.3g} bar-evals, {dt:.2f} s wall on "
                      f"{threads} threads = {dt * threads:.1f} thread-s; oracle/oracle.c "
                      f"orc_sma_grid_mt, gcc -O2 -ffp-contract=off)"}


def load_traffic():
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary."""
    path = os.path.join(ROOT, "profiles", "pmc_sma_config2.json")
    if not os.path.exists(path):
        return None
    try:
        return float(json.load(open(path))["hbm_bytes_per_launch"])
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

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

    grid = D.config2_grid()
    P = grid.n_params
    eng = D.Engine(grid, device=device, topk=TOPK, timing=True)
    eng.load_synthetic(SEED, rank * S_PER_GPU, S_PER_GPU, BARS, D.BT_DAILY)

    def step():
        eng.run()
        top = eng.read_topk()          # syncs the engine stream
        if dist is None:
            return top
        # the one exchange step: RCCL all-gather of k x 24 B per rank + counter all-reduce
        top = PAR.gather_topk(top, TOPK, dist)
        PAR.allreduce_counters([S_PER_GPU * BARS * P, eng.stats()["trades"]], dist)
        return top

    for _ in range(args.warmup):
        step()
    eng.sync()
    eng.reset_timing()
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        top = step()
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
        alg = algorithmic_bytes(S_PER_GPU, BARS, P)
        achieved = alg / kavg_s / 1e9
        traffic = load_traffic()
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
            "config": {"workload": "BASELINE config 2: SMA fast/slow crossover",
                       "symbols_per_gpu": S_PER_GPU, "bars": BARS, "params": P,
                       "topk": TOPK, "parallelism": f"dp{world} (symbol shards, "
                       f"{'RCCL' if dist is None or dist.get_backend() == 'nccl' else 'gloo'} top-k gather)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel": kname, "kernel_avg_ms": kavg_s * 1e3,
                         "alg_bytes_per_launch": alg},
            "trades_per_step": stats["trades"],
            "top1": {"sharpe": float(top[0]["sharpe"]), "sym": int(top[0]["sym"]),
                     "param": int(top[0]["param"])} if len(top) else None,
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(grid)
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
