"""bench.py — bar-evals/s of the backtest hot path on 1..N MI355X (BASELINE.json metric).

Default workload (the driver's line): BASELINE config 2 — SMA fast/slow crossover, 5,000 symbols
x 2,520 daily bars x 400 param pairs per GPU (weak scaling: config 2 is a one-GPU config, so N
GPUs run N such shards), synthetic OHLC (docs/oracle_spec.md §1) generated directly in HBM
before timing. One step = one pass of the hot path over that batch: the fused strategy kernel
(indicators + signals + position/PnL/drawdown/Sharpe per lane), the per-GPU top-k and its
read-back; for N > 1 also the exchange step: ONE RCCL all-gather of every
rank's top-k records and counters, issued through the C ABI (bt_exchange_async, csrc/comm.cpp)
straight from the engine's device buffers. Step i+1 (at N > 1 also step i+2) is enqueued before
step i's read-back / exchange is consumed, so host work and the collective overlap the next pass.

`--config 3|4|5` runs BASELINE's other configs with STRONG scaling by default: the pinned
totals (config 3: 500 symbols x 98,280 1-min bars x 64 params, quoted at 1 and 2 GPUs; config 4:
2,000 x 98,280 x 256 at 4 and 8 GPUs; config 5: 10,000 x 491,400 x 1,024 at 8 GPUs) are split
into contiguous symbol shards (parallel.shard), so `--gpus 8 --config 4` runs 250 symbols per
rank. `--scaling weak` keeps the per-GPU shard fixed instead (config 4: 500 per GPU).

`--leg ingest` times the engine's own share of a gRPC-fed run instead: bt_run_batch (the
drop-in for process_incoming_job) on 256 config-5 symbols as DBXCOL1 payloads in host memory —
payload validation and staging, H2D, the kernel, the summaries' read-back and the
CompleteRequest.data strings — and prints its own JSON line.

Run: python bench.py [--gpus N --steps K --warmup W] [--config C] [--scaling weak|strong]
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

# BASELINE configs: grid, symbols (per GPU for weak scaling, the pinned total for strong), bars,
# bar frequency, annualization, default scaling, and the SURVEY.md §8(d) byte-model terms c (OHLC
# columns consumed) and W (indicator series)
CONFIGS = {
    2: dict(grid=D.config2_grid, S=5000, B=2520, freq=D.BT_DAILY, ann=252, c=1, W=40,
            scaling="weak", name="BASELINE config 2: SMA fast/slow crossover, 5,000 symbols x "
            "2,520 daily bars x 400 params per GPU"),
    3: dict(grid=D.config3_grid, S=500, B=98280, freq=D.BT_MINUTE, ann=98280, c=1, W=16,
            scaling="strong", name="BASELINE config 3: EMA + rolling-OLS-slope mean reversion, "
            "500 symbols x 98,280 1-min bars x 64 params in total"),
    4: dict(grid=D.config4_grid, S=2000, B=98280, freq=D.BT_MINUTE, ann=98280, c=3, W=16,
            scaling="strong", name="BASELINE config 4: Bollinger z-score with SL/TP, 2,000 "
            "symbols x 98,280 1-min bars x 256 params in total"),
    5: dict(grid=D.config5_grid, S=10000, B=491400, freq=D.BT_MINUTE, ann=98280, c=1, W=64,
            scaling="strong", name="BASELINE config 5: SMA 32x32 grid, 10,000 symbols x 491,400 "
            "1-min bars (5 y) x 1,024 params in total"),
}
# the per-GPU shard the weak-scaling mode keeps for configs 3/4/5 (round-1 shard sizes)
WEAK_SHARD = {2: 5000, 3: 500, 4: 500, 5: 1250}


def algorithmic_bytes(S, B, P, c=1, W=40):
    """SURVEY.md §8(d) pinned byte model: B_alg = S*B*(8c + 16W) + 32*S*P."""
    return S * B * (8 * c + 16 * W) + 32 * S * P


def host_cpus():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota if any (the
    GPU box gives a job a share of a large host: nproc shows the whole machine)."""
    nproc = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, period = open(path).read().split()[:2]
            if q != "max":
                quota = int(q) / int(period)
        except (OSError, ValueError):
            pass
    usable = max(1, min(aff, int(quota) if quota else aff))
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable,
            "model": model}


def cpu_baseline(cfg, grid, sym0, shard, target_thread_s=25.0, target_1t_s=8.0):
    """The C oracle (oracle/oracle.c, -O2 -ffp-contract=off) on the first symbols of
    rank 0's shard of the same workload, on 1 thread and on every usable host CPU, each sample
    sized from a one-symbol probe (~8 s on one thread, ~25 thread-seconds on all), on the
    oracle's pthread pool (orc_*_grid_mt: one task per symbol, every param of it)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc_ffi as F
    cpus = host_cpus()
    B, freq, ann = cfg["B"], 1 if cfg["freq"] == D.BT_MINUTE else 0, cfg["ann"]
    cache = {}

    def cols(n):
        for s in range(len(cache), n):
            cache[s] = F.gen(SEED, sym0 + s, B, freq)
        return [cache[s] for s in range(n)]

    def run(n, threads):
        cs = cols(n)
        t0 = time.perf_counter()
        closes = np.stack([x[3] for x in cs])
        if grid.strategy == D.BT_SMA_CROSS:
            F.sma_grid_mt(closes, grid.axes[0], grid.axes[1], ann, threads)
        elif grid.strategy == D.BT_EMA_OLS:
            F.ema_grid_mt(closes, grid.axes[0], grid.axes[1], grid.band_bps, ann, threads)
        else:
            F.boll_grid_mt(np.stack([x[1] for x in cs]), np.stack([x[2] for x in cs]), closes,
                           grid.axes[0], grid.axes[1], grid.k_den, grid.axes[2], grid.axes[3],
                           ann, threads)
        return time.perf_counter() - t0

    per_sym = run(1, 1)  # one symbol on one thread: the probe
    n1 = int(min(shard, max(1, target_1t_s / max(per_sym, 1e-9))))
    dt1 = run(n1, 1) if n1 > 1 else per_sym
    T = cpus["usable"]
    nA = int(min(shard, max(T, target_thread_s / max(per_sym, 1e-9))))
    dtA = run(nA, T)
    per_eval = B * grid.n_params
    v1, vA = n1 * per_eval / dt1, nA * per_eval / dtA
    return {"value": vA, "unit": "bar-evals/s", "cores": T, "kind": "port",
            "sample": f"first {nA} symbols of the shard x {B} bars x {grid.n_params} params on "
                      f"{T} threads ({dtA:.2f} s wall); 1 thread: first {n1} symbols ({dt1:.2f} s); "
                      f"oracle/oracle.c orc_*_grid_mt, gcc -O2 -ffp-contract=off",
            "value_1t": v1, "value_all": vA, "threads_all": T, "nproc": cpus["nproc"],
            "affinity_cpus": cpus["affinity"], "cgroup_quota_cpus": cpus["cgroup_quota_cpus"],
            "model": cpus["model"]}


def load_pmc(config):
    """Measured HBM bytes and VALU instructions per launch of the dominant kernel from the
    committed rocprofv3 PMC summaries (profiles/pmc_config<C>.json, written by
    scripts/summarize_profile.py from separate --pmc passes of this same bench command)."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", f"pmc_config{config}.json")))
        return d
    except (OSError, ValueError):
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="default: weak for config 2, strong (BASELINE totals) for 3/4/5")
    ap.add_argument("--symbols", type=int, default=None,
                    help="override: symbols per GPU (weak) or in total (strong)")
    ap.add_argument("--leg", choices=["kernel", "ingest"], default="kernel")
    ap.add_argument("--topk", type=int, default=TOPK,
                    help="0 skips the top-k chain (profiling-build ablations, where Sharpes tie)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--segments", type=int, default=0,
                    help="bar segments per symbol (bt_set_segments): 0 = automatic, 1 = off")
    ap.add_argument("--burn", type=int, default=0,
                    help="burn-in tiles of a speculative segment: 0 = the strategy's default")
    ap.add_argument("--verify", action="store_true",
                    help="after timing, rank 0 runs every rank's symbols in one engine and asserts "
                         "that the exchanged top-k and counters equal it (N > 1 rehearsals)")
    args = ap.parse_args()
    if args.leg == "ingest":
        return ingest_leg(args)
    cfg = CONFIGS[args.config]
    scaling = args.scaling or cfg["scaling"]
    BARS = cfg["B"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if scaling == "weak":
        per = args.symbols or WEAK_SHARD[args.config]
        sym0, n_sym, total = rank * per, per, per * world
    else:
        total = args.symbols or cfg["S"]
        sym0, n_sym = PAR.shard(total, world, rank)
    dist = None
    comm = None
    device = local
    if world > 1:
        import torch
        import torch.distributed as dist
        # one process per GPU; ranks outnumbering the visible GPUs (a rehearsal on a 1-GPU box)
        # share devices, and RCCL needs distinct devices, so the exchange then uses gloo
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
    topk = args.topk
    eng = D.Engine(grid, device=device, topk=topk, timing=True)
    if args.segments or args.burn:
        eng.set_segments(args.segments, args.burn)
    eng.load_synthetic(SEED, sym0, n_sym, BARS, cfg["freq"])
    exchange = "none"
    if dist is not None:
        if dist.get_backend() == "nccl":
            try:  # the C-ABI exchange (RCCL from the engine's device buffers)
                comm = PAR.make_comm(dist, device, max(topk, 1))
                exchange = "RCCL all-gather via bt_exchange (C ABI)"
            except Exception as why:  # noqa: BLE001 — fall back to torch's RCCL all-gather
                print(f"bt_comm unavailable ({why}); exchanging over torch.distributed", file=sys.stderr)
        if comm is None:
            exchange = f"{dist.get_backend()} all-gather via torch.distributed"

    # steps in flight ahead of the one being consumed: at N > 1 two, so step i+2 is already
    # enqueued when finish(i) blocks. A step's top-k chain gets CU slots only once the next
    # step's kernel drains (config 4: persistent blocks hold every CU's LDS), so finish(i)
    # returns about when kernel i+1 ends; one step ahead would leave the GPU idle for the
    # exchange, the host merge and the next launch. N = 1 keeps one.
    depth = 2 if world > 1 else 1
    assert depth < D.PIPE_SLOTS

    def issue(i):
        eng.run()                      # kernels of step i, enqueued on the engine stream
        if topk == 0:
            return
        slot = i % D.PIPE_SLOTS
        if comm is not None:
            comm.exchange_async(eng, slot)   # RCCL all-gather behind the run's top-k chain
        else:
            eng.topk_fetch_async(slot)       # its top-k + trade count into a pinned slot

    xch_s = [0.0]  # host time in the torch.distributed exchange proper (issue + merge)
    pending = [None]  # torch.distributed carrier: the exchange still in flight

    def finish(i):
        """(top-k, [bar-evals, trades]) over every rank of step i (torch.distributed carrier: of
        step i - 1, the exchange of step i is left in flight; drain() completes it)."""
        if topk == 0:
            return None, None
        slot = i % D.PIPE_SLOTS
        if comm is not None:
            return comm.exchange_wait(slot)
        top, trades = eng.topk_fetch_wait(slot)
        if dist is None:
            return top, [n_sym * BARS * P, trades]
        # the one exchange step: a single all-gather carrying each rank's k x 24 B top-k records
        # and its run counters (summed on the host), in the C-ABI exchange's byte format, issued
        # asynchronously; the previous step's is merged now, a step after it was issued (the
        # RCCL carrier's all-gather likewise runs behind the next step's kernel)
        tx = time.perf_counter()
        prev, pending[0] = pending[0], PAR.exchange_async(top, topk, [n_sym * BARS * P, trades], dist)
        r = prev.wait() if prev is not None else (None, None)
        xch_s[0] += time.perf_counter() - tx
        return r

    def drain(res):
        """The last step's exchange, if one is in flight (torch.distributed carrier)."""
        if pending[0] is None:
            return res
        tx = time.perf_counter()
        res, pending[0] = pending[0].wait(), None
        xch_s[0] += time.perf_counter() - tx
        return res

    wait_s = [0.0]  # host time blocked in finish() this run: the wait for the step's GPU work
                    # (kernel, top-k chain, read-back or RCCL all-gather) plus the exchange

    def steps(n):
        """n steps; steps i+1 .. i+depth are enqueued before step i's read-back and exchange,
        so the GPU runs the next passes while the host consumes (and, for N > 1, exchanges)
        this one."""
        res = (None, None)
        wait_s[0] = xch_s[0] = 0.0
        for i in range(min(depth, n)):
            issue(i)
        for i in range(n):
            if i + depth < n:
                issue(i + depth)
            tw = time.perf_counter()
            res = finish(i)
            wait_s[0] += time.perf_counter() - tw
        tw = time.perf_counter()
        res = drain(res)
        wait_s[0] += time.perf_counter() - tw
        return res

    steps(args.warmup)
    eng.sync()
    eng.reset_timing()
    if dist is not None:
        import torch
        dist.barrier()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    top, counters = steps(args.steps)
    eng.sync()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kms, launches, kname = eng.kernel_timing()
    per_rank = None
    if dist is not None:
        # max over ranks of the timed region; and, gathered once after it, every rank's own
        # kernel average (HIP events), its host wait in finish() per step, the exchange proper
        # (torch.distributed carrier: all-gather + merge once the rank's top-k is on the host;
        # the RCCL all-gather runs on the GPU's top-k stream instead, -1 here) and the kernel
        # stream's idle time per step (timed region / steps - kernel average: what the exchange,
        # the host merge and the launches cost the GPU; meaningless when ranks share a device),
        # so a scaling loss can be told apart: load imbalance (kernel times differ) vs the exchange
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        k_avg = kms / max(launches, 1)
        mine = torch.tensor([elapsed, k_avg, wait_s[0] * 1e3 / max(args.steps, 1),
                             float(n_sym),
                             xch_s[0] * 1e3 / max(args.steps, 1) if comm is None else -1.0,
                             elapsed * 1e3 / max(args.steps, 1) - k_avg],
                            dtype=torch.float64, device=dev)
        alls = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(alls, mine)
        rows = torch.stack(alls).cpu().numpy()
        elapsed = float(rows[:, 0].max())

        def mm(col):
            return {"min": float(rows[:, col].min()), "max": float(rows[:, col].max()),
                    "by_rank": [float(x) for x in rows[:, col]]}
        per_rank = {"kernel_avg_ms": mm(1), "host_wait_ms_per_step": mm(2),
                    "exchange_ms_per_step": mm(4) if comm is None else None,
                    "gpu_idle_ms_per_step": mm(5),
                    "ranks_share_device": torch.cuda.device_count() < world,
                    "pipeline_depth": depth,
                    "timed_region_s": mm(0), "symbols": [int(x) for x in rows[:, 3]]}
    stats = eng.stats()
    # bar segments per symbol of the last run and the blocks its fix passes re-walked (read
    # after the timed region: the count is a device read-back)
    n_seg, refixed = eng.last_segments(with_refixed=True)

    verified = None
    if args.verify and rank == 0 and topk > 0:
        verified = verify_exchange(cfg, grid, total, top, counters, device, topk, args)

    if rank == 0:
        evals_per_step = total * BARS * P
        value = evals_per_step * args.steps / elapsed
        kavg_s = kms / 1e3 / max(launches, 1)
        alg = algorithmic_bytes(n_sym, BARS, P, cfg["c"], cfg["W"])
        achieved = alg / kavg_s / 1e9
        pmc = load_pmc(args.config)
        # measured traffic applies to the shard it was profiled on
        same_shard = pmc.get("symbols") == n_sym
        traffic = pmc.get("hbm_bytes_per_launch") if same_shard else None
        valu = pmc.get("SQ_INSTS_VALU") if same_shard else None
        valu_frac = (valu / kavg_s / 1e9 / VALU_PEAK_GINST) if valu else None
        line = {
            "metric": "bar-evals/sec (symbols x params x bars)",
            "value": value,
            "unit": "bar-evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64+int64",
            "data": "synthetic (SplitMix64 integer OHLC walk, docs/oracle_spec.md §1, generated in HBM)",
            "config": {"workload": cfg["name"] if scaling == cfg["scaling"] and args.symbols is None
                       else f"{cfg['name'].split(':')[0]}: {total} symbols in total, {scaling} scaling",
                       "symbols_total": total, "symbols_per_gpu": n_sym, "bars": BARS, "params": P,
                       "topk": TOPK, "parallelism": f"dp{world} (contiguous symbol shards; "
                       f"exchange: {exchange})"},
            # The fused kernels move far fewer bytes than the pinned two-stage model charges, so
            # they are not HBM-bound: achieved/frac are the SURVEY.md §8(d) model (B_alg / kernel
            # time, the number BASELINE asks for); traffic/traffic_GBps are the measured PMC
            # bytes; the binding limit is VALU issue/latency (valu_issue_frac).
            "roofline": {"bound": "valu", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "model": "SURVEY.md §8(d) pinned bytes B_alg = S*B*(8c+16W) + 32*S*P",
                         "alg_bytes_per_launch": alg,
                         "traffic": traffic,
                         "traffic_GBps": traffic / kavg_s / 1e9 if traffic else None,
                         "traffic_frac": traffic / kavg_s / 1e9 / HBM_PEAK_GBS if traffic else None,
                         "valu_insts_per_launch": valu,
                         "valu_issue_frac": valu_frac,
                         "pmc_source": pmc.get("source") if same_shard else None,
                         "kernel": kname, "kernel_avg_ms": kavg_s * 1e3},
            "trades_per_step": stats["trades"],
            "trades_per_step_all_ranks": counters[1] if counters else None,
            "bar_segments": {"per_symbol": n_seg, "refixed_blocks_last_step": refixed},
            "top1": {"sharpe": float(top[0]["sharpe"]), "sym": int(top[0]["sym"]),
                     "param": int(top[0]["param"])} if top is not None and len(top) else None,
        }
        if per_rank is not None:
            line["per_rank"] = per_rank
        if verified is not None:
            line["verified_exchange"] = verified
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, grid, sym0, n_sym)
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def verify_exchange(cfg, grid, total, top, counters, device, k, args):
    """Rank 0, after the timed region: one engine over every rank's symbols (0 .. total-1) on this
    GPU; the exchanged top-k must equal its device top-k record for record, and the summed
    counters its bar-evals and trade count. Raises on a mismatch (a nonzero exit)."""
    ref = D.Engine(grid, device=device, topk=k)
    if args.segments or args.burn:
        ref.set_segments(args.segments, args.burn)
    ref.load_synthetic(SEED, 0, total, cfg["B"], cfg["freq"])
    ref.run()
    want = ref.read_topk(k)
    st = ref.stats()
    ref.close()
    got = np.asarray(top, D.TOPK_DTYPE)
    assert got.tobytes() == np.asarray(want, D.TOPK_DTYPE).tobytes(), \
        f"exchanged top-{k} differs from a single engine over all {total} symbols"
    assert counters == [st["bar_evals"], st["trades"]], (counters, st)
    return {"symbols": total, "topk": len(got), "bar_evals": counters[0], "trades": counters[1]}


def ingest_leg(args):
    """bt_run_batch alone on host-resident DBXCOL1 payloads of config-5 symbols (SURVEY.md §8(f)
    rows 1-2): the engine's share of a gRPC-fed run, without the gRPC transport."""
    from concurrent.futures import ThreadPoolExecutor
    from dbx_amd import payload as PL
    cfg = CONFIGS[5]
    n_jobs = args.symbols or 256
    grid = cfg["grid"]()
    with ThreadPoolExecutor(16) as ex:
        payloads = list(ex.map(lambda s: PL.gen_payload(SEED, s, cfg["B"], cfg["freq"]), range(n_jobs)))
    jobs = [(f"job-{s}", b) for s, b in enumerate(payloads)]
    eng = D.Engine(grid, device=0)
    for _ in range(max(args.warmup, 1)):
        eng.run_batch(jobs)
    profs, walls = [], []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        res = eng.run_batch(jobs)
        walls.append(time.perf_counter() - t0)
        profs.append(eng.batch_profile())
    assert all(st == 0 for st, _ in res)
    med = {k: float(np.median([p[k] for p in profs])) for k in profs[0] if k.endswith("_ms")}
    pb, bars = profs[0]["payload_bytes"], profs[0]["bars"]
    pr = profs[0]["payload_bytes_read"]  # the volume column is carried but never read
    wall = float(np.median(walls))
    line = {
        "leg": "bt_run_batch on DBXCOL1 payloads (engine share of a gRPC-fed run)",
        "workload": f"{n_jobs} config-5 symbols x {cfg['B']} 1-min bars x {grid.n_params} params",
        "jobs": n_jobs, "payload_bytes": pb, "payload_bytes_read": pr,
        "result_bytes": sum(len(d) for _, d in res),
        "steps": args.steps, "phase_ms_median": med, "call_wall_ms_median": wall * 1e3,
        # rates over the bytes ingest actually reads (header + four int32 price columns)
        "ingest_GBps": pr / ((med["host_ingest_ms"] + med["upload_ms"]) * 1e6),
        "host_ingest_GBps": pr / (med["host_ingest_ms"] * 1e6),
        "ingest_GBps_all_payload_bytes": pb / ((med["host_ingest_ms"] + med["upload_ms"]) * 1e6),
        "upload_GBps": bars * 4 / (med["upload_ms"] * 1e6),
        "bar_evals_per_s_end_to_end": bars * grid.n_params / wall,
        "bar_evals_per_s_kernel": bars * grid.n_params / (med["compute_ms"] * 1e-3),
        "host_threads": min(16, os.cpu_count() or 1),
    }
    print(json.dumps(line), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
