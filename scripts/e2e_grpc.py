"""End-to-end gRPC-fed run on one GPU (the config-5 pipeline at a reduced symbol count):
dispatcher counterpart serving DBXCOL1 payload files (no gzip) -> worker counterpart with the
HIP engine (one bt_run_batch per JobsReply) -> results sink. Reports wall-clock bar-evals/s
end to end (host I/O, gRPC transfer, ingest, H2D, kernels, result strings) beside the kernel
time. Config 5 is 10,000 symbols x 491,400 bars x 1,024 params over 8 GPUs.

  python scripts/e2e_grpc.py --symbols 64 --bars 491400 --batch 16
"""
import argparse
import json
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import dbx_amd as D  # noqa: E402
from dbx_amd import dispatcher as DSP  # noqa: E402
from dbx_amd import payload as PL  # noqa: E402
from dbx_amd import worker as WK  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--symbols", type=int, default=64)
    ap.add_argument("--bars", type=int, default=491400)
    ap.add_argument("--batch", type=int, default=16, help="jobs per RequestJobs (cores)")
    ap.add_argument("--max-batch-mb", type=int, default=0, help="worker-side reply merging")
    ap.add_argument("--min-batch-jobs", type=int, default=0, help="worker-side linger target")
    ap.add_argument("--fetchers", type=int, default=1, help="worker RequestJobs connections")
    a = ap.parse_args()
    grid = D.config5_grid()
    tmp = tempfile.mkdtemp(prefix="dbx_e2e_")
    t0 = time.perf_counter()
    paths = []
    for s in range(a.symbols):
        p = os.path.join(tmp, f"SYM{s:05d}.dbxcol")
        with open(p, "wb") as f:
            f.write(PL.gen_payload(0x5EED, s, a.bars, D.BT_MINUTE))
        paths.append(p)
    t_gen = time.perf_counter() - t0
    disp = DSP.Dispatcher(paths, results_path=os.path.join(tmp, "results.jsonl"))
    server, port = DSP.serve(disp, "127.0.0.1:0", max_send=1 << 30, gzip=False)
    with D.Engine(grid, timing=True) as eng:
        w = WK.Worker(f"127.0.0.1:{port}", WK.engine_processor(eng), cores=a.batch,
                      job_tick=0.01, status_tick=0.5, max_receive=1 << 30,
                      max_batch_bytes=a.max_batch_mb << 20, min_batch_jobs=a.min_batch_jobs,
                      fetchers=a.fetchers)
        th = threading.Thread(target=w.run, daemon=True)
        t0 = time.perf_counter()
        th.start()
        last, beat = 0, time.perf_counter()
        while not disp.all_done() and time.perf_counter() - t0 < 600:
            time.sleep(0.02)
            if time.perf_counter() - beat > 10:
                beat = time.perf_counter()
                print(f"  ... {len(disp.done_paths)} done, {len(disp.files)} queued", flush=True)
            if len(disp.done_paths) != last:
                last = len(disp.done_paths)
                print(f"  {last}/{a.symbols} jobs done at {time.perf_counter() - t0:.1f} s", flush=True)
        wall = time.perf_counter() - t0
        w.stop.set()
        th.join(10)
        kms, nl, kname = eng.kernel_timing()
    server.stop(0)
    disp.close()
    evals = a.symbols * a.bars * grid.n_params
    n_lines = sum(len(v.strip().split("\n")) for v in disp.results.values())
    print(json.dumps({"workload": "config-5 pipeline, gRPC-fed, 1 GPU", "symbols": a.symbols,
                      "bars": a.bars, "params": grid.n_params, "batch": a.batch, "max_batch_mb": a.max_batch_mb, "min_batch_jobs": a.min_batch_jobs, "fetchers": a.fetchers,
                      "payload_mb": sum(os.path.getsize(p) for p in paths) / 2**20,
                      "gen_s": t_gen, "wall_s": wall, "bar_evals_per_s_end_to_end": evals / wall,
                      "kernel": kname, "kernel_ms_total": kms, "launches": nl,
                      "bar_evals_per_s_kernel": evals / (kms * 1e-3) if kms else None,
                      "all_done": disp.all_done(), "result_lines": n_lines}))
    for p in paths:
        os.unlink(p)


if __name__ == "__main__":
    main()
