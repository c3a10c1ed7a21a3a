"""gRPC-fed config-5 pipeline with the counterparts in separate processes: the dispatcher
(dispatcher.main, DBXCOL1 payload files, no gzip) in one process and W worker processes
(worker.main, each its own engine on GPU 0, F RequestJobs connections each), so grpcio's Python
work no longer shares one interpreter lock (scripts/e2e_grpc.py runs both in one process).
Workers are started first and the clock runs from the dispatcher's "serving" line to its
"done" line; every result line is checked in the results sink.

  python scripts/e2e_grpc_mp.py --symbols 256 --workers 4 --fetchers 4
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dbx_amd as D  # noqa: E402
from dbx_amd import payload as PL  # noqa: E402

BOOT = "import sys; sys.path.insert(0, {root!r}); from dbx_amd import {mod} as M; M.main(sys.argv[1:])"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _lines(proc, sink):
    for line in proc.stdout:
        sink.append((time.perf_counter(), line.rstrip()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--symbols", type=int, default=256)
    ap.add_argument("--bars", type=int, default=491400)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--fetchers", type=int, default=4)
    ap.add_argument("--batch", type=int, default=16, help="jobs per RequestJobs (cores)")
    ap.add_argument("--max-batch-mb", type=int, default=2048)
    ap.add_argument("--min-batch-jobs", type=int, default=0)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="dbx_e2e_mp_")
    data = os.path.join(tmp, "data")
    os.makedirs(data)

    def gen(s):
        with open(os.path.join(data, f"SYM{s:05d}.dbxcol"), "wb") as f:
            f.write(PL.gen_payload(0x5EED, s, a.bars, D.BT_MINUTE))

    t0 = time.perf_counter()
    with ThreadPoolExecutor(16) as ex:
        list(ex.map(gen, range(a.symbols)))
    payload = sum(os.path.getsize(os.path.join(data, f)) for f in os.listdir(data))
    print(f"generated {a.symbols} payloads ({payload / 2 ** 20:.0f} MiB) in {time.perf_counter() - t0:.1f} s",
          flush=True)
    port = _free_port()
    target = f"127.0.0.1:{port}"
    workers, wout = [], []
    for _ in range(a.workers):
        p = subprocess.Popen([sys.executable, "-u", "-c", BOOT.format(root=ROOT, mod="worker"),
                              "--target", target, "--grid", "config5", "--quiet",
                              "--cores", str(a.batch), "--max-receive-mb", "2000",
                              "--max-batch-mb", str(a.max_batch_mb),
                              "--min-batch-jobs", str(a.min_batch_jobs),
                              "--fetchers", str(a.fetchers), "--duration", "300"],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        workers.append(p)
        threading.Thread(target=_lines, args=(p, wout), daemon=True).start()
    t_ready = time.perf_counter()
    beat = t_ready
    while sum(1 for _, ln in wout if ln == "worker ready") < a.workers:
        if time.perf_counter() - beat > 20:  # the first torch import on a fresh box takes minutes
            beat = time.perf_counter()
            print(f"  ... waiting for workers ({time.perf_counter() - t_ready:.0f} s)", flush=True)
        if time.perf_counter() - t_ready > 240 or any(p.poll() is not None for p in workers):
            for p in workers:
                p.kill()
            raise SystemExit("workers did not start: " + "\n".join(ln for _, ln in wout[-20:]))
        time.sleep(0.05)
    print(f"{a.workers} workers ready in {time.perf_counter() - t_ready:.1f} s", flush=True)
    results = os.path.join(tmp, "results.jsonl")
    disp = subprocess.Popen([sys.executable, "-u", "-c", BOOT.format(root=ROOT, mod="dispatcher"), data,
                             "--addr", target, "--no-gzip", "--max-send-mb", "2000",
                             "--exit-when-done", "--results", results],
                            stdout=subprocess.PIPE, stderr=open(os.path.join(tmp, "dispatcher.err"), "w"),
                            text=True)
    dout = []
    th = threading.Thread(target=_lines, args=(disp, dout), daemon=True)
    th.start()
    try:
        t_wait = time.perf_counter()
        beat = t_wait
        while disp.poll() is None:
            time.sleep(0.5)
            if time.perf_counter() - beat > 20:  # progress (a silent GPU command looks hung)
                beat = time.perf_counter()
                done = sum(1 for _ in open(results)) if os.path.exists(results) else 0
                print(f"  ... {done}/{a.symbols} jobs done", flush=True)
            if time.perf_counter() - t_wait > 240 or all(p.poll() is not None for p in workers):
                disp.kill()
                disp_err = open(os.path.join(tmp, "dispatcher.err")).read()[-2000:]
                raise SystemExit("dispatcher did not finish: " + "\n".join(ln for _, ln in (dout + wout)[-20:])
                                 + "\n--- dispatcher stderr:\n" + disp_err)
    finally:
        for p in workers:
            p.terminate()
        for p in workers:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
    th.join(timeout=5)
    t_serve = next(t for t, ln in dout if ln == "dispatcher serving")
    t_done = next(t for t, ln in dout if ln.startswith("dispatcher done"))
    wall = t_done - t_serve
    n_lines, n_jobs = 0, 0
    with open(results) as f:
        for line in f:
            rec = json.loads(line)
            n_jobs += 1
            n_lines += rec["data"].count("\n")
    grid = D.config5_grid()
    line = {"workload": "config-5 pipeline, gRPC-fed, 1 GPU, counterparts in separate processes",
            "symbols": a.symbols, "bars": a.bars, "params": grid.n_params, "workers": a.workers,
            "fetchers": a.fetchers, "batch": a.batch, "max_batch_mb": a.max_batch_mb,
            "payload_mb": payload / 2 ** 20, "wall_s": wall, "GBps": payload / wall / 1e9,
            "bar_evals_per_s_end_to_end": a.symbols * a.bars * grid.n_params / wall,
            "jobs_done": n_jobs, "result_lines": n_lines,
            "all_done": n_jobs == a.symbols and n_lines == a.symbols * grid.n_params}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
