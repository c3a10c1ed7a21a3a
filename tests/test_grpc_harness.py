"""BASELINE config 1 end-to-end over the reference's wire contract: a dispatcher counterpart
serving 16 synthetic daily CSVs and one worker counterpart requesting jobs, processing each
JobsReply and completing every job with CompleteRequest{id, data}.

CPU test: the worker's processor is the C oracle (test infrastructure standing in for the GPU
so the control-plane semantics are checked here). GPU test: the processor is libbt.so."""
import json
import os
import threading
import time

import numpy as np
import pytest

import dbx_amd as D
from dbx_amd import dispatcher as DSP
from dbx_amd import proto as P
from dbx_amd import worker as WK

N_FILES, BARS = 16, 2520


def _write_files(tmp_path):
    import oracle_np as N
    paths, closes = [], []
    o, h, lo, c, v = N.gen(0x5EED, list(range(N_FILES)), BARS, 0)
    for i in range(N_FILES):
        pth = tmp_path / f"SYM{i:02d}_daily.csv"
        pth.write_bytes(N.csv_bytes(o[i], h[i], lo[i], c[i], v[i], 0))
        paths.append(str(pth))
        closes.append(c[i].astype(np.int32))
    return paths, closes


def oracle_processor(grid):
    """Test stand-in for the engine: parse with the C oracle, score every param, format the
    same JSON lines as the engine (docs/oracle_spec.md §6)."""
    import orc_ffi as F

    def run(jobs):
        out = []
        for _jid, data in jobs:
            try:
                _o, _h, _l, c, _v = F.parse_csv(bytes(data))
            except ValueError as e:
                out.append(json.dumps({"error": str(e)}) + "\n")
                continue
            lines = []
            for p in range(grid.n_params):
                kw = grid.param(p)
                s, _ = F.sma(c, kw["f"], kw["s"], 252)
                lines.append(json.dumps({"param": p, "n": int(s["n_trades"]), "pnl": int(s["pnl"]),
                                         "mdd": int(s["mdd"]), "exp": int(s["exposure"]),
                                         "sharpe": repr(float(s["sharpe"])),
                                         "h": f"{int(s['hash']):016x}"}))
            out.append("\n".join(lines) + "\n")
        return out
    return run


def _run_e2e(tmp_path, processor, grid, cores=4, timeout=60, **worker_kw):
    paths, closes = _write_files(tmp_path)
    disp = DSP.Dispatcher(paths)
    replies = []
    orig = disp.request_jobs

    def spy(req, ctx):  # record which files each reply carried
        before = list(disp.files)
        rep = orig(req, ctx)
        replies.append([p for p in before if p not in disp.files])
        return rep
    disp.request_jobs = spy
    server, port = DSP.serve(disp, "127.0.0.1:0")
    w = WK.Worker(f"127.0.0.1:{port}", processor, cores=cores, job_tick=0.05, status_tick=0.2,
                  **worker_kw)
    th = threading.Thread(target=w.run, daemon=True)
    t0 = time.time()
    th.start()
    try:
        while len(disp.jobs_completed) < N_FILES and time.time() - t0 < timeout:
            time.sleep(0.05)
    finally:
        w.stop.set()
        th.join(10)
        server.stop(0)
        disp.close()
    wall = time.time() - t0
    assert len(disp.jobs_completed) == N_FILES, f"completed {len(disp.jobs_completed)}"
    return disp, replies, paths, closes, wall


def _check_results(disp, paths, closes, grid):
    import orc_ffi as F
    by_path = {disp.job_paths[j]: d for j, d in disp.results.items()}
    for pth, c in zip(paths, closes):
        lines = by_path[pth].strip().split("\n")
        assert len(lines) == grid.n_params
        for p, line in enumerate(lines):
            j = json.loads(line)
            kw = grid.param(p)
            s, _ = F.sma(c, kw["f"], kw["s"], 252)
            assert j["param"] == p and j["n"] == int(s["n_trades"]) and j["pnl"] == int(s["pnl"])
            assert j["mdd"] == int(s["mdd"]) and float(j["sharpe"]) == float(s["sharpe"])
            assert int(j["h"], 16) == int(s["hash"])


def test_config1_end_to_end_cpu_processor(tmp_path):
    grid = D.config2_grid()
    disp, replies, paths, closes, wall = _run_e2e(tmp_path, oracle_processor(grid), grid)
    # split_off semantics (server/main.rs:151-162): reply 1 = files[4..16], reply 2 = files[0..4]
    nonempty = [r for r in replies if r]
    assert nonempty[0] == paths[4:] and nonempty[1] == paths[:4]
    _check_results(disp, paths, closes, grid)


def test_extra_fetchers_complete_every_job_once(tmp_path):
    """Worker with three RequestJobs connections (fetchers) and reply merging: every file is
    handed out once (no re-dispatch), completed, and its results are the oracle's."""
    grid = D.config2_grid()
    disp, replies, paths, closes, wall = _run_e2e(tmp_path, oracle_processor(grid), grid, cores=2,
                                                  fetchers=3, max_batch_bytes=1 << 20)
    assert sorted(disp.job_paths.values()) == sorted(paths)  # each path handed out once
    assert disp.requeued == 0
    assert len({ctx for ctx in disp.peers}) >= 2  # the fetchers' own connections
    _check_results(disp, paths, closes, grid)


@pytest.mark.gpu
def test_config1_end_to_end_gpu_engine(tmp_path):
    grid = D.config2_grid()
    with D.Engine(grid) as eng:
        disp, replies, paths, closes, wall = _run_e2e(tmp_path, WK.engine_processor(eng), grid)
    _check_results(disp, paths, closes, grid)
    print(f"config 1 end-to-end: {N_FILES} jobs in {wall:.2f} s wall")


def test_split_off_semantics():
    f = list("abcdefghijklmnop")
    assert DSP.split_off_n_jobs(f, 4) == list("efghijklmnop") and f == list("abcd")
    assert DSP.split_off_n_jobs(f, 4) == list("abcd") and f == []
    assert DSP.split_off_n_jobs(f, 4) is None
    g = list("xyz")
    assert DSP.split_off_n_jobs(g, 0) == list("xyz") and g == []


def test_wire_bytes_match_reference_contract(golden_dir):
    pins = json.load(open(os.path.join(golden_dir, "wire.json")))
    assert P.JobsRequest(cores=4).SerializeToString().hex() == pins["JobsRequest{cores=4}"]
    assert P.StatusRequest(status=P.RUNNING).SerializeToString().hex() == pins["StatusRequest{RUNNING}"]
    rep = P.JobsReply(jobs=[P.Job(id="abc", File=b"t,o,h,l,c,v\n")])
    assert rep.SerializeToString().hex() == pins["JobsReply{[Job{id:'abc', File:'t,o,h,l,c,v\\n'}]}"]
    # field numbers/types of the other messages (proto:29-32)
    cr = P.CompleteRequest(id="i", data="d").SerializeToString()
    assert cr == b"\x0a\x01i\x12\x01d"
    # the dispatcher's direct encoder writes the same bytes as the message runtime
    assert P.encode_jobs_reply([("abc", b"t,o,h,l,c,v\n")]).hex() == pins["JobsReply{[Job{id:'abc', File:'t,o,h,l,c,v\\n'}]}"]


def test_jobs_reply_encoder_matches_message_runtime():
    """proto.encode_jobs_reply == JobsReply(...).SerializeToString(): empty ids / files (omitted
    in proto3), multi-byte varints (127/128/16383/16384-byte and 2 MB payloads), many jobs, and
    the dispatcher's Reply parses back to the same jobs."""
    import random
    rng = random.Random(7)
    sizes = [0, 1, 127, 128, 16383, 16384, 2 << 20] + [rng.randrange(0, 5000) for _ in range(20)]
    jobs = [(("" if i % 5 == 0 else str(rng.getrandbits(128))), bytes(rng.getrandbits(8) for _ in range(min(n, 64))) * (n // 64) + b"z" * (n % 64))
            for i, n in enumerate(sizes)]
    ref = P.JobsReply(jobs=[P.Job(id=j, File=f) for j, f in jobs]).SerializeToString()
    assert P.encode_jobs_reply(jobs) == ref
    assert P.encode_jobs_reply([]) == P.JobsReply().SerializeToString() == b""
    back = P.JobsReply.FromString(DSP.Reply([DSP.Job(j, f) for j, f in jobs]).SerializeToString())
    assert [(j.id, j.File) for j in back.jobs] == jobs


def test_process_incoming_job_flag_and_order():
    import queue
    seen = []

    def proc(jobs):
        assert WK.PROC_FLAG.is_set()       # process.rs:18
        seen.extend(j for j, _ in jobs)
        return [f"r{j}" for j, _ in jobs]
    q = queue.Queue()
    rep = P.JobsReply(jobs=[P.Job(id=str(i), File=b"x") for i in range(5)])
    WK.process_incoming_job(rep, q, proc)
    assert not WK.PROC_FLAG.is_set()       # process.rs:28
    assert [q.get_nowait() for _ in range(5)] == [(str(i), f"r{i}") for i in range(5)]


class _Ctx:
    """Minimal grpc ServicerContext stand-in for direct handler calls."""
    def __init__(self, peer, metadata=()):
        self._peer = peer
        self._md = tuple(metadata)

    def peer(self):
        return self._peer

    def invocation_metadata(self):
        return self._md

    def abort(self, code, msg):
        raise RuntimeError(msg)


def test_dispatcher_redispatches_jobs_of_lost_worker(tmp_path):
    """jobs held by a worker that stops checking in (pruned after the
    silence limit, server/main.rs:183-190) go back to the queue; a second worker completes
    them. The results sink keeps each path's first completion (row 3)."""
    paths = [str(tmp_path / f"f{i}.csv") for i in range(6)]
    for p in paths:
        open(p, "wb").write(b"2020-01-01,1,1,1,1,1\n")
    sink = tmp_path / "results.jsonl"
    d = DSP.Dispatcher(paths, prune_after_s=0.3, check_every_s=0.05, results_path=str(sink))
    try:
        a = d.request_jobs(P.JobsRequest(cores=4), _Ctx("ipv4:10.0.0.1:1"))   # tail: f4, f5
        assert [d.job_paths[j.id] for j in a.jobs] == paths[4:]
        b = d.request_jobs(P.JobsRequest(cores=4), _Ctx("ipv4:10.0.0.2:2"))   # f0..f3
        for j in b.jobs:
            d.complete_job(P.CompleteRequest(id=j.id, data="ok-b"), _Ctx("ipv4:10.0.0.2:2"))
        assert not d.all_done()
        t0 = time.time()
        while d.requeued < 2 and time.time() - t0 < 5:
            # worker B keeps polling (upserting its last_connection); worker A is silent
            d.peers["ipv4:10.0.0.2:2"]["last_connection"] = time.time()
            time.sleep(0.05)
        assert d.requeued == 2 and "ipv4:10.0.0.1:1" not in d.peers
        c = d.request_jobs(P.JobsRequest(cores=4), _Ctx("ipv4:10.0.0.2:2"))
        assert sorted(d.job_paths[j.id] for j in c.jobs) == paths[4:]
        assert {j.id for j in c.jobs}.isdisjoint({j.id for j in a.jobs})    # fresh ids
        for j in c.jobs:
            d.complete_job(P.CompleteRequest(id=j.id, data="ok-c"), _Ctx("ipv4:10.0.0.2:2"))
        d.complete_job(P.CompleteRequest(id=a.jobs[0].id, data="late-a"), _Ctx("x"))  # late
        assert d.all_done()
    finally:
        d.close()
    rows = [json.loads(x) for x in sink.read_text().splitlines()]
    assert sorted(r["path"] for r in rows) == sorted(paths)            # one row per path
    assert all(r["data"] != "late-a" for r in rows)


@pytest.mark.gpu
def test_binary_payload_minute_jobs_end_to_end_gpu(tmp_path):
    """§8(f) rows 1-2: 1-minute symbols as DBXCOL1 payloads (2.4 MB each, 4 per JobsReply =
    9.4 MB > grpc's 4 MiB default: the worker raises its receive limit), served without gzip,
    EMA+OLS grid (config 3) on the GPU engine, results checked against the C oracle."""
    import orc_ffi as F
    from dbx_amd import payload as PL
    bars, n = 98280, 8
    paths = []
    for s in range(n):
        pth = tmp_path / f"S{s}.dbxcol"
        pth.write_bytes(PL.gen_payload(0x5EED, s, bars, D.BT_MINUTE))
        paths.append(str(pth))
    grid = D.config3_grid()
    disp = DSP.Dispatcher(paths, results_path=str(tmp_path / "res.jsonl"))
    server, port = DSP.serve(disp, "127.0.0.1:0", gzip=False)
    with D.Engine(grid) as eng:
        w = WK.Worker(f"127.0.0.1:{port}", WK.engine_processor(eng), cores=4, job_tick=0.05,
                      status_tick=0.2, max_receive=64 << 20)
        th = threading.Thread(target=w.run, daemon=True)
        t0 = time.time()
        th.start()
        try:
            while not disp.all_done() and time.time() - t0 < 90:
                time.sleep(0.05)
        finally:
            w.stop.set()
            th.join(10)
            server.stop(0)
            disp.close()
    assert disp.all_done()
    print(f"{n} x {bars} minute bars over gRPC in {time.time() - t0:.2f} s")
    rows = [json.loads(x) for x in (tmp_path / "res.jsonl").read_text().splitlines()]
    for r in rows:
        s = paths.index(r["path"])
        o, h, lo, c = F.gen(0x5EED, s, bars, 1)[:4]
        lines = r["data"].strip().split("\n")
        assert len(lines) == grid.n_params
        for p in (0, 9, 27, 63):
            kw = grid.param(p)
            ref, _ = F.ema_ols(c, kw["n"], kw["w"], kw["band_bps"], 98280)
            j = json.loads(lines[p])
            assert j["n"] == int(ref["n_trades"]) and j["pnl"] == int(ref["pnl"])
            assert float(j["sharpe"]) == float(ref["sharpe"]) and int(j["h"], 16) == int(ref["hash"])


def test_dispatcher_caps_reply_bytes(tmp_path):
    """A reply larger than the send limit would fail after its files left the queue; the
    dispatcher caps each JobsReply by bytes and requeues the overflow."""
    paths = [str(tmp_path / f"f{i}") for i in range(10)]
    for p in paths:
        open(p, "wb").write(b"x" * 1000)
    d = DSP.Dispatcher(paths, max_reply_bytes=3500)
    try:
        r = d.request_jobs(P.JobsRequest(cores=2), _Ctx("a"))          # tail f2..f9, capped
        assert [d.job_paths[j.id] for j in r.jobs] == paths[2:5]
        assert d.files == paths[:2] + paths[5:]
        got = [d.job_paths[j.id] for j in r.jobs]
        while d.files:
            got += [d.job_paths[j.id] for j in d.request_jobs(P.JobsRequest(cores=2), _Ctx("a")).jobs]
        assert sorted(got) == sorted(paths)
    finally:
        d.close()
