"""Worker / dispatcher counterparts on the CPU, without a server:
reply merging on the compute thread, engine failures answered per job, receive-limit-aware
reply caps, unreadable paths counted as finished."""
import json
import queue
import threading
import time

from dbx_amd import dispatcher as DSP
from dbx_amd import proto as P
from dbx_amd import worker as WK
from test_grpc_harness import _Ctx


def _reply(ids, size=10):
    return P.JobsReply(jobs=[P.Job(id=str(i), File=b"x" * size) for i in ids])


def _run_compute(w, replies, wait_jobs, timeout=5.0):
    """Feed replies to the worker's compute thread (main.rs:38-42) and collect completions."""
    for r in replies:
        w.reply_q.put(r)
    th = threading.Thread(target=w._compute, daemon=True)
    th.start()
    got = []
    t0 = time.time()
    while len(got) < wait_jobs and time.time() - t0 < timeout:
        try:
            got.append(w.complete_q.get(timeout=0.05))
        except queue.Empty:
            pass
    w.stop.set()
    th.join(2)
    return got


def test_reply_merging_batches_queued_replies_in_order():
    """f2: with max_batch_bytes the compute thread merges the JobsReplies already queued into one
    engine batch (one launch), up to the byte budget, keeping job order."""
    calls = []

    def proc(jobs):
        calls.append([j for j, _ in jobs])
        return [f"r{j}" for j, _ in jobs]
    w = WK.Worker("127.0.0.1:1", proc, cores=2, max_batch_bytes=45)
    got = _run_compute(w, [_reply([0, 1]), _reply([2, 3]), _reply([4, 5]), _reply([6])], 7)
    assert [g[0] for g in got] == [str(i) for i in range(7)]
    assert [g[1] for g in got] == [f"r{i}" for i in range(7)]
    # 20 B per reply: the first batch stops once it holds >= 45 B (three replies)
    assert calls[0] == ["0", "1", "2", "3", "4", "5"] and calls[1] == ["6"]


def test_reply_merging_lingers_for_min_batch_jobs():
    """f2: while a batch holds fewer than min_batch_jobs symbols the thread waits linger_s for
    another reply instead of launching a nearly empty grid."""
    calls = []

    def proc(jobs):
        calls.append(len(jobs))
        return ["ok"] * len(jobs)
    w = WK.Worker("127.0.0.1:1", proc, cores=2, max_batch_bytes=1 << 20, min_batch_jobs=4,
                  linger_s=0.5)

    def late():
        time.sleep(0.15)
        w.reply_q.put(_reply([2, 3]))
    threading.Thread(target=late, daemon=True).start()
    got = _run_compute(w, [_reply([0, 1])], 4)
    assert len(got) == 4 and calls == [4]


def test_without_merging_one_reply_per_call():
    calls = []

    def proc(jobs):
        calls.append(len(jobs))
        return ["ok"] * len(jobs)
    w = WK.Worker("127.0.0.1:1", proc, cores=2)
    _run_compute(w, [_reply([0, 1]), _reply([2])], 3)
    assert calls == [2, 1]                               # main.rs:38-42: one reply per call


def test_engine_failure_completes_every_job_with_an_error():
    """An exception in the processor (HIP error, BtError) must not end the compute thread: every
    job of the batch completes with {"error": ...} and later batches still run."""
    n = {"calls": 0}

    def proc(jobs):
        n["calls"] += 1
        if n["calls"] == 1:
            raise RuntimeError("hipErrorLaunchFailure")
        return ["fine"] * len(jobs)
    w = WK.Worker("127.0.0.1:1", proc, cores=2)
    got = _run_compute(w, [_reply([0, 1, 2]), _reply([3])], 4)
    assert [g[0] for g in got] == ["0", "1", "2", "3"]
    for _, data in got[:3]:
        assert "hipErrorLaunchFailure" in json.loads(data)["error"]
    assert got[3][1] == "fine" and not WK.PROC_FLAG.is_set()


def test_processor_with_wrong_result_count_is_an_error():
    q = queue.Queue()
    WK.process_incoming_job(_reply([0, 1]), q, lambda jobs: ["only one"])
    assert [q.get_nowait()[0] for _ in range(2)] == ["0", "1"]


def test_reply_capped_below_worker_receive_limit(tmp_path):
    """The worker advertises its receive limit in metadata; the dispatcher keeps replies below
    it (less framing) so a reply is never refused after its files left the queue."""
    paths = [str(tmp_path / f"f{i}") for i in range(8)]
    for p in paths:
        open(p, "wb").write(b"x" * 30000)
    d = DSP.Dispatcher(paths)
    try:
        md = ((P.MAX_RECEIVE_KEY, str(DSP.REPLY_MARGIN + 100000)),)
        r = d.request_jobs(P.JobsRequest(cores=0), _Ctx("a", md))     # all 8 asked for
        assert len(r.jobs) == 3                                       # 3 x (30000 + 64) fit
        assert len(r.SerializeToString()) < DSP.REPLY_MARGIN + 100000
        r2 = d.request_jobs(P.JobsRequest(cores=0), _Ctx("b"))        # default 4 MiB: the rest
        assert len(r2.jobs) == 5 and not d.files
    finally:
        d.close()


def test_unreadable_and_undeliverable_paths_count_as_finished(tmp_path):
    """An unreadable path, or one larger than the server's own send limit, is finished (failed);
    one that is only larger than the asking worker's receive limit stays queued for a worker
    with a larger limit (--max-receive-mb)."""
    good = tmp_path / "good"
    good.write_bytes(b"2020-01-01,1,1,1,1,1\n")
    big = tmp_path / "big"
    big.write_bytes(b"y" * 5000)
    huge = tmp_path / "huge"
    huge.write_bytes(b"z" * 20000)
    paths = [str(tmp_path / "missing"), str(huge), str(good), str(big)]
    d = DSP.Dispatcher(paths, max_reply_bytes=10000)
    try:
        md = ((P.MAX_RECEIVE_KEY, str(DSP.REPLY_MARGIN + 1000)),)
        r = d.request_jobs(P.JobsRequest(cores=0), _Ctx("a", md))
        assert [d.job_paths[j.id] for j in r.jobs] == [str(good)]
        assert sorted(d.failed_paths) == sorted([str(tmp_path / "missing"), str(huge)])
        assert d.files == [str(big)]
        r2 = d.request_jobs(P.JobsRequest(cores=0), _Ctx("a", md))   # big cannot reach "a"...
        assert len(r2.jobs) == 0 and d.files == [str(big)] and d.oversize_skips == 1
        d.complete_job(P.CompleteRequest(id=r.jobs[0].id, data="ok"), _Ctx("a"))
        assert not d.all_done()
        r3 = d.request_jobs(P.JobsRequest(cores=0), _Ctx("b"))        # ...but reaches "b"
        assert [d.job_paths[j.id] for j in r3.jobs] == [str(big)] and not d.files
        d.complete_job(P.CompleteRequest(id=r3.jobs[0].id, data="ok"), _Ctx("b"))
        assert d.all_done()                                           # --exit-when-done ends
    finally:
        d.close()


def test_failed_complete_job_is_retried_until_the_dispatcher_is_done(tmp_path):
    """A CompleteJob RPC that fails is kept and retried with backoff (dropping it would leave
    the job in flight forever and --exit-when-done would never end)."""
    import grpc
    p = tmp_path / "f0"
    p.write_bytes(b"2020-01-01,1,1,1,1,1\n")
    d = DSP.Dispatcher([str(p)])
    calls = {"n": 0}

    def flaky(req):
        calls["n"] += 1
        if calls["n"] == 1:
            raise grpc.RpcError("transient")
        return d.complete_job(req, _Ctx("w"))
    w = WK.Worker("127.0.0.1:1", lambda jobs: ["ok"] * len(jobs), cores=1)
    w.retry_base_s = 0.02
    w._complete = flaky
    try:
        r = d.request_jobs(P.JobsRequest(cores=1), _Ctx("w"))
        WK.process_incoming_job(r, w.complete_q, w.processor)
        t0 = time.time()
        while not d.all_done() and time.time() - t0 < 5:
            w._send_completions()
        assert d.all_done() and calls["n"] == 2 and not w._retry
    finally:
        w.channel.close()
        d.close()


def test_pending_retries_get_a_last_attempt_and_a_log_on_stop(caplog):
    """completions waiting for a retry when the worker stops get one last attempt;
    what still fails is logged with its job ids instead of vanishing."""
    import grpc
    import logging
    sent = []
    timeouts = []

    def down(req, timeout=None):
        timeouts.append(timeout)  # the last attempts are bounded
        if req.id == "j1":
            sent.append(req.id)
            return None
        raise grpc.RpcError("server down")
    w = WK.Worker("127.0.0.1:1", lambda jobs: ["ok"] * len(jobs), cores=1)
    w._complete = down
    try:
        w._retry = [("j1", "ok", time.monotonic() + 60, 3), ("j2", "ok", time.monotonic() + 60, 3)]
        w.complete_q.put(("j3", "ok"))
        with caplog.at_level(logging.WARNING):
            w._flush_retries()
        assert sent == ["j1"] and not w._retry
        # one deadline for the whole flush: every attempt gets what is left of it
        assert len(timeouts) == 3 and w.flush_timeout_s > 0
        assert all(0 < t <= w.flush_timeout_s for t in timeouts) and timeouts == sorted(timeouts, reverse=True)
        assert "2 completions undelivered" in caplog.text and "j2" in caplog.text and "j3" in caplog.text
    finally:
        w.channel.close()


def test_flush_stops_at_the_first_deadline(caplog):
    """a hung dispatcher costs the shutdown one deadline, not one per completion:
    after DEADLINE_EXCEEDED the remaining completions are logged as lost without an attempt."""
    import grpc
    import logging

    class Hung(grpc.RpcError):
        def code(self):
            return grpc.StatusCode.DEADLINE_EXCEEDED
    calls = []

    def hung(req, timeout=None):
        calls.append(req.id)
        raise Hung()
    w = WK.Worker("127.0.0.1:1", lambda jobs: ["ok"] * len(jobs), cores=1)
    w._complete = hung
    try:
        for i in range(5):
            w.complete_q.put((f"j{i}", "ok"))
        with caplog.at_level(logging.WARNING):
            w._flush_retries()
        assert calls == ["j0"]
        assert "5 completions undelivered" in caplog.text and "j4" in caplog.text
    finally:
        w.channel.close()


def test_status_keeps_a_peer_alive():
    """SendStatus from a known peer refreshes its last connection (a throttled fetcher's
    keep-alive), so the health thread does not prune it and re-dispatch its jobs."""
    d = DSP.Dispatcher([], prune_after_s=3600)
    try:
        d.peers["w"] = {"status": P.IDLE, "last_connection": 0.0}
        d.send_status(P.StatusRequest(status=P.RUNNING), _Ctx("w"))
        assert time.time() - d.peers["w"]["last_connection"] < 5
        d.send_status(P.StatusRequest(status=P.RUNNING), _Ctx("stranger"))
        assert "stranger" not in d.peers                 # main.rs:80-102: no upsert on status
    finally:
        d.close()


def test_file_above_every_workers_limit_is_dropped_after_repeated_skips(tmp_path):
    """a file within the server's send limit but above every connected worker's
    receive limit is dropped (failed, logged) after oversize_drop_after skips instead of being
    requeued forever, so all_done() (--exit-when-done) still becomes true."""
    big = tmp_path / "big"
    big.write_bytes(b"y" * 5000)
    d = DSP.Dispatcher([str(big)], max_reply_bytes=10000, oversize_drop_after=3)
    try:
        md = ((P.MAX_RECEIVE_KEY, str(DSP.REPLY_MARGIN + 1000)),)
        for n in (1, 2):
            r = d.request_jobs(P.JobsRequest(cores=0), _Ctx("a", md))
            assert len(r.jobs) == 0 and d.files == [str(big)] and not d.all_done(), n
        r = d.request_jobs(P.JobsRequest(cores=0), _Ctx("a", md))
        assert len(r.jobs) == 0 and not d.files and d.failed_paths == [str(big)]
        assert d.all_done()
    finally:
        d.close()


def test_oversize_file_waits_while_a_larger_worker_is_connected(tmp_path):
    big = tmp_path / "big"
    big.write_bytes(b"y" * 5000)
    d = DSP.Dispatcher([str(big)], max_reply_bytes=10000, oversize_drop_after=2)
    try:
        md = ((P.MAX_RECEIVE_KEY, str(DSP.REPLY_MARGIN + 1000)),)
        d.request_jobs(P.JobsRequest(cores=5), _Ctx("b"))            # "b" (4 MiB) takes it...
        d.files.append(str(big))                                     # ...say it was lost
        for _ in range(4):
            r = d.request_jobs(P.JobsRequest(cores=0), _Ctx("a", md))
            assert len(r.jobs) == 0 and d.files == [str(big)]         # "b" could still take it
    finally:
        d.close()

