"""Worker counterpart of the reference (`src/worker/*.rs`) with the HIP engine as its job path.

Reference behaviour mirrored (control plane unchanged; only the job function is new):
  * one compute OS thread fed by a bounded(1024) channel            main.rs:32-42
  * a 250 ms job tick: SendStatus(IDLE) then RequestJobs(cores)      main.rs:68,76-78; handlers.rs:34-64
  * a 1 s status tick: SendStatus(RUNNING) only while PROC_FLAG      main.rs:69,73-75; handlers.rs:14-32
  * completions forwarded as CompleteRequest{id, data}               main.rs:80-83
  * process_incoming_job sets PROC_FLAG, handles the jobs of one
    JobsReply in order, sends one completion per job, clears it      process.rs:13-29
The only change is inside process_incoming_job: instead of `sleep(1000 ms)` per job
(process.rs:23) the whole JobsReply is one batch call into libbt.so (bt_run_batch), and the
completion carries the results string as `data` (the reference sends `data = id`, main.rs:82).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import queue
import threading
import time
from typing import Callable, Optional, Sequence

import grpc

from . import proto as P

log = logging.getLogger("dbx_amd.worker")

# process.rs / main.rs statics
PROC_FLAG = threading.Event()   # main.rs:24 (OnceLock<AtomicBool>)
CONNECTED = threading.Event()   # main.rs:25

# A processor maps [(id, file_bytes)] -> [data_string] (same order). The product processor is
# the HIP engine (engine_processor); tests may plug the C oracle in as a checker.
Processor = Callable[[Sequence[tuple]], Sequence[str]]


class _Merged:  # JobsReplies merged into one engine batch (worker-side batching)
    __slots__ = ("jobs",)

    def __init__(self, jobs):
        self.jobs = jobs


def engine_processor(engine) -> Processor:
    def run(jobs):
        return [data for _status, data in engine.run_batch(jobs)]
    return run


def process_incoming_job(jobs_reply, complete_send: "queue.Queue", processor: Processor) -> None:
    """Drop-in for `process_incoming_job` (process.rs:13-29): PROC_FLAG up, the reply's jobs
    processed (one GPU batch), one (id, data) completion per job in job order, PROC_FLAG down.

    An engine failure (HIP error, BtError) does not end the compute thread: every job of the
    batch completes with one `{"error": ...}` line, as INTEGRATION.md's Rust body does, so the
    dispatcher records the jobs instead of waiting for completions that never come (the
    reference has no retry, README.md:82)."""
    PROC_FLAG.set()
    try:
        jobs = [(j.id, j.File) for j in jobs_reply.jobs]
        if jobs:
            try:
                results = list(processor(jobs))
                if len(results) != len(jobs):
                    raise RuntimeError(f"processor returned {len(results)} results for {len(jobs)} jobs")
            except Exception as why:  # noqa: BLE001 — reported per job, thread stays alive
                log.error("batch of %d jobs failed: %s", len(jobs), why)
                msg = json.dumps({"error": f"engine failure: {why}"}) + "\n"
                results = [msg] * len(jobs)
            for (jid, _), data in zip(jobs, results):
                complete_send.put((jid, data))
    finally:
        PROC_FLAG.clear()


class Worker:
    def __init__(self, target: str, processor: Processor, cores: Optional[int] = None,
                 job_tick: float = 0.250, status_tick: float = 1.0,
                 max_receive: int = 4 * 1024 * 1024, max_batch_bytes: int = 0,
                 min_batch_jobs: int = 0, linger_s: float = 0.2, fetchers: int = 1,
                 max_queued_bytes: int = 0):
        self.target = target
        self.processor = processor
        # handlers.rs:35 reports num_cpus/2; a GPU worker reports its batch capacity instead
        self.cores = cores if cores is not None else max(1, (os.cpu_count() or 2) // 2)
        self.job_tick, self.status_tick = job_tick, status_tick
        self.reply_q: "queue.Queue" = queue.Queue(maxsize=1024)      # main.rs:32
        self.complete_q: "queue.Queue" = queue.Queue(maxsize=1024)   # main.rs:33
        self.stop = threading.Event()
        # GPU-aware batching: the compute thread merges the JobsReplies
        # already queued, up to this many payload bytes, into one engine batch (one launch
        # fills the GPU only with hundreds of symbols); 0 keeps the reference's one reply per
        # call (main.rs:38-42).
        self.max_batch_bytes = max_batch_bytes
        # ... and waits up to `linger_s` for more replies while the batch holds fewer than
        # `min_batch_jobs` symbols (a launch runs one workgroup per symbol: hundreds fill it)
        self.min_batch_jobs, self.linger_s = min_batch_jobs, linger_s
        self.max_receive = max_receive
        # extra fetchers: threads with their own channels (TCP connections) that keep RequestJobs
        # in flight beside the job tick, while fewer than `max_queued_bytes` of replies wait for
        # the compute thread: one grpcio channel moves ~1 GB/s, the engine ingests 100+ GB/s
        self.fetchers = max(1, fetchers)
        self.max_queued_bytes = max_queued_bytes or max(4 * max_batch_bytes, 1 << 30)
        self._queued = 0
        self._qlock = threading.Lock()
        # completions whose CompleteJob failed: (id, data, retry time, attempts)
        self._retry: list = []
        self.retry_base_s, self.retry_max_s = 0.25, 8.0
        # shutdown: how long to wait for the compute thread, and per last CompleteJob attempt
        self.stop_join_s, self.flush_timeout_s = 60.0, 5.0
        self._opts = [("grpc.max_receive_message_length", max_receive)]
        self.channel = grpc.insecure_channel(target, options=self._opts)
        u = self.channel.unary_unary
        ser = lambda m: m.SerializeToString()  # noqa: E731
        self._status = u(P.method_path("SendStatus"), request_serializer=ser,
                         response_deserializer=P.StatusReply.FromString)
        self._request = u(P.method_path("RequestJobs"), request_serializer=ser,
                          response_deserializer=P.JobsReply.FromString)
        self._complete = u(P.method_path("CompleteJob"), request_serializer=ser,
                           response_deserializer=P.CompleteReply.FromString)

    def _put(self, reply):
        with self._qlock:
            self._queued += sum(len(j.File) for j in reply.jobs)
        self.reply_q.put(reply)

    def _take(self, timeout=None):
        reply = self.reply_q.get(timeout=timeout) if timeout is not None else self.reply_q.get_nowait()
        with self._qlock:
            self._queued -= sum(len(j.File) for j in reply.jobs)
        return reply

    def _fetch(self, idx):
        """Extra fetcher `idx` >= 1: RequestJobs on its own connection while the queue has room."""
        ch = grpc.insecure_channel(self.target, options=self._opts + [
            ("grpc.use_local_subchannel_pool", 1), ("dbx.fetcher", idx)])
        ser = lambda m: m.SerializeToString()  # noqa: E731
        req = ch.unary_unary(P.method_path("RequestJobs"), request_serializer=ser,
                             response_deserializer=P.JobsReply.FromString)
        status = ch.unary_unary(P.method_path("SendStatus"), request_serializer=ser,
                                response_deserializer=P.StatusReply.FromString)
        try:
            while not self.stop.is_set():
                with self._qlock:
                    full = self._queued >= self.max_queued_bytes
                if full:
                    # a keep-alive on this connection while throttled: the dispatcher keys peers
                    # by connection, and one silent for its prune window would have the jobs it
                    # still holds in this worker's queue re-dispatched (duplicate GPU work)
                    try:
                        status(P.StatusRequest(status=P.RUNNING))
                    except grpc.RpcError:
                        pass
                    time.sleep(self.job_tick)
                    continue
                try:
                    reply = req(P.JobsRequest(cores=self.cores),
                                metadata=((P.MAX_RECEIVE_KEY, str(self.max_receive)),))
                except grpc.RpcError:  # empty queue / server gone
                    time.sleep(self.job_tick)
                    continue
                self._put(reply)
        finally:
            ch.close()

    # main.rs:38-42 — the compute OS thread
    def _compute(self):
        while not self.stop.is_set():
            try:
                reply = self._take(timeout=0.05)
            except queue.Empty:
                continue
            if self.max_batch_bytes > 0:
                # the replies' Job messages by reference (a merged JobsReply would copy payloads)
                jobs = list(reply.jobs)
                size = sum(len(j.File) for j in jobs)
                while size < self.max_batch_bytes:
                    try:
                        more = self._take(self.linger_s if len(jobs) < self.min_batch_jobs else None)
                    except queue.Empty:
                        break
                    jobs.extend(more.jobs)
                    size += sum(len(j.File) for j in more.jobs)
                reply = _Merged(jobs)
            process_incoming_job(reply, self.complete_q, self.processor)

    # handlers.rs:14-32
    def send_status(self):
        if PROC_FLAG.is_set():
            try:
                self._status(P.StatusRequest(status=P.RUNNING))
            except grpc.RpcError as why:
                log.error("%s", why)

    # handlers.rs:34-64
    def handle_job(self):
        try:
            self._status(P.StatusRequest(status=P.IDLE))
        except grpc.RpcError as why:
            if CONNECTED.is_set():
                log.error("Unable to send status: %s", why)
            CONNECTED.clear()
        try:
            # the receive limit travels as metadata (the proto stays unchanged): the dispatcher
            # caps the reply below it instead of sending one this channel would refuse
            reply = self._request(P.JobsRequest(cores=self.cores),
                                  metadata=((P.MAX_RECEIVE_KEY, str(self.max_receive)),))
        except grpc.RpcError:
            return  # empty queue / server gone: the reference ignores it (handlers.rs:59)
        self._put(reply)

    def run(self, duration: Optional[float] = None):
        CONNECTED.set()
        th = threading.Thread(target=self._compute, daemon=True, name="compute")
        th.start()
        fetch = [threading.Thread(target=self._fetch, args=(i,), daemon=True, name=f"fetch{i}")
                 for i in range(1, self.fetchers)]
        for f in fetch:
            f.start()
        t_end = None if duration is None else time.monotonic() + duration
        next_job = next_status = time.monotonic()
        try:
            while not self.stop.is_set() and (t_end is None or time.monotonic() < t_end):
                now = time.monotonic()
                if now >= next_status:
                    self.send_status()
                    next_status = now + self.status_tick
                if now >= next_job:
                    self.handle_job()
                    next_job = now + self.job_tick
                # main.rs:80-83: a completion is sent as soon as it is ready (the select loop
                # takes ready completions between ticks), so every queued one goes now
                self._send_completions()
        finally:
            self.stop.set()
            # the compute thread finishes its batch first (a GPU batch takes seconds at most),
            # so the flush below sees every completion it produces
            th.join(timeout=self.stop_join_s)
            for f in fetch:
                f.join(timeout=5)
            self._flush_retries()
            if th.is_alive():
                log.warning("Compute thread still running after %.0f s: completions of the batch "
                            "it holds are not delivered by this worker", self.stop_join_s)
            self.channel.close()

    def _flush_retries(self):
        """On stop: one last attempt for every completion still waiting for a retry (and any
        queued one); what still fails is logged with its job id, since the dispatcher re-runs
        those jobs only after it prunes this worker."""
        pending = list(self._retry)
        self._retry = []
        while True:
            try:
                pending.append(self.complete_q.get_nowait() + (0.0, 0))
            except queue.Empty:
                break
        lost = []
        # one deadline for the whole flush (a hung dispatcher must not block the worker's
        # shutdown for flush_timeout_s per completion), and after the first deadline or
        # unavailable error the rest are logged as lost without another attempt
        deadline = time.monotonic() + self.flush_timeout_s
        give_up = False
        for jid, data, _, _ in pending:
            left = deadline - time.monotonic()
            if give_up or left <= 0:
                lost.append(jid)
                continue
            try:
                self._complete(P.CompleteRequest(id=jid, data=data), timeout=left)
            except grpc.RpcError as why:
                lost.append(jid)
                code = why.code() if hasattr(why, "code") else None
                give_up = code in (grpc.StatusCode.DEADLINE_EXCEEDED, grpc.StatusCode.UNAVAILABLE)
        if lost:
            log.warning("Stopping with %d completions undelivered (the dispatcher re-runs them "
                        "once it prunes this worker): %s", len(lost), ", ".join(lost))

    def _send_completions(self):
        """Send every ready completion. One that fails (the reference unwraps and panics here,
        main.rs:80-83, which ends the worker so the server prunes it and its jobs are lost) is
        kept and retried with a capped exponential backoff: the dispatcher keeps the job in
        flight until its completion arrives, so dropping it would leave the run unfinished."""
        now = time.monotonic()
        due = [r for r in self._retry if r[2] <= now]
        self._retry = [r for r in self._retry if r[2] > now]
        try:
            if not due:
                due.append(self.complete_q.get(timeout=0.01) + (now, 0))
            while True:
                while due:
                    jid, data, _, tries = due.pop(0)
                    try:
                        self._complete(P.CompleteRequest(id=jid, data=data))
                    except grpc.RpcError as why:
                        log.error("Unable to complete %s (attempt %d): %s", jid, tries + 1, why)
                        back = min(self.retry_max_s, self.retry_base_s * (2 ** tries))
                        self._retry.append((jid, data, time.monotonic() + back, tries + 1))
                due.append(self.complete_q.get_nowait() + (now, 0))
        except queue.Empty:
            pass


def main(argv=None):
    from .engine import Engine, config2_grid, config3_grid, config4_grid, config5_grid
    ap = argparse.ArgumentParser(description="GPU worker for the backtesting dispatcher")
    ap.add_argument("--target", default="[::1]:50051")            # main.rs:48
    ap.add_argument("--strategy", default="sma", choices=["sma", "ema_ols", "boll"])
    ap.add_argument("--grid", default=None, choices=["config2", "config3", "config4", "config5"],
                    help="a BASELINE config's parameter grid (overrides --strategy)")
    ap.add_argument("--quiet", action="store_true", help="log warnings only")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--cores", type=int, default=None, help="jobs per RequestJobs")
    ap.add_argument("--max-receive-mb", type=int, default=4)
    ap.add_argument("--max-batch-mb", type=int, default=0,
                    help="merge queued JobsReplies into one GPU batch up to this size")
    ap.add_argument("--min-batch-jobs", type=int, default=0,
                    help="linger for more replies while a batch has fewer jobs")
    ap.add_argument("--fetchers", type=int, default=1,
                    help="RequestJobs connections kept busy (1: the reference's job tick only)")
    ap.add_argument("--duration", type=float, default=None)
    ap.add_argument("--job-tick", type=float, default=0.250,
                    help="seconds between RequestJobs on the main connection (main.rs:68)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING if a.quiet else logging.INFO)
    grids = {"config2": config2_grid, "config3": config3_grid, "config4": config4_grid,
             "config5": config5_grid}
    grid = grids[a.grid]() if a.grid else \
        {"sma": config2_grid, "ema_ols": config3_grid, "boll": config4_grid}[a.strategy]()
    eng = Engine(grid, device=a.device)
    print("worker ready", flush=True)
    Worker(a.target, engine_processor(eng), a.cores,
           max_receive=a.max_receive_mb << 20, max_batch_bytes=a.max_batch_mb << 20,
           min_batch_jobs=a.min_batch_jobs, fetchers=a.fetchers, job_tick=a.job_tick).run(a.duration)


if __name__ == "__main__":
    main()
