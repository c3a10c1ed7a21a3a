"""Dispatcher counterpart of the reference server (`src/server/main.rs`), for driving the
worker end-to-end (BASELINE config 1) without Rust or protoc. SURVEY.md §8(f) row 3.

Mirrored semantics:
  * Dispatcher{files, peers, jobs_completed}                               main.rs:26-34
  * peer-health thread: every 100 ms drop peers silent for > 10 s          main.rs:39-52, 183-190
  * complete_job records id -> True (and, new here, keeps `data`)          main.rs:66-78
  * send_status updates an existing peer's status only                     main.rs:80-102
  * request_jobs upserts the peer, splits off jobs, reads each file whole,
    assigns a UUIDv4 id, drops unreadable paths                            main.rs:105-147,164-180
  * split_off_n_jobs: None on empty; drain all if n >= len; otherwise
    Vec::split_off(n) — hand out the TAIL [n, len) and keep the first n    main.rs:151-162
  * empty queue: Status::new(Code::Ok, "No more jobs available")           main.rs:139-141
  * replies gzip-compressed                                                main.rs:212
Known reference quirk kept visible, not copied: peers are keyed by the server's own
local_addr (main.rs:84,109); here they are keyed by the client's peer string.

Additions (the reference's known gaps, README.md:80-82):
  * results sink: every CompleteRequest.data is kept and, with `results_path`, appended as one
    JSON line {"id", "path", "data"} (the reference drops `data`, main.rs:70,76);
  * re-dispatch on worker loss: jobs handed to a peer that the health thread prunes (silent
    > 10 s) go back to the queue and are handed out again under new ids; a late completion of
    an old id is still recorded, and each path's first completion wins;
  * `gzip=False` serves uncompressed replies (binary columnar payloads, §8(f) row 1, gain little
    from gzip and its CPU cost would bound a gRPC-fed sweep).
"""
from __future__ import annotations

import argparse
import json
import logging
import threading
import time
import uuid
from concurrent import futures
from typing import Dict, List, NamedTuple, Optional

import grpc

from . import proto as P

log = logging.getLogger("dbx_amd.dispatcher")

DEFAULT_RECEIVE = 4 * 1024 * 1024   # grpcio's (and tonic's) default client receive limit
REPLY_MARGIN = 64 * 1024            # JobsReply framing beyond the payload bytes
JOB_OVERHEAD = 64                   # per Job: UUID string, field tags and lengths


class Job(NamedTuple):  # a JobsReply entry before serialization
    id: str
    File: bytes


class Reply:
    """A JobsReply as (id, File) pairs, serialized straight to wire bytes by
    proto.encode_jobs_reply: building protobuf messages first would copy every payload twice
    more (the message runtime moves ~1 GB/s, a join several)."""
    __slots__ = ("jobs",)

    def __init__(self, jobs: List[Job]):
        self.jobs = jobs

    def SerializeToString(self) -> bytes:
        return P.encode_jobs_reply(self.jobs)


def split_off_n_jobs(files: List[str], n: int) -> Optional[List[str]]:
    """main.rs:151-162, including Vec::split_off's tail semantics."""
    if not files:
        return None
    if n >= len(files):
        out = files[:]
        files.clear()
        return out
    n = max(n, 0)
    tail = files[n:]
    del files[n:]
    return tail


class Dispatcher:
    def __init__(self, paths: List[str], prune_after_s: float = 10.0, check_every_s: float = 0.1,
                 results_path: Optional[str] = None, max_reply_bytes: int = 60 << 20,
                 oversize_drop_after: int = 3):
        self.files = list(paths)
        self.n_paths = len(set(paths))
        self.files_lock = threading.Lock()
        self.peers: Dict[str, dict] = {}
        self.peers_lock = threading.Lock()
        self.jobs_completed: Dict[str, bool] = {}
        self.results: Dict[str, str] = {}      # results sink (the reference ignores data)
        self.job_paths: Dict[str, str] = {}
        self.inflight: Dict[str, tuple] = {}   # id -> (peer, path) until completed
        self.done_paths: Dict[str, str] = {}   # path -> id of its first completion
        self.requeued = 0
        self.oversize_skips = 0  # replies that could not carry their first file (receive limit)
        # a file above every connected worker's receive limit is dropped (failed, logged) after
        # this many such skips, so all_done() / --exit-when-done still finish
        self.oversize_drop_after = oversize_drop_after
        self._oversize_by_path: Dict[str, int] = {}
        self.failed_paths: List[str] = []     # unreadable / undeliverable (counted done)
        self.done_lock = threading.Lock()
        self.results_path = results_path
        # a JobsReply larger than the server's send limit fails after its files left the queue
        # (the reference loses them); replies are capped and the overflow goes back to the queue
        self.max_reply_bytes = max_reply_bytes
        self._sink = open(results_path, "a", encoding="utf-8") if results_path else None
        self._stop = threading.Event()
        self.prune_after_s = prune_after_s
        threading.Thread(target=self._health, args=(check_every_s,), daemon=True).start()

    def _health(self, every):
        while not self._stop.is_set():
            now = time.time()
            lost = []
            with self.peers_lock:
                for addr, peer in list(self.peers.items()):
                    if now - peer["last_connection"] > self.prune_after_s:
                        log.info("Removing addr %s", addr)
                        del self.peers[addr]
                        lost.append(addr)
            if lost:
                self._requeue(set(lost))
            time.sleep(every)

    def _requeue(self, peers):
        with self.done_lock:
            back = [(jid, path) for jid, (peer, path) in self.inflight.items()
                    if peer in peers and path not in self.done_paths]
            for jid, _ in back:
                del self.inflight[jid]
        if back:
            with self.files_lock:
                self.files.extend(path for _, path in back)
            self.requeued += len(back)
            log.info("Re-dispatching %d jobs of lost peers", len(back))

    def all_done(self) -> bool:
        with self.done_lock:
            return len(self.done_paths) >= self.n_paths

    def close(self):
        self._stop.set()
        if self._sink:
            self._sink.close()
            self._sink = None

    # ---- RPC handlers
    def complete_job(self, req, ctx):
        with self.done_lock:
            self.jobs_completed[req.id] = True
            self.results[req.id] = req.data
            self.inflight.pop(req.id, None)
            path = self.job_paths.get(req.id)
            first = path is not None and path not in self.done_paths
            if first:
                self.done_paths[path] = req.id
            if self._sink and first:
                self._sink.write(json.dumps({"id": req.id, "path": path, "data": req.data}) + "\n")
                self._sink.flush()
        return P.CompleteReply()

    def send_status(self, req, ctx):
        with self.peers_lock:
            peer = self.peers.get(ctx.peer())
            if peer is not None:
                peer["status"] = req.status
                # a status from a known peer is a sign of life as well (the reference refreshes
                # only on RequestJobs, main.rs:105-113): a worker connection that is throttled
                # and only keeps alive must not be pruned with jobs it still holds
                peer["last_connection"] = time.time()
        return P.StatusReply()

    def _reply_cap(self, ctx) -> int:
        """Largest reply for this request: the server's own cap, and below the receive limit the
        worker advertised in metadata (grpcio's default 4 MiB when it sent none), less room for
        the message framing (per job: id, tags, lengths)."""
        limit = DEFAULT_RECEIVE
        for key, value in ctx.invocation_metadata() or ():
            if key == P.MAX_RECEIVE_KEY:
                try:
                    limit = int(value)
                except ValueError:
                    pass
        return max(1, min(self.max_reply_bytes, limit - REPLY_MARGIN))

    def _drop_unreadable(self, path):
        """An unreadable path is finished (failed): the reference silently drops it
        (main.rs:170-172); here it is also counted done so all_done() can become true."""
        with self.done_lock:
            if path not in self.done_paths:
                self.done_paths[path] = None
                self.failed_paths.append(path)

    def _no_peer_can_take(self, need: int) -> bool:
        with self.peers_lock:
            return all(need > p.get("cap", 0) for p in self.peers.values())

    def request_jobs(self, req, ctx):
        cap = self._reply_cap(ctx)
        with self.peers_lock:
            self.peers[ctx.peer()] = {"status": P.IDLE, "last_connection": time.time(), "cap": cap}
        with self.files_lock:
            files = split_off_n_jobs(self.files, req.cores)
        if files is None:
            # main.rs:139-141 answers Status::new(Code::Ok, ...) with no body; grpcio cannot send
            # an OK status without a message (it surfaces as UNKNOWN), so the empty queue is an
            # error status here too. Either way the worker ignores it (handlers.rs:59).
            ctx.abort(grpc.StatusCode.NOT_FOUND, "No more jobs available")
        jobs = []
        size = 0
        for i, path in enumerate(files):
            jid = str(uuid.uuid4())
            try:
                with open(path, "rb") as f:
                    data = f.read()
            except OSError:
                self._drop_unreadable(path)
                continue
            need = len(data) + JOB_OVERHEAD
            if need > self.max_reply_bytes:  # no worker can ever receive it from this server
                log.error("%s (%d bytes) exceeds the server's send limit", path, len(data))
                self._drop_unreadable(path)
                continue
            if size + need > cap:
                # too large for what is left of this reply, or for this worker's receive limit
                # altogether: back to the queue, for a later request or a worker with a larger
                # limit (--max-receive-mb) to take; dropped once it has been skipped
                # oversize_drop_after times while no connected worker's limit admits it
                rest = files[i:]
                if not jobs and need > cap:
                    # request_jobs runs on the server's thread pool: both counters under the
                    # files lock, so no count is lost and the drop fires exactly once
                    with self.files_lock:
                        self.oversize_skips += 1
                        n = self._oversize_by_path[path] = self._oversize_by_path.get(path, 0) + 1
                    if n >= self.oversize_drop_after and self._no_peer_can_take(need):
                        log.error("%s (%d bytes) exceeds every connected worker's receive limit "
                                  "after %d requests: dropped", path, len(data), n)
                        self._drop_unreadable(path)
                        rest = files[i + 1:]
                with self.files_lock:
                    self.files.extend(rest)
                break
            size += need
            with self.done_lock:
                self.job_paths[jid] = path
                self.inflight[jid] = (ctx.peer(), path)
            jobs.append(Job(jid, data))
        log.info("Num files to run: %d", len(jobs))
        return Reply(jobs)


def serve(dispatcher: Dispatcher, addr: str = "[::1]:50051", max_send: int = 64 << 20,
          gzip: bool = True, threads: int = 16):
    dispatcher.max_reply_bytes = min(dispatcher.max_reply_bytes, max_send - REPLY_MARGIN)
    ser = lambda m: m.SerializeToString()  # noqa: E731
    handlers = {
        "CompleteJob": grpc.unary_unary_rpc_method_handler(
            dispatcher.complete_job, request_deserializer=P.CompleteRequest.FromString,
            response_serializer=ser),
        "SendStatus": grpc.unary_unary_rpc_method_handler(
            dispatcher.send_status, request_deserializer=P.StatusRequest.FromString,
            response_serializer=ser),
        "RequestJobs": grpc.unary_unary_rpc_method_handler(
            dispatcher.request_jobs, request_deserializer=P.JobsRequest.FromString,
            response_serializer=ser),
    }
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=threads),
                         compression=grpc.Compression.Gzip if gzip else grpc.Compression.NoCompression,
                         options=[("grpc.max_send_message_length", max_send)])
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(P.SERVICE, handlers),))
    port = server.add_insecure_port(addr)
    server.start()
    return server, port


def main(argv=None):
    ap = argparse.ArgumentParser(description="backtest job dispatcher")
    ap.add_argument("paths", nargs="+", help="files (CSV or DBXCOL1 payloads) or directories")
    ap.add_argument("--addr", default="[::1]:50051")  # main.rs:195
    ap.add_argument("--results", default=None, help="append {id, path, data} JSON lines here")
    ap.add_argument("--no-gzip", action="store_true")
    ap.add_argument("--max-send-mb", type=int, default=64)
    ap.add_argument("--exit-when-done", action="store_true")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    import os
    paths = []
    for p in a.paths:
        paths += sorted(os.path.join(p, f) for f in os.listdir(p)) if os.path.isdir(p) else [p]
    d = Dispatcher(paths, results_path=a.results)
    server, _ = serve(d, a.addr, max_send=a.max_send_mb << 20, gzip=not a.no_gzip)
    print("dispatcher serving", flush=True)
    t0 = time.perf_counter()
    try:
        while not (a.exit_when_done and d.all_done()):
            time.sleep(0.01 if a.exit_when_done else 0.1)
        if a.exit_when_done:
            print(f"dispatcher done {len(d.done_paths)} paths in {time.perf_counter() - t0:.3f} s",
                  flush=True)
    finally:
        server.stop(1)
        d.close()


if __name__ == "__main__":
    main()
