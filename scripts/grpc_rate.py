"""Transport ceiling of the Python gRPC counterparts, engine excluded: one RequestJobs-shaped
unary call per message over 127.0.0.1, (a) payload bytes pre-serialized (grpcio core only) and
(b) a JobsReply of DBXCOL1-sized jobs built and parsed with the proto runtime (what
dispatcher.py / worker.py do). Prints one JSON line.
  python scripts/grpc_rate.py [--mb 60] [--jobs 5] [--calls 3]"""
import argparse
import json
import os
import sys
import time
from concurrent import futures

import grpc

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbx_amd import proto as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=60, help="message size (the dispatcher's default reply cap)")
    ap.add_argument("--jobs", type=int, default=5, help="jobs per JobsReply (11.8 MB config-5 payloads)")
    ap.add_argument("--calls", type=int, default=3)
    a = ap.parse_args()
    size = a.mb << 20
    blob = os.urandom(size)
    job = blob[: size // a.jobs]
    ident = lambda b: b  # noqa: E731
    ser = lambda m: m.SerializeToString()  # noqa: E731
    handlers = {
        "RequestJobs": grpc.unary_unary_rpc_method_handler(
            lambda r, c: blob, request_deserializer=ident, response_serializer=ident),
        "SendStatus": grpc.unary_unary_rpc_method_handler(
            lambda r, c: P.JobsReply(jobs=[P.Job(id="%036d" % i, File=job) for i in range(a.jobs)]),
            request_deserializer=ident, response_serializer=ser),
    }
    opts = [("grpc.max_send_message_length", 1 << 30), ("grpc.max_receive_message_length", 1 << 30)]
    srv = grpc.server(futures.ThreadPoolExecutor(4), options=opts)
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(P.SERVICE, handlers),))
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    ch = grpc.insecure_channel(f"127.0.0.1:{port}", options=opts)
    raw = ch.unary_unary(P.method_path("RequestJobs"), request_serializer=ident, response_deserializer=ident)
    # the second method carries a proto-built JobsReply (method name reused: only shapes matter)
    msg = ch.unary_unary(P.method_path("SendStatus"), request_serializer=ident,
                         response_deserializer=P.JobsReply.FromString)
    out = {"message_mb": a.mb, "jobs_per_reply": a.jobs, "cpus": os.cpu_count()}
    for name, call in (("raw_bytes", raw), ("jobs_reply_proto", msg)):
        best = None
        for _ in range(a.calls):
            t = time.perf_counter()
            call(b"")
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        out[name + "_GBps"] = size / best / 1e9
    t = time.perf_counter()
    s = P.JobsReply(jobs=[P.Job(id="%036d" % i, File=job) for i in range(a.jobs)]).SerializeToString()
    t1 = time.perf_counter()
    P.JobsReply.FromString(s)
    t2 = time.perf_counter()
    out["proto_build_serialize_GBps"] = size / (t1 - t) / 1e9
    out["proto_parse_GBps"] = size / (t2 - t1) / 1e9
    srv.stop(0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
