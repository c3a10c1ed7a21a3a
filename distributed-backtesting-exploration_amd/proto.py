"""Runtime protobuf descriptors for the reference wire contract — no protoc needed.

Field-for-field restatement of /root/reference/proto/backtesting.proto:1-39 (package
`backtesting`, service `Processor`), kept byte-identical on the wire: this engine is a drop-in
for the worker side only, so the contract must not change (BASELINE.json north_star).
"""
from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_F = descriptor_pb2.FieldDescriptorProto

SERVICE = "backtesting.Processor"
METHODS = {  # proto:23-27
    "CompleteJob": ("CompleteRequest", "CompleteReply"),
    "SendStatus": ("StatusRequest", "StatusReply"),
    "RequestJobs": ("JobsRequest", "JobsReply"),
}


def _file():
    fd = descriptor_pb2.FileDescriptorProto(name="backtesting.proto", package="backtesting",
                                            syntax="proto3")

    def msg(name, *fields):
        m = fd.message_type.add(name=name)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m

    opt, rep = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    msg("JobsRequest", ("cores", 1, _F.TYPE_INT32, opt, None))                      # proto:4-6
    e = fd.enum_type.add(name="WorkerStatus")                                        # proto:8-11
    e.value.add(name="IDLE", number=0)
    e.value.add(name="RUNNING", number=1)
    msg("Job", ("id", 1, _F.TYPE_STRING, opt, None),                                 # proto:13-16
        ("File", 2, _F.TYPE_BYTES, opt, None))
    msg("JobsReply", ("jobs", 1, _F.TYPE_MESSAGE, rep, ".backtesting.Job"))          # proto:18-20
    msg("CompleteRequest", ("id", 1, _F.TYPE_STRING, opt, None),                     # proto:29-32
        ("data", 2, _F.TYPE_STRING, opt, None))
    msg("CompleteReply")                                                             # proto:34
    msg("StatusRequest", ("status", 1, _F.TYPE_ENUM, opt, ".backtesting.WorkerStatus"))  # :36-38
    msg("StatusReply")                                                               # proto:39
    svc = fd.service.add(name="Processor")
    for mname, (req, rep_) in METHODS.items():
        svc.method.add(name=mname, input_type=f".backtesting.{req}", output_type=f".backtesting.{rep_}")
    return fd


_pool = descriptor_pool.DescriptorPool()
_pool.Add(_file())


def _cls(name):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(f"backtesting.{name}"))


JobsRequest = _cls("JobsRequest")
Job = _cls("Job")
JobsReply = _cls("JobsReply")
CompleteRequest = _cls("CompleteRequest")
CompleteReply = _cls("CompleteReply")
StatusRequest = _cls("StatusRequest")
StatusReply = _cls("StatusReply")
IDLE, RUNNING = 0, 1

MESSAGES = {c.DESCRIPTOR.name: c for c in
            (JobsRequest, Job, JobsReply, CompleteRequest, CompleteReply, StatusRequest, StatusReply)}


# gRPC metadata key (not a proto field: the contract stays byte-identical) with which a worker
# tells the dispatcher its max receive size, so JobsReplies are capped below it
MAX_RECEIVE_KEY = "x-dbx-max-receive"


def method_path(name: str) -> str:
    return f"/{SERVICE}/{name}"


def _varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def encode_jobs_reply(jobs) -> bytes:
    """Wire bytes of JobsReply{jobs: [Job{id, File}]} for (id, file_bytes) pairs, identical to
    JobsReply(...).SerializeToString() (proto3: empty fields omitted, fields in number order),
    built with one join: the payload bytes are copied once, not into message objects first."""
    parts = []
    for jid, data in jobs:
        idb = jid.encode("utf-8")
        head = (b"\x0a" + _varint(len(idb)) if idb else b"")
        fhead = (b"\x12" + _varint(len(data)) if data else b"")
        parts.append(b"\x0a" + _varint(len(head) + len(idb) + len(fhead) + len(data)))
        parts += [head, idb, fhead, data]
    return b"".join(parts)
