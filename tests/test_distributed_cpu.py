"""The N>1 path on CPU: world_size-2 gloo processes run the shard -> local top-k -> all-gather
-> merge exchange of dbx_amd.parallel and must reproduce the single-process global top-k.

Per-rank results come from the C oracle (test infrastructure) because this container has no
GPU; on the box the same functions carry engine results over RCCL (bench.py)."""
import os
import socket

import numpy as np
import pytest

import dbx_amd as D
from dbx_amd import parallel as PAR

S, BARS, K = 23, 300, 17
FAST, SLOW = np.array([4, 8, 12], np.int32), np.array([30, 50], np.int32)


def _all_results(sym_ids):
    import orc_ffi as F
    closes = np.stack([F.gen(7, int(s), BARS, 0)[3] for s in sym_ids])
    res = F.sma_grid_mt(closes, FAST, SLOW, 252, 2)
    recs = np.zeros(res.size, D.TOPK_DTYPE)
    P = res.shape[1]
    recs["sharpe"] = res["sharpe"].reshape(-1)
    recs["pnl"] = res["pnl"].reshape(-1)
    recs["sym"] = np.repeat(np.asarray(sym_ids), P)
    recs["param"] = np.tile(np.arange(P), len(sym_ids))
    return recs


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        begin, count = PAR.shard(S, world, rank)
        local = _all_results(range(begin, begin + count))
        local_top = D.merge_topk(local, K)
        top = PAR.gather_topk(local_top, K, dist)
        tot = PAR.allreduce_counters([count, len(local)], dist)
        # bench.py's single-collective form: same merge, same sums
        top2, tot2 = PAR.exchange(local_top, K, [count, len(local)], dist)
        assert top2.tolist() == top.tolist() and tot2 == tot
        # ... and its asynchronous form, two in flight at once as bench.py keeps them (the
        # second message is the first with its counters doubled)
        p1 = PAR.exchange_async(local_top, K, [count, len(local)], dist)
        p2 = PAR.exchange_async(local_top, K, [2 * count, 2 * len(local)], dist)
        top3, tot3 = p1.wait()
        top4, tot4 = p2.wait()
        assert top3.tolist() == top.tolist() and tot3 == tot
        assert top4.tolist() == top.tolist() and tot4 == [2 * x for x in tot]
        q.put((rank, top.tolist(), tot))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_topk_equals_global(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = D.merge_topk(_all_results(range(S)), K).tolist()
    for rank, top, tot in out:
        assert top == expect, rank
        assert tot == [S, S * len(FAST) * len(SLOW)]


def test_shard_covers_every_symbol_once():
    for n in (1, 7, 5000, 10000):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                b, c = PAR.shard(n, world, r)
                got += list(range(b, b + c))
            assert got == list(range(n))


class _FakeComm:
    """Stands in for engine.Comm in the failure tests (no GPU here): rank 0 has an id, rank
    `fail_rank` cannot join."""
    fail_rank = -1
    closed = False

    @staticmethod
    def unique_id():
        return b"\0" * 128

    def __init__(self, uid, rank, world, device, k):
        if rank == _FakeComm.fail_rank:
            raise RuntimeError(f"rank {rank} cannot join")

    def close(self):
        _FakeComm.closed = True


def _comm_worker(rank, world, port, q, mode):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "tests")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from dbx_amd import engine as E
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        if mode == "no_id":      # rank 0 cannot produce the RCCL unique id
            def no_id():
                raise E.BtError("RCCL is not loadable")
            E.Comm.unique_id = staticmethod(no_id)
        else:                    # the last rank cannot join the communicator
            _FakeComm.fail_rank = world - 1
            E.Comm = _FakeComm
        try:
            PAR.make_comm(dist, 0, 5)
            q.put((rank, "ok", False))
        except E.BtError as e:
            q.put((rank, str(e), _FakeComm.closed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["no_id", "join_fails"])
def test_make_comm_fails_on_every_rank_together(mode):
    """bench.py falls back to the torch.distributed exchange when the C-ABI communicator cannot
    be made; every rank must reach that decision (a rank left waiting in the id broadcast or in
    the communicator's join would hang the run)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = "no RCCL unique id on rank 0" if mode == "no_id" else "not created on every rank"
    for rank, msg, closed in out:
        assert want in msg, (rank, msg)
        if mode == "join_fails" and rank < world - 1:
            assert closed, rank  # the ranks that had joined released their communicator
