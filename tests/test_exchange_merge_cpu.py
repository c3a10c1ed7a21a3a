"""The host half of the N-GPU exchange (csrc/comm.cpp merge_block, exported as
bt_exchange_merge) on gathered blocks for world sizes 2, 3 and 8: ranks with no records, ranks
with fewer than k, ties on Sharpe across ranks, counts above k_msg (clipped), counter sums. The
expected merge is an independent numpy sort in the engine's order (Sharpe desc, symbol, param).

The reference's only parallelism is job farming over gRPC (/root/reference/src/server/main.rs:
131-143); the exchange replaces nothing there. The world-3 gloo test moves the
byte messages bt_exchange_async sends through a real all-gather and merges them with the same
C function bt_exchange_wait calls, so the world > 1 parse runs on the product code."""
import os
import socket
import subprocess

import numpy as np
import pytest

import dbx_amd as D
from dbx_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _engine_order(recs):
    """Sharpe descending by its orderable bit pattern (internal.h order_key: +0.0 ranks above
    -0.0), then symbol, then param."""
    recs = np.asarray(recs, D.TOPK_DTYPE)
    u = np.ascontiguousarray(recs["sharpe"]).view(np.uint64)
    key = np.where(u >> np.uint64(63), ~u, u | np.uint64(1 << 63))
    idx = np.lexsort((recs["param"], recs["sym"], ~key))
    return recs[idx]


def _rank_records(rng, rank, n, ties):
    """n records of one rank's shard (symbols rank*1000..), sorted in engine order."""
    r = np.zeros(n, D.TOPK_DTYPE)
    r["sharpe"] = rng.choice(ties, n) if len(ties) else rng.normal(size=n)
    r["sym"] = rank * 1000 + rng.integers(0, 50, n)
    r["param"] = rng.permutation(4 * n + 1)[:n]  # distinct (sym, param) pairs within the rank
    r["pnl"] = rng.integers(-10**9, 10**9, n)
    return _engine_order(r)


def _block(parts, k_msg, counters):
    return b"".join(E.exchange_message(p, k_msg, *c) for p, c in zip(parts, counters))


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("ties", [False, True])
def test_exchange_merge_matches_numpy_order(world, ties):
    rng = np.random.default_rng(100 * world + ties)
    k_msg = 100
    tie_vals = np.array([1.5, 0.25, -0.0, 0.0, -2.0]) if ties else np.array([])
    sizes = [int(x) for x in rng.integers(0, k_msg + 1, world)]
    sizes[0] = 0                      # a rank with no records
    sizes[-1] = k_msg                 # a full rank
    if world > 2:
        sizes[1] = 3                  # a rank with n < k
    parts = [_rank_records(rng, r, n, tie_vals) for r, n in enumerate(sizes)]
    counters = [(int(rng.integers(0, 2**40)), int(rng.integers(0, 2**30))) for _ in range(world)]
    block = _block(parts, k_msg, counters)
    assert len(block) == world * E.sym("bt_exchange_message_bytes")(k_msg)
    for k in (1, 7, k_msg, 3 * k_msg):
        got, cnt = E.exchange_merge(block, world, k_msg, k)
        exp = _engine_order(np.concatenate(parts))[:min(k, k_msg)]
        assert len(got) == len(exp)
        for f in ("sharpe", "sym", "param", "pnl"):
            assert np.array_equal(got[f], exp[f]), (k, f)
        assert cnt == [sum(c[0] for c in counters), sum(c[1] for c in counters)]


def test_exchange_merge_all_ranks_empty_and_clipped_counts():
    k_msg = 5
    empty = [np.zeros(0, D.TOPK_DTYPE)] * 3
    got, cnt = E.exchange_merge(_block(empty, k_msg, [(1, 2), (3, 4), (5, 6)]), 3, k_msg, 5)
    assert len(got) == 0 and cnt == [9, 12]
    # a header count above k_msg reads only the k_msg slots the message has
    rng = np.random.default_rng(3)
    full = _rank_records(rng, 0, k_msg, np.array([]))
    msg = bytearray(E.exchange_message(full, k_msg, 10, 1))
    msg[:4] = np.int32(1_000_000).tobytes()
    got, cnt = E.exchange_merge(bytes(msg), 1, k_msg, 50)
    assert len(got) == k_msg and np.array_equal(got["param"], full["param"]) and cnt == [10, 1]


def test_exchange_merge_rejects_a_negative_count():
    msg = bytearray(E.exchange_message(np.zeros(0, D.TOPK_DTYPE), 4, 0, 0))
    msg[:4] = np.int32(-1).tobytes()
    block = E.exchange_message(np.zeros(0, D.TOPK_DTYPE), 4, 0, 0) + bytes(msg)
    with pytest.raises(D.BtError, match="rank 1"):
        E.exchange_merge(block, 2, 4, 4)


def test_exchange_merge_rejects_a_mismatched_block():
    """A short block (a truncated gather) or one built for another k_msg is rejected by the C side
    itself, not read past its end."""
    import ctypes as C
    k_msg = 4
    one = E.exchange_message(np.zeros(0, D.TOPK_DTYPE), k_msg, 0, 0)
    with pytest.raises(D.BtError, match="expected"):
        E.exchange_merge(one * 2 + one[:-1], 3, k_msg, 4)         # Python wrapper check
    with pytest.raises(D.BtError, match="expected"):
        E.exchange_merge(one * 2, 2, k_msg + 1, 4)                # sent with another k
    raw = np.frombuffer(one * 2, np.uint8)
    out = np.zeros(4, D.TOPK_DTYPE)
    cnt = np.zeros(2, np.int64)
    for nbytes in (len(raw) - 1, len(raw) + 8, 0):                 # the C check alone
        rc = E.sym("bt_exchange_merge")(raw.ctypes.data, nbytes, 2, k_msg, out.ctypes.data, 4,
                                        cnt.ctypes.data)
        assert rc == -1 and b"bytes" in E.lib().bt_last_error()
    assert E.sym("bt_exchange_merge")(raw.ctypes.data, len(raw), 2, k_msg, out.ctypes.data, 4,
                                      cnt.ctypes.data) == 0


def test_libbt_does_not_link_rccl():
    """A single-GPU worker loads the engine without RCCL: comm.cpp dlopens it on the first
    communicator call (VERDICT r3 missing #3)."""
    so = os.path.join(ROOT, "distributed-backtesting-exploration_amd", "libbt.so")
    out = subprocess.run(["readelf", "-d", so], capture_output=True, text=True, check=True).stdout
    needed = [l for l in out.splitlines() if "(NEEDED)" in l]
    assert needed and not any("rccl" in l for l in needed), needed


def _gloo_worker(rank, world, port, q):
    import sys
    for p in (ROOT, os.path.join(ROOT, "tests")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    from dbx_amd import engine as E2
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        rng = np.random.default_rng(rank)
        k_msg = 16
        mine = _rank_records(rng, rank, [0, 9, 16][rank], np.array([0.5, 0.25]))
        msg = E2.exchange_message(mine, k_msg, 1000 + rank, 10 + rank)
        t = torch.frombuffer(bytearray(msg), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        block = b"".join(bytes(o.numpy()) for o in outs)
        got, cnt = E2.exchange_merge(block, world, k_msg, k_msg)
        q.put((rank, got.tobytes(), cnt, mine.tobytes()))
    finally:
        dist.destroy_process_group()


def test_exchange_merge_over_gloo_world3():
    import multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 3
    ps = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    mine = np.concatenate([np.frombuffer(r[3], D.TOPK_DTYPE) for r in sorted(res, key=lambda r: r[0])])
    exp = _engine_order(mine)[:16]
    for rank, got, cnt, _ in res:
        got = np.frombuffer(got, D.TOPK_DTYPE)
        assert got.tobytes() == exp.tobytes(), rank
        assert cnt == [3003, 33]
