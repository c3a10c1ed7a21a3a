"""BASELINE's multi-GPU shard shapes at full size on one MI355X (the reference's
only parallelism is file-level job farming, /root/reference/src/server/main.rs:131-143).

* Sharded union: every config's workload run as the contiguous symbol
  shards the N-GPU bench gives its ranks (parallel.shard; small shards split their bars into
  segments automatically), each in its own engine, must equal the single-engine run of the
  whole workload byte for byte — every summary, the merged top-100 (bt_merge_topk, the host
  merge of the exchange) and the summed counters.
* Strong-scaling shards (config 4 on 8 GPUs, config 3 on 2 GPUs: 250 x 98,280 each): the
  automatic bar split runs (>= 2 segments), equals the unsplit kernel over all 250 symbols, and
  every parameter of every symbol matches the C oracle."""
import os

import numpy as np
import pytest

import dbx_amd as D
import orc_ffi as F
from dbx_amd import parallel as PAR
from helpers import compare_summaries

pytestmark = pytest.mark.gpu

SEED, K = 0x5EED, 100
MINUTE_BARS = 98280
# (grid, symbols in total, bars, freq, ranks in BASELINE's multi-GPU line)
WORKLOADS = {
    2: (D.config2_grid, 5000, 2520, D.BT_DAILY, 2),
    3: (D.config3_grid, 500, MINUTE_BARS, D.BT_MINUTE, 2),
    4: (D.config4_grid, 2000, MINUTE_BARS, D.BT_MINUTE, 8),
    5: (D.config5_grid, 10000, 5 * MINUTE_BARS, D.BT_MINUTE, 8),
}


def _threads():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 8
    return max(1, min(16, aff))


def _run(grid, sym0, n, bars, freq, segments=0):
    with D.Engine(grid, topk=K) as e:
        e.set_segments(segments)
        e.load_synthetic(SEED, sym0, n, bars, freq)
        e.run()
        return e.summaries().copy(), e.read_topk().copy(), e.stats(), e.last_segments()


@pytest.mark.parametrize("config", [2, 3, 4, 5])
def test_sharded_union_equals_single_run(config):
    mk, S, bars, freq, world = WORKLOADS[config]
    grid = mk()
    full, top, st, _ = _run(grid, 0, S, bars, freq, segments=1)
    parts, tops, trades, evals, used = [], [], 0, 0, []
    for rank in range(world):
        sym0, n = PAR.shard(S, world, rank)
        got, t, s, g = _run(grid, sym0, n, bars, freq)
        parts.append(got)
        tops.append(t)
        trades += s["trades"]
        evals += s["bar_evals"]
        used.append(g)
    print(f"config {config}: {world} shards, segments per shard {used}")
    assert np.concatenate(parts).tobytes() == full.tobytes(), "sharded union differs"
    merged = D.merge_topk(np.concatenate(tops), K)
    assert merged.tobytes() == top.tobytes(), "merged shard top-k differs from the single run's"
    assert trades == st["trades"] and evals == st["bar_evals"] == S * bars * grid.n_params


@pytest.mark.parametrize("config,world,rank", [(4, 8, 5), (3, 2, 1)])
def test_strong_scaling_shard_full_shape(config, world, rank):
    mk, S, bars, freq, _ = WORKLOADS[config]
    grid = mk()
    sym0, n = PAR.shard(S, world, rank)
    assert n == 250
    with D.Engine(grid, topk=K) as e:
        e.load_synthetic(SEED, sym0, n, bars, freq)
        e.set_segments(0)  # automatic: a 250-symbol shard has fewer blocks than CUs
        e.run()
        split = e.summaries().copy()
        used, refixed = e.last_segments(with_refixed=True)
        st_split = e.stats()
        e.set_segments(1)
        e.run()
        unsplit = e.summaries().copy()
        assert e.last_segments() == 1
        st_unsplit = e.stats()
    print(f"config {config} shard {rank}/{world}: {used} segments, {refixed} blocks re-walked")
    assert used >= 2
    assert split.tobytes() == unsplit.tobytes(), "split shard differs from the unsplit kernel"
    assert st_split["trades"] == st_unsplit["trades"] == int(split["n_trades"].sum())
    sample = list(range(n))  # every symbol of the shard (the oracle's pool: seconds)
    cols = [F.gen(SEED, sym0 + s, bars, 1) for s in sample]
    closes = np.stack([c[3] for c in cols])
    if config == 3:
        orc = F.ema_grid_mt(closes, grid.axes[0], grid.axes[1], grid.band_bps, 98280, _threads())
    else:
        orc = F.boll_grid_mt(np.stack([c[1] for c in cols]), np.stack([c[2] for c in cols]), closes,
                             grid.axes[0], grid.axes[1], grid.k_den, grid.axes[2], grid.axes[3],
                             98280, _threads())
    compare_summaries(split, orc, lambda i: f"config {config} sym {sym0 + i[0]} {grid.param(i[1])}")
