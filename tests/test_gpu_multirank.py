"""bench.py's WORLD_SIZE > 1 branch on the one-GPU box: torchrun starts two
ranks as a child process; both share the GPU, so the launcher's process group is gloo and the
exchange is parallel.exchange — the same byte message bt_exchange_async sends over RCCL, merged
by the same C function bt_exchange_wait calls (bt_exchange_merge). Each rank runs its contiguous
shard through its own engine; with --verify rank 0 then runs every rank's symbols in one engine
and asserts that the exchanged top-100 and the summed counters (bar-evals, trades) equal it.

The reference's only parallelism is whole-file job farming (/root/reference/src/server/main.rs:
131-143); this checks the MI355X replacement's exchange step at world 2."""
import json
import os
import signal
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("config,extra", [
    (2, ["--symbols", "600"]),                    # weak: 2 x 600 symbols
    (3, ["--symbols", "9"]),                      # strong: 9 symbols, ranks of 5 and 4
    (4, ["--symbols", "7"]),                      # strong, Bollinger
    (5, ["--symbols", "3"]),                      # strong, SMA 1,024 params on 491,400 bars
])
def test_torchrun_two_ranks_exchange_equals_single_engine(config, extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", str(config), "--steps", "2",
           "--warmup", "1", "--verify", "--no-cpu-baseline"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="4")
    # its own session: on a timeout the whole group goes (the launcher AND its rank processes,
    # which hold the GPU), not only the launcher
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=ROOT,
                         env=env, start_new_session=True)
    try:
        out, err = p.communicate(timeout=110)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        raise
    assert p.returncode == 0, err[-3000:]
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    # per-rank attribution of a scaling loss
    pr = d["per_rank"]
    assert len(pr["kernel_avg_ms"]["by_rank"]) == 2 and pr["kernel_avg_ms"]["min"] > 0
    assert len(pr["host_wait_ms_per_step"]["by_rank"]) == 2
    # two steps in flight at N > 1; the gloo exchange proper is timed apart from the GPU wait
    #  and is a small share of the step
    assert pr["pipeline_depth"] == 2 and pr["ranks_share_device"]
    step_ms = d["ms_per_step"]
    assert 0 <= pr["exchange_ms_per_step"]["max"] < step_ms
    assert sum(pr["symbols"]) == d["config"]["symbols_total"]
    assert "gloo all-gather" in d["config"]["parallelism"], d["config"]["parallelism"]
    v = d["verified_exchange"]
    assert v["topk"] == 100 and v["symbols"] == d["config"]["symbols_total"]
    assert v["bar_evals"] == d["config"]["symbols_total"] * d["config"]["bars"] * d["config"]["params"]
