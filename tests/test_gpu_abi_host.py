"""The drop-in boundary driven by a compiled C host (tests/abi_host.c: engine create, one
bt_run_batch per JobsReply, bt_job_out_free, destroy — the sequence INTEGRATION.md gives the Rust
worker, /root/reference/src/worker/process.rs:13-29). Its CompleteRequest.data strings must be
byte-identical to the Python host's for the same jobs."""
import subprocess

import pytest

import dbx_amd as D
from dbx_amd import payload as PL

from test_abi_cpu import build_abi_host


@pytest.mark.gpu
def test_c_host_batch_matches_python_host(tmp_path):
    seed, n, bars = 9, 5, 700
    exe = build_abi_host(tmp_path)
    r = subprocess.run([exe, "run", str(seed), str(n), str(bars)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    got = []
    for block in r.stdout.split("== job ")[1:]:
        head, _, data = block.partition("\n")
        i, _, status, _, length = head.split()
        assert int(i) == len(got) and int(length) == len(data.encode())
        got.append((int(status), data))
    grid = D.Grid.sma([4, 6, 10], [50, 60, 120], annualization=252)
    jobs = [(f"job-{i}", PL.gen_payload(seed, i, bars, D.BT_DAILY)) for i in range(n)]
    with D.Engine(grid) as e:
        want = e.run_batch(jobs)
    assert len(got) == n
    for (gs, gd), (ws, wd) in zip(got, want):
        assert gs == ws == 0
        assert gd == wd
        assert gd.count("\n") == grid.n_params
