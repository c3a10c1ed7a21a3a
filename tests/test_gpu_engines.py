"""Engines side by side on one GPU (include/bt.h: one engine per caller thread, bt_config.stream):
an engine launching on a caller-owned stream gives the same bytes as one on its own stream, and
engines driven concurrently from separate host threads (ctypes drops the GIL across each call,
as a worker with several compute threads would) match their serial runs, error text staying
per thread (bt_last_error is thread-local)."""
import threading

import pytest

import dbx_amd as D

pytestmark = pytest.mark.gpu


def _serial(grid, sym0, n_sym, bars):
    with D.Engine(grid) as e:
        e.load_synthetic(0x5EED, sym0, n_sym, bars, D.BT_MINUTE)
        e.run()
        return e.summaries().copy()


def test_engine_on_caller_stream_matches_own_stream():
    import torch
    grid = D.Grid.ema_ols([5, 20, 60], [10, 40, 150], band_bps=10)
    ref = _serial(grid, 3, 20, 9000)
    s = torch.cuda.Stream(device=0)
    with D.Engine(grid, stream=s.cuda_stream) as e:
        e.load_synthetic(0x5EED, 3, 20, 9000, D.BT_MINUTE)
        for _ in range(3):
            e.run()
        got = e.summaries().copy()
    s.synchronize()
    assert got.tobytes() == ref.tobytes()


def test_engines_in_concurrent_threads_match_serial_runs():
    cases = [
        (D.Grid.sma([3, 5, 9, 14], [20, 31, 50]), 0, 40, 5000),
        (D.Grid.ema_ols([5, 20, 60], [10, 40, 150], band_bps=10), 50, 30, 7000),
        (D.Grid.boll([10, 30, 90], [2, 4, 6], [50], [50, 200], k_den=2), 90, 30, 7000),
        (D.config2_grid(), 200, 64, 2520),
    ]
    want = [_serial(*c) for c in cases]
    got = [None] * len(cases)
    errs = []
    start = threading.Barrier(len(cases))

    def work(i):
        grid, sym0, n_sym, bars = cases[i]
        try:
            with D.Engine(grid) as e:
                start.wait()
                out = []
                for r in range(4):
                    # alternate datasets so a run that read another engine's buffers would show
                    e.load_synthetic(0x5EED, sym0 + (r & 1), n_sym, bars, D.BT_MINUTE)
                    e.run()
                    out.append(e.summaries().copy())
                with pytest.raises(D.BtError):  # a refused call reports on this thread only
                    e.set_segments(-1)
                got[i] = out
        except Exception as why:  # noqa: BLE001 — reported by the main thread
            errs.append((i, repr(why)))

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(cases))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    for i, (grid, sym0, n_sym, bars) in enumerate(cases):
        shifted = _serial(grid, sym0 + 1, n_sym, bars)
        for r, out in enumerate(got[i]):
            exp = want[i] if r % 2 == 0 else shifted
            assert out.tobytes() == exp.tobytes(), f"case {i} run {r}"
