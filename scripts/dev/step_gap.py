"""Config-2 step time with and without the engine's per-kernel timing events (dev probe): the same
pipelined loop as bench.py (issue i+1, then read back i), 40 timed steps after 5 warm-up."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import dbx_amd as D  # noqa: E402

grid = D.config2_grid()
for rep in range(2):
    for timing in (True, False):
        eng = D.Engine(grid, device=0, topk=100, timing=timing)
        eng.load_synthetic(0x5EED, 0, 5000, 2520, D.BT_DAILY)

        def steps(n):
            eng.run(); eng.topk_fetch_async(0)
            for i in range(n):
                if i + 1 < n:
                    eng.run(); eng.topk_fetch_async((i + 1) & 1)
                eng.topk_fetch_wait(i & 1)

        steps(5)
        eng.sync()
        t0 = time.perf_counter()
        steps(40)
        eng.sync()
        dt = (time.perf_counter() - t0) / 40
        extra = ""
        if timing:
            kms, n, _ = eng.kernel_timing()
            extra = f" kernel {kms / max(n, 1):.4f} ms"
        print(f"timing events {timing}: {dt * 1e3:.4f} ms per step{extra}", flush=True)
        eng.close()
