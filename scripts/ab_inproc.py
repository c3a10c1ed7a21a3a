"""Interleaved in-process A/B of library builds (profiling aid, cdna_hip_programming.md §5.4
rule 24: compare arms on one device, in one process, alternating). Every build gets its own
engine on the same synthetic shard; rounds alternate A, B, ... and each round times `steps`
back-to-back runs with the engine's HIP events (bt_kernel_timing: the dominant kernel).
The builds' summaries are compared bit for bit after the first round.

usage: python scripts/ab_inproc.py CONFIG SYMBOLS LIB [LIB ...]
       (LIB: in-tree path under the package, e.g. libbt.so dev/e2.so; env ROUNDS, STEPS)"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import dbx_amd as D  # noqa: E402
from dbx_amd import engine as E  # noqa: E402

cfg, S, libs = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3:]
rounds, steps = int(os.environ.get("ROUNDS", 5)), int(os.environ.get("STEPS", 5))
grid = {2: D.config2_grid, 3: D.config3_grid, 4: D.config4_grid, 5: D.config5_grid}[cfg]()
bars = {2: 2520, 3: 98280, 4: 98280, 5: 491400}[cfg]
freq = D.BT_DAILY if cfg == 2 else D.BT_MINUTE
E._one_hip_runtime()
P = C.c_void_p
arms = []
for name in libs:
    L = C.CDLL(os.path.join(E.PKG_DIR, name))
    L.bt_engine_create.argtypes = [C.POINTER(E._Config), C.c_char_p, C.c_size_t]
    L.bt_engine_create.restype = P
    L.bt_load_synthetic.argtypes = [P, C.c_uint64, C.c_int64, C.c_int32, C.c_int32, C.c_int32]
    for f in ("bt_run", "bt_sync", "bt_reset_timing", "bt_engine_destroy"):
        getattr(L, f).argtypes = [P]
    L.bt_kernel_timing.argtypes = [P, C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_char_p)]
    L.bt_read_summaries.argtypes = [P, P, C.c_size_t]
    L.bt_num_params.argtypes = [P]
    conf = grid.to_c(0, 0, D.BT_FLAG_TIMING, 0, 0, None)
    err = C.create_string_buffer(512)
    h = L.bt_engine_create(C.byref(conf), err, 512)
    assert h, err.value
    assert L.bt_load_synthetic(h, 0x5EED, 0, S, bars, freq) >= 0
    arms.append((name, L, h, []))
ref = None
for r in range(rounds):
    for name, L, h, ts in arms:
        L.bt_run(h)
        L.bt_sync(h)
        L.bt_reset_timing(h)
        for _ in range(steps):
            L.bt_run(h)
        L.bt_sync(h)
        ms, n, kn = C.c_double(), C.c_int64(), C.c_char_p()
        L.bt_kernel_timing(h, C.byref(ms), C.byref(n), C.byref(kn))
        ts.append(ms.value / max(n.value, 1))
        if r == 0:
            out = np.zeros(S * grid.n_params, D.SUMMARY_DTYPE)
            assert L.bt_read_summaries(h, out.ctypes.data, out.size) >= 0
            if ref is None:
                ref = out
            elif out.tobytes() != ref.tobytes():
                print(f"{name}: SUMMARIES DIFFER from {arms[0][0]}")
for name, L, h, ts in arms:
    print(f"config {cfg} S {S} {name:16s} kernel ms median {np.median(ts):.4f} min {min(ts):.4f} "
          f"all {[round(x, 4) for x in ts]}")
    L.bt_engine_destroy(h)
