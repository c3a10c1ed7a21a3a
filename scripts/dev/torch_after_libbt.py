"""Diagnostic: torch's HIP init after libbt.so has created an engine in the same process."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import dbx_amd as D

order = sys.argv[1] if len(sys.argv) > 1 else "libbt-first"
if order == "torch-first":
    import torch
e = D.Engine(D.Grid.sma([3, 5], [20, 30]))
e.load_synthetic(1, 0, 4, 500, D.BT_DAILY)
e.run()
e.close()
import torch  # noqa: E402
print(order, "device_count", torch.cuda.device_count(), flush=True)
for ln in open("/proc/self/maps"):
    if "amdhip64" in ln or "hsa-runtime" in ln:
        print(ln.split()[-1])
s = torch.cuda.Stream(device=0)
print("stream ok", s)
