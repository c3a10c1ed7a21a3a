"""Print vgpr / spill / scratch counts of the tile and SMA kernels inside a libbt build
(developer aid; the same metadata tests/test_kernel_resources.py checks).
usage: python scripts/dev/kernel_res.py [path/to/libbt.so]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import test_kernel_resources as T  # noqa: E402

if len(sys.argv) > 1:
    T.LIB = sys.argv[1]
for name, d in sorted(T._kernels().items()):
    if "tile_kernel" not in name and "sma" not in name:
        continue
    print(f"{name[:70]:70s} vgpr {d.get('vgpr_count')} spill {d.get('vgpr_spill_count')} "
          f"priv {d.get('private_segment_fixed_size')}")
