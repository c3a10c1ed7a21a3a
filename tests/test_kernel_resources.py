"""Resource checks of the gfx950 code objects inside libbt.so (CPU only: the metadata notes of
the kernels, read with the ROCm LLVM tools).

* No product kernel may use private (scratch) memory: a scratch spill inside a walk loop turned a
  30-instruction iteration into two dependent scratch round trips (the split Bollinger walk's
  first version, round 2), and it happens silently.
* The tile kernels must keep <= 128 VGPRs: two 8-wave blocks per CU (config 4 at 500 symbols
  per GPU) need 4 waves per SIMD.
Parity instantiations (trade lists, test path only: the SMA ones spill a few VGPRs at their 80-VGPR
budget) are exempt from the scratch and spill checks."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed-backtesting-exploration_amd", "libbt.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _kernels():
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf")]
    if not all(os.path.exists(t) for t in tools) or not os.path.exists(LIB):
        pytest.skip("ROCm LLVM tools or libbt.so missing")
    objcopy, bundler, readelf = tools
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([objcopy, "--dump-section", f".hip_fatbin={fat}", LIB], check=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            part = os.path.join(d, f"b{i}.bin")
            open(part, "wb").write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, f"co{i}.o")
            r = subprocess.run([bundler, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                                f"--input={part}", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([readelf, "--notes", co], capture_output=True, text=True).stdout
            name = None
            for line in notes.splitlines():
                line = line.strip()
                if line.startswith(".name:"):
                    name = line.split(":", 1)[1].strip()
                    out.setdefault(name, {})
                elif name and ":" in line:
                    k, v = line.split(":", 1)
                    if k in (".private_segment_fixed_size", ".vgpr_count", ".vgpr_spill_count"):
                        out[name][k[1:]] = int(v)
    if not out:
        pytest.skip("no gfx950 code objects found in libbt.so")
    return out


def _parity(name):
    # template args <PARITY, STAMPS, ...>: the mangled name starts "ILb1E" for parity kernels
    return re.search(r"kernelILb1E", name) is not None


def test_product_kernels_use_no_scratch():
    ks = _kernels()
    assert any("boll_tile_kernel" in n for n in ks) and any("sma_kernel" in n for n in ks)
    bad = {n: k for n, k in ks.items() if not _parity(n) and k.get("private_segment_fixed_size", 0) != 0}
    assert not bad, f"kernels with scratch: {bad}"
    spills = {n: k for n, k in ks.items() if not _parity(n) and k.get("vgpr_spill_count", 0) != 0}
    assert not spills, f"kernels spilling VGPRs: {spills}"


def test_tile_kernels_fit_four_waves_per_simd():
    ks = _kernels()
    for n, k in ks.items():
        if "tile_kernel" in n:
            assert k["vgpr_count"] <= 128, (n, k)
