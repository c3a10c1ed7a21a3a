"""Resource checks of the gfx950 code objects inside libbt.so (CPU only: the metadata notes of
the kernels, read with the ROCm LLVM tools).

* No product kernel may touch private (scratch) memory inside a loop: a scratch spill inside a
  walk loop turned a 30-instruction iteration into two dependent scratch round trips (the split
  Bollinger walk's first version, round 2), and it happens silently. The check disassembles
  every kernel and requires each scratch access to lie outside every backward branch's range
  (a value kept from the prologue to the result write, once per workgroup, is tolerated:
  the Bollinger release kernel keeps its parameter index that way at the 128-VGPR edge).
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
    objdump = os.path.join(LLVM, "llvm-objdump")
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
            if os.path.exists(objdump):
                dis = subprocess.run([objdump, "-d", "--mcpu=gfx950", co], capture_output=True, text=True).stdout
                for fname, hot in _scratch_in_loops(dis).items():
                    out.setdefault(fname, {})["scratch_in_loops"] = hot
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


_FUNC = re.compile(r"^[0-9a-f]+ <([^>]+)>:")
_INST = re.compile(r"^\s+(\S+)\s*(.*?)\s*// ([0-9A-F]+):")


def _scratch_in_loops(dis):
    """Per function of an llvm-objdump listing: the scratch accesses that lie inside the range of
    some backward branch (a loop body). Branch targets: address + 4 + 4 * simm16."""
    funcs, cur = {}, None
    for line in dis.splitlines():
        m = _FUNC.match(line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        m = _INST.match(line)
        if m and cur is not None:
            cur.append((int(m.group(3), 16), m.group(1), m.group(2)))
    out = {}
    for name, insts in funcs.items():
        loops = []
        for addr, op, args in insts:
            if (op.startswith("s_cbranch") or op == "s_branch") and args.split()[:1]:
                try:
                    imm = int(args.split()[0])
                except ValueError:
                    continue
                off = imm - 65536 if imm >= 32768 else imm
                tgt = addr + 4 + 4 * off
                if tgt <= addr:
                    loops.append((tgt, addr))
        out[name] = [hex(a) for a, op, _ in insts
                     if op.startswith("scratch_") and any(lo <= a <= hi for lo, hi in loops)]
    return out


def _parity(name):
    # template args <PARITY, STAMPS, ...>: the mangled name starts "ILb1E" for parity kernels
    return re.search(r"kernelILb1E", name) is not None


def test_product_kernels_keep_scratch_out_of_loops():
    ks = _kernels()
    assert any("boll_tile_kernel" in n for n in ks) and any("sma_kernel" in n for n in ks)
    product = {n: k for n, k in ks.items() if not _parity(n) and "private_segment_fixed_size" in k}
    assert all("scratch_in_loops" in k for k in product.values()), "llvm-objdump listing missing"
    hot = {n: k["scratch_in_loops"] for n, k in product.items() if k["scratch_in_loops"]}
    assert not hot, f"scratch accesses inside loops: {hot}"
    # only the Bollinger release kernel may keep a value in scratch at all, and only a few bytes
    big = {n: k["private_segment_fixed_size"] for n, k in product.items()
           if k["private_segment_fixed_size"] > (16 if "boll_tile_kernel" in n else 0)}
    assert not big, f"kernels with scratch: {big}"


def test_tile_kernels_fit_four_waves_per_simd():
    ks = _kernels()
    for n, k in ks.items():
        if "tile_kernel" in n:
            assert k["vgpr_count"] <= 128, (n, k)
