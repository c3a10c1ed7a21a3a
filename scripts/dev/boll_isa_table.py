"""VALU of the Bollinger kernel's loops by component, from a hipcc -S listing
built with -gline-tables-only (make asm-g, or the hipcc line in profiles/r06/boll_isa_table.md).

Every VALU instruction of a loop body is attributed by its .loc (the innermost inlined source
line) to a component: the source line's text decides it (hash, accounts, path aggregate, return
sums, entry, exit, level tables, record codec, loop control). Counts are static over each loop's
blocks; the narrow/wide account paths are exclusive (a scalar branch), both are listed.
usage: python scripts/dev/boll_isa_table.py LISTING.s [KERNEL_SUBSTRING]"""
import os
import re
import subprocess
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "distributed-backtesting-exploration_amd", "csrc")
listing = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "boll_tile_kernelILb0ELb0ELb0E"
src = {f: open(os.path.join(CSRC, f)).read().split("\n")
       for f in ("k_tile.hip", "tile_common.h", "device_common.h", "internal.h")}

RULES = [  # (component, file, regex on the source line)
    ("trade hash", "device_common.h", r"trade_mix|0xBF58|z \^ \(z|const uint32_t (lo|hi) = "),
    ("trade hash", "tile_common.h", r"trade_term|a\.h \+="),
    ("accounts (gap/mdd/pnl/expo/ntr)", "tile_common.h", r"."),
    ("path aggregate (sparse table, merges)", "device_common.h", r"agg_|dst_|clz|Dr\[|int4|r\.(mx|mn|dd|du)|max\(|min\("),
    ("return sums (ps1/ps2)", "k_tile.hip", r"ps1|ps2"),
    ("level tables / levels", "k_tile.hip", r"\bPL\[|\bPH\[|\bTL\[|\bTH\[|\brl\b|\brh\b|lev_|XL|XHm1|level_y|levf"),
    ("entry search (ctz of z words)", "k_tile.hip", r"ZL|ZH|bits_from|ctzll\(m\)|np = |acct_open|cur = b"),
    ("exit search (signal / SL-TP / fill)", "k_tile.hip", r"\bsig\b|DP|DN|xlo|xhi|\bhit\b|\bxs\b|\blow\b|\bpx\b|\bqi\b|\bxc\b|x = |cur = x"),
    ("record codec", "k_tile.hip", r"\brec\b|RB\[|nr\b|kind|emit|more"),
    ("z tests (fp64 bracket, int128 settle)", "k_tile.hip", r"Dd|S1d|S2d|\bpd\b|Qd|QH|QL|\blh\b|ztest|kn2|vcmp_gt|writelane|big|small|unc|settle"),
    ("window sums (ring reads)", "k_tile.hip", r"ring_back|r1\[|r2\[|\bWn\b|winreg|dH|dL|P1t|P2t|dp|dn|vcmp_le|vcmp_ge"),
    ("first-passage search", "k_tile.hip", r"first_low|first_high|gt8|alignbit|ld4|LH\[|0xFE|0xFF|__builtin_ctz|kLhTs|kLhSuf|kLhBx"),
    ("level (fp64 floor)", "k_tile.hip", r"level_y|levf|X\[u\]|2147483648"),
    ("table / word stores", "k_tile.hip", r"tab\[|ptab\[|Wd\["),
    ("task grab", "k_tile.hip", r"grab|\bbase\b|\bo = "),
    ("trade path / close", "k_tile.hip", r"seg|\bsp\b|\bst\b|close_trade|acct_close|agg_merge|cxx|cT\["),
]


def component(f, n):
    if f.startswith("__clang_hip_math"):
        return "min/max helpers"
    if f not in src or n <= 0 or n > len(src[f]):
        return "compiler (copies, control)"
    text = src[f][n - 1]
    for comp, rf, rx in RULES:
        if rf == f and re.search(rx, text):
            return comp
    return "loop control / other"


loops = subprocess.run([sys.executable, os.path.join(HERE, "loop_isa.py"), listing, kern, "--lines"],
                       capture_output=True, text=True, check=True).stdout
blocks, cur = [], None
for line in loops.split("\n"):
    m = re.match(r"loop @(\d+) .*own \{([^}]*)\}\s+k_tile\.hip (\S+)", line)
    if m:
        own = dict((k.strip("' "), int(v)) for k, v in (kv.split(":") for kv in m.group(2).split(",")))
        cur = {"at": int(m.group(1)), "own": own, "range": m.group(3), "lines": []}
        blocks.append(cur)
        continue
    m = re.match(r"\s+(\d+) valu\s+(\S+):(\d+)", line)
    if m and cur is not None:
        cur["lines"].append((int(m.group(1)), m.group(2), int(m.group(3))))


def kind(b):
    ks = [n for c, f, n in b["lines"] if f == "k_tile.hip"]
    txt = " ".join(src["k_tile.hip"][n - 1] for n in ks if 0 < n <= len(src["k_tile.hip"]))
    if "sltp_search" in txt or ("ZL" in txt and "acct" in txt) or ("ZL" in txt and "ps1" in txt):
        return "walker trade iteration"
    if "RB[nr" in txt or "rec |=" in txt:
        return "finder iteration"
    if "RB[i" in txt or "kind" in txt:
        return "accountant record"
    if "first_low" in txt or "first_high" in txt or "levf[side" in txt:
        return "level task (2 levels)"
    if "ztest" in txt or "kn2" in txt or "Dd" in txt:
        return "window task (4 k)"
    return None


print("| loop | VALU (static, own) | " + " | ".join(["component: VALU"]) + " |")
print("|---|---|---|")
seen = set()
for b in blocks:
    k = kind(b)
    if k is None or not 30 <= b["own"].get("valu", 0) <= 400:
        continue
    tag = (k, b["own"].get("valu"))
    if tag in seen:
        continue
    seen.add(tag)
    comp = defaultdict(int)
    for c, f, n in b["lines"]:
        comp[component(f, n)] += c
    parts = "; ".join(f"{c} {v}" for c, v in sorted(comp.items(), key=lambda x: -x[1]))
    print(f"| {k} (listing @{b['at']}) | {b['own'].get('valu')} (+{b['own'].get('xlane', 0)} cross-lane) | {parts} |")
