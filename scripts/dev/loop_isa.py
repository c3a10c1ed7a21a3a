"""ISA census of the loops of one kernel in a hipcc -S listing built with -gline-tables-only
(developer aid, VERDICT r5 item 3: VALU per walk iteration by component).

Builds the kernel's control-flow graph from the listing (blocks start at .LBB labels and after
branches), finds the natural loops (back edges to a dominating header), and prints for every
loop its instruction classes and, with --lines, its VALU by source line (.loc of the
instruction: the innermost inlined function's line). Classes: valu (v_*, cross-lane
v_readlane / v_readfirstlane / v_writelane counted apart as xlane), salu, lds (ds_*), vmem,
wait (s_waitcnt), branch. Counts are static: a loop's body holds every path through it (the
paths a uniform branch selects are shown per block with --blocks).
usage: python scripts/dev/loop_isa.py LISTING.s KERNEL_SUBSTRING [--lines] [--blocks]"""
import re
import sys
from collections import defaultdict

path, want = sys.argv[1], sys.argv[2]
show_lines, show_blocks = "--lines" in sys.argv, "--blocks" in sys.argv
text = open(path).read().split("\n")
files = {}
for l in text:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[int(m.group(1))] = (m.group(3) or m.group(2)).split("/")[-1]
start = next(i for i, l in enumerate(text) if re.match(r"^_Z\w*:", l) and want in l)
end = next(i for i in range(start + 1, len(text)) if text[i].startswith(".Lfunc_end"))


def klass(op):
    if op in ("v_readlane_b32", "v_readfirstlane_b32", "v_writelane_b32"):
        return "xlane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op == "s_waitcnt":
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return None


# blocks: [label, [(op, args, src)], succ labels]
blocks, cur, loc = [], None, ("?", 0)
def new_block(label):
    global cur
    cur = {"label": label, "ins": [], "succ": [], "falls": True, "line": None}
    blocks.append(cur)

new_block("<entry>")
for i in range(start + 1, end):
    l = text[i]
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        if cur["ins"] or cur["label"] != "<entry>" or len(blocks) > 1:
            prev = cur
            new_block(m.group(1))
            if prev["falls"]:
                prev["succ"].append(m.group(1))
        else:
            cur["label"] = m.group(1)
        cur["line"] = i + 1
        continue
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        loc = (files.get(int(m.group(1)), m.group(1)), int(m.group(2)))
        continue
    s = l.strip()
    if not s or s.startswith((";", ".")):
        continue
    m = re.match(r"([a-z_0-9]+)\s*(.*)", s)
    if not m:
        continue
    op, args = m.group(1), m.group(2)
    if cur["line"] is None:
        cur["line"] = i + 1
    cur["ins"].append((op, args, loc))
    if op.startswith("s_cbranch") or op == "s_branch":
        tgt = args.split()[0].rstrip(",")
        cur["succ"].append(tgt)
        falls = op != "s_branch"
        prev = cur
        new_block(f"<after {i + 1}>")
        cur["line"] = i + 2
        if falls:
            prev["succ"].append(cur["label"])
        prev["falls"] = False
    elif op in ("s_endpgm", "s_setpc_b64"):
        cur["falls"] = False
        new_block(f"<after {i + 1}>")

blocks = [b for b in blocks if b["ins"] or b["succ"] or b["label"].startswith(".LBB")]
idx = {b["label"]: n for n, b in enumerate(blocks)}
succ = [[idx[s] for s in b["succ"] if s in idx] for b in blocks]
pred = defaultdict(list)
for u, ss in enumerate(succ):
    for v in ss:
        pred[v].append(u)
# dominators (iterative, reverse postorder)
N = len(blocks)
order, seen = [], set()
def dfs(u):
    stack = [(u, iter(succ[u]))]
    seen.add(u)
    while stack:
        v, it = stack[-1]
        nxt = next(it, None)
        if nxt is None:
            order.append(v)
            stack.pop()
        elif nxt not in seen:
            seen.add(nxt)
            stack.append((nxt, iter(succ[nxt])))
dfs(0)
rpo = order[::-1]
pos = {u: n for n, u in enumerate(rpo)}
idom = {0: 0}
def intersect(a, b):
    while a != b:
        while pos[a] > pos[b]:
            a = idom[a]
        while pos[b] > pos[a]:
            b = idom[b]
    return a
changed = True
while changed:
    changed = False
    for u in rpo[1:]:
        ps = [p for p in pred[u] if p in idom]
        if not ps:
            continue
        d = ps[0]
        for p in ps[1:]:
            d = intersect(d, p)
        if idom.get(u) != d:
            idom[u] = d
            changed = True
def dominates(h, u):
    while True:
        if u == h:
            return True
        if u == 0 or u not in idom:
            return False
        u = idom[u]
loops = defaultdict(set)
for u in range(N):
    for h in succ[u]:
        if u in idom and dominates(h, u):
            body, work = {h, u}, [u]
            while work:
                x = work.pop()
                for p in pred[x]:
                    if p not in body and p in idom:
                        body.add(p)
                        work.append(p)
            loops[h] |= body


def census(bs):
    cnt = defaultdict(int)
    for b in bs:
        for op, _, _ in blocks[b]["ins"]:
            k = klass(op)
            if k:
                cnt[k] += 1
    return dict(cnt)


for h in sorted(loops, key=lambda x: blocks[x]["line"] or 0):
    body = loops[h]
    inner = [g for g in loops if g != h and loops[g] < body]
    own = body - set().union(*[loops[g] for g in inner]) if inner else body
    lines = sorted(blocks[b]["line"] or 0 for b in body)
    src = defaultdict(int)
    for b in own:
        for op, _, lc in blocks[b]["ins"]:
            if klass(op) in ("valu", "xlane"):
                src[lc] += 1
    kt = sorted(n for (f, n) in src if f == "k_tile.hip" and n > 0)
    print(f"loop @{blocks[h]['line']} ({len(body)} blocks, listing {lines[0]}-{lines[-1]}, "
          f"{len(inner)} inner): all {census(body)}  own {census(own)}  "
          f"k_tile.hip {kt[0] if kt else '-'}-{kt[-1] if kt else '-'}")
    if show_lines:
        for (f, n), c in sorted(src.items(), key=lambda x: (-x[1], x[0])):
            print(f"      {c:4d} valu  {f}:{n}")
    if show_blocks:
        for b in sorted(own, key=lambda x: blocks[x]["line"] or 0):
            print(f"      block @{blocks[b]['line']} {census([b])} -> {[blocks[s]['line'] for s in succ[b]]}")
