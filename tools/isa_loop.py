"""Instruction mix of a k_lean kernel's round loop from hipcc -S device assembly (static).

    python tools/isa_loop.py /tmp/asm/fix3128.s '512, 1, true, 0' [--blocks]

The loop is the kernel's outermost loop with the most blocks (the rounds).  Its blocks are split into
the main chain — the loop header up to the latch block that branches back to it, LLVM's placement of
the likely path — and the rest: blocks placed after the latch (the unlikely branches: dense rounds,
large-argument sincos, ...) and the child loops (the generic obstacle-count loops, not taken for 9-12
obstacles).  The main chain still holds some branch-skipped blocks (per-lane endpoint rows, the
lane-0 flag update, the rejected-step exit), so its counts bound a GD single-loop round from above;
the executed per-round counts are the SQ_INSTS_* counters (tools/summarize_pmc_round.py)."""
import collections
import re
import subprocess
import sys

path, want = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
labels = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_ZN3irm\w+:", l)]
names = subprocess.run(["c++filt"], input="\n".join(n for _, n in labels), capture_output=True, text=True).stdout.split("\n")
for (i, n), dn in zip(labels, names):
    if want in dn and "k_lean" in dn:
        start, kname = i, dn
        break
else:
    sys.exit("kernel not found")
end = next(j for j in range(start, len(lines)) if lines[j].startswith(".Lfunc_end"))

# blocks: [label, loop header (depth-1 loop it belongs to) or None, in a child loop?, ops, branch targets]
blocks, cur = [], None
for l in lines[start:end]:
    m = re.match(r"^(\.LBB\w+|; %bb\.\d+):\s*(;.*)?$", l)
    if m:
        name, com = m.group(1), m.group(2) or ""
        if "Loop Header: Depth=1" in com:
            hdr = name[2:]
        else:
            h = re.search(r"Header=(BB\w+) Depth=1", com)
            hdr = h.group(1) if h else (cur[1] if cur and "Parent Loop" in com else None)
        cur = [name, hdr, "Parent Loop" in com or "Depth=2" in com, [], []]
        blocks.append(cur)
        continue
    t = l.strip()
    if cur is None or not t or t.startswith((".", ";", "//")):
        continue
    op = t.split()[0]
    cur[3].append(op)
    if op.startswith(("s_branch", "s_cbranch")):
        cur[4].append(t.split()[1])

loops = collections.defaultdict(list)
for b in blocks:
    if b[1]:
        loops[b[1]].append(b)
hdr = max(loops, key=lambda k: len(loops[k]))
lb = loops[hdr]
latch = max((i for i, b in enumerate(lb) if (".L" + hdr) in b[4]), default=len(lb) - 1)  # (fall-through back edge: the last block)
hot = [b for i, b in enumerate(lb) if i <= latch and not b[2]]
cold = [b for i, b in enumerate(lb) if not (i <= latch and not b[2])]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_pk_"):
        return "valu packed f32"
    if re.match(r"v_(add|sub|subrev|mul|fma|fmac|fmaak|fmamk|max|min|max3|min3)_f32", op):
        return "valu f32 arith"
    if op.startswith(("v_rcp", "v_sqrt", "v_rsq", "v_exp", "v_log", "v_sin", "v_cos")):
        return "valu trans"
    if op.startswith("v_cmp"):
        return "valu compare"
    if op.startswith("v_cndmask"):
        return "valu select"
    if op.startswith("v_mov"):
        return "valu move"
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane")):
        return "valu lane access"
    if "_dpp" in op:
        return "valu dpp"
    if op.startswith("v_"):
        return "valu int / bit"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op == "s_nop":
        return "nop"
    return "salu"


def report(title, bl):
    ops = [op for b in bl for op in b[3]]
    cls = collections.Counter(classify(op) for op in ops)
    valu = sum(v for k, v in cls.items() if k.startswith("valu"))
    print(f"{title}: {len(bl)} blocks, {len(ops)} instructions, VALU {valu} (+ {cls['mfma']} MFMA)")
    for k, v in sorted(cls.items(), key=lambda kv: -kv[1]):
        print(f"    {k:18s} {v:5d}")
    return ops


print(kname)
print(f"round loop {hdr}: {len(lb)} blocks, latch {lb[latch][0]}")
ops = report("main chain (header .. latch, no child loops)", hot)
c = collections.Counter(op for op in ops if op.startswith("v_") and not op.startswith("v_mfma"))
print("  VALU opcodes of the main chain:")
for k, v in c.most_common():
    print(f"    {k:28s} {v:4d}")
report("off the main chain (after the latch, child loops)", cold)
if "--blocks" in sys.argv:
    for b in lb:
        cnt = collections.Counter(classify(op) for op in b[3])
        tag = "hot " if b in hot else "cold"
        print(f"  {tag} {b[0]:12s} " + " ".join(f"{k}={v}" for k, v in sorted(cnt.items())))
