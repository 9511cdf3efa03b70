"""Static instruction mix of a kernel's optimiser loop from hipcc -S device assembly: the code between
the loop's s_setprio (the start of the rounds) and the kernel end, by instruction class, plus the
lines with IRM_STAMP-free region markers if present.

    python tools/isa_loop.py /tmp/asm/fix3128.s '512, 1, true, 0'
"""
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
        start = i
        break
else:
    sys.exit("kernel not found")
end = next(j for j in range(start, len(lines)) if lines[j].startswith(".Lfunc_end"))
body = lines[start:end]
k0 = next(j for j, l in enumerate(body) if "s_setprio 1" in l)
loop = body[k0:]
ins = []
for l in loop:
    t = l.strip()
    if not t or t.startswith((".", ";", "//")) or t.endswith(":"):
        continue
    ins.append(t.split()[0])
cls = collections.Counter()
for op in ins:
    if op.startswith("v_mfma"):
        cls["mfma"] += 1
    elif op.startswith("v_pk_"):
        cls["valu_packed"] += 1
    elif op.startswith(("v_accvgpr",)):
        cls["accvgpr"] += 1
    elif op.startswith("v_"):
        cls["valu"] += 1
    elif op.startswith("s_waitcnt"):
        cls["waitcnt"] += 1
    elif op.startswith(("s_barrier",)):
        cls["barrier"] += 1
    elif op.startswith(("s_cbranch", "s_branch")):
        cls["branch"] += 1
    elif op.startswith("s_"):
        cls["salu"] += 1
    elif op.startswith("ds_"):
        cls["lds"] += 1
    elif op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        cls["vmem"] += 1
    else:
        cls["other:" + op] += 1
print(f"{len(ins)} static instructions after s_setprio: " + ", ".join(f"{k} {v}" for k, v in cls.most_common()))
c = collections.Counter(op for op in ins if op.startswith("v_"))
print("top VALU opcodes:", ", ".join(f"{k} {v}" for k, v in c.most_common(40)))
