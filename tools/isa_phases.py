"""Static instruction counts between the IRM_STAMP phase markers of one kernel (build with
-DIRM_ISA_MARKS, which turns the stamps into assembly comments):

    hipcc ... -DIRM_ISA_MARKS -DIRM_INST_FIX_D=3 -DIRM_INST_FIX_N=128 --cuda-device-only -S -o k.s irm_opt_inst.hip
    python tools/isa_phases.py k.s '_ZN3irm6k_leanINS_8FixShapeILi3ELi128ELi32EEELi512ELi1ELb1ELi0EEEvNS_7KParamsE'
"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split("\n")
want = sys.argv[2] + ":"
st = next(i for i, l in enumerate(L) if l.startswith(want))
en = next(j for j in range(st, len(L)) if L[j].startswith(".Lfunc_end"))
seg = collections.OrderedDict()
cur = "prologue"
seq = []


def cls(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "bar"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith("s_"):
        return "salu"
    return "mem"


for l in L[st:en]:
    m = re.search(r"IRM_PHASE (\d+)", l)
    if m:
        cur = "P" + m.group(1)
        seq.append(cur)
        continue
    t = l.strip()
    if not t or t.startswith((".", ";", "//")) or t.endswith(":"):
        continue
    seg.setdefault(cur, collections.Counter())[cls(t.split()[0])] += 1
print("marker order:", " ".join(seq))
for k, v in seg.items():
    print(f"{k:9s} total {sum(v.values()):5d}  " + "  ".join(f"{c} {n}" for c, n in sorted(v.items())))
