"""VGPR / AGPR / spill / scratch per kernel of a hipcc -S device assembly file (its amdhsa metadata).

    python tools/spills.py /tmp/asm/fix3256.s [name-filter]
"""
import re
import subprocess
import sys

text = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
meta = text[text.index("amdhsa.kernels:"):]
rows = []
for blk in re.split(r"\n  - ", meta)[1:]:
    kv = dict(re.findall(r"^\s*\.(\w+):\s+(\S.*)$", blk, re.M))
    if "name" not in kv:
        continue
    rows.append((kv["name"], int(kv.get("vgpr_count", 0)), int(kv.get("agpr_count", 0)),
                 int(kv.get("vgpr_spill_count", 0)), int(kv.get("private_segment_fixed_size", 0))))
names = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True, text=True).stdout.split("\n")
print(f"{'vgpr':>5} {'agpr':>5} {'spill':>6} {'scratch':>8}  kernel")
for r, nm in sorted(zip(rows, names), key=lambda x: x[1]):
    if flt in nm:
        print(f"{r[1]:5d} {r[2]:5d} {r[3]:6d} {r[4]:8d}  {nm.replace('irm::', '').replace('(KParams)', '')}")
