"""profiles/<tag>_flops.json from a tools/pmc_flops.sh pass: fp32 flops the optimiser launch issued.

Per dispatch of k_lean / k_optimize (mean over dispatches):
  v_mfma_f32_16x16x4_f32: 16·16·4 MACs = 2048 flops per wave-instruction (SQ_INSTS_MFMA; the kernels
  issue no other MFMA shape);  VALU: 64 lanes × (2 per FMA, 1 per MUL / ADD) per wave-instruction.
Counts are per issued wave-instruction, so masked-off lanes, padding MFMA columns and the packed
pair-halves (v_pk_* counted once) are not corrected for; transcendental ops (v_rcp, v_sin ...) are
reported but not priced as flops.  bench.py compares this issued count with its algorithmic count.
"""
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_lean", "k_optimize")


def main():
    tag, out = sys.argv[1], sys.argv[2]
    extra = sys.argv[3:]
    cfg = extra[extra.index("--config") + 1] if "--config" in extra else "c3"
    per = {}
    for path in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if not any(k in row["Kernel_Name"] for k in KERNELS):
                    continue
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    names = {}
    for (_, c), v in per.items():
        names.setdefault(c, []).append(v)
    mean = {c: sum(v) / len(v) for c, v in names.items()}
    mfma = mean.get("SQ_INSTS_MFMA", 0.0) * 2048.0
    valu = 64.0 * (2.0 * mean.get("SQ_INSTS_VALU_FMA_F32", 0.0) + mean.get("SQ_INSTS_VALU_MUL_F32", 0.0)
                   + mean.get("SQ_INSTS_VALU_ADD_F32", 0.0))
    res = {"round": tag, "config": cfg, "command": "python bench.py --no-cpu-baseline --steps 3 --warmup 1 " + " ".join(extra),
           "dispatches": len(names.get("SQ_WAVES", [])), "counters_per_dispatch": mean,
           "mfma_flops_per_launch": mfma, "valu_flops_per_launch": valu, "flops_per_launch": mfma + valu,
           "formula": "2048 x SQ_INSTS_MFMA + 64 x (2 x VALU_FMA_F32 + VALU_MUL_F32 + VALU_ADD_F32); issued, "
                      "padding and inactive lanes included"}
    os.makedirs(os.path.join(HERE, "profiles"), exist_ok=True)
    with open(os.path.join(HERE, "profiles", f"{tag}_{cfg}_flops.json" if cfg != "c3" else f"{tag}_flops.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
