"""Per wave-round SQ counters of the optimiser launch from a rocprofv3 --pmc CSV (tools/gpu/varab.sh):
counter mean per dispatch ÷ SQ_WAVES ÷ rounds.   python tools/summarize_pmc_round.py DIR [rounds]"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    per = collections.defaultdict(float)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            if "k_lean" not in row["Kernel_Name"] and "k_optimize" not in row["Kernel_Name"]:
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    names = collections.defaultdict(list)
    for (_, c), x in per.items():
        names[c].append(x)
    m = {c: sum(x) / len(x) for c, x in names.items()}
    w = m.get("SQ_WAVES", 1.0)
    for c in sorted(m):
        unit = "  (quad-cycles)" if c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY",
                                           "SQ_ACTIVE_INST_ANY") else ""
        print(f"{c:28s} {m[c]:16.0f}   per wave-round {m[c] / w / rounds:8.1f}{unit}")


if __name__ == "__main__":
    main()
