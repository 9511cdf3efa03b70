"""Per-dispatch SQ counter means of the optimiser launch (k_lean / k_optimize) from tools/pmc_sq.sh output."""
import csv
import glob
import os
import sys


def main():
    out = sys.argv[1]
    vals = {}
    for path in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = {}
        with open(path) as f:
            for row in csv.DictReader(f):
                if "k_optimize" not in row["Kernel_Name"] and "k_lean" not in row["Kernel_Name"]:
                    continue
                key = (row["Dispatch_Id"], row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        names = {}
        for (d, c), v in per.items():
            names.setdefault(c, []).append(v)
        for c, v in names.items():
            vals[c] = sum(v) / len(v)
    for c in sorted(vals):
        print(f"{c:32s} {vals[c]:16.0f}")


if __name__ == "__main__":
    main()
