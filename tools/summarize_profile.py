"""Condense a tools/profile_round.sh run into profiles/<round>_*.

profiles/<round>_kernel_stats.csv  rocprofv3 --stats table (as produced)
profiles/<round>_pmc.json          per-dispatch FETCH_SIZE / WRITE_SIZE of the optimiser kernel and the
                                   corrected HBM bytes (MI355X_MICROARCH.md §HBM: FETCH_SIZE
                                   counts half the bytes of wide streaming reads on gfx950 → ×2)
bench.py reads the newest *_pmc.json for roofline.traffic.
"""
import csv
import glob
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    return hits[0] if hits else None


def counter_rows(path, kernel_subs=("k_lean", "k_optimize")):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if not any(k in row.get("Kernel_Name", "") for k in kernel_subs):
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    tag, out = sys.argv[1], sys.argv[2]
    extra = sys.argv[3:]
    cfg = extra[extra.index("--config") + 1] if "--config" in extra else "c3"
    prof = os.path.join(HERE, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = find(os.path.join(out, "stats"), "*kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    res = {"round": tag, "config": cfg, "faithful": "--faithful" in extra,
           "kernel": "irm::k_lean / irm::k_optimize (the optimiser launch)",
           "command": "python bench.py --no-cpu-baseline --steps 5 --warmup 1 " + " ".join(extra)}
    for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        path = find(os.path.join(out, sub), "*counter_collection.csv")
        if not path:
            continue
        v = counter_rows(path)
        res[name] = {"dispatches": len(v), "mean_kb": sum(v) / max(1, len(v)), "min_kb": min(v) if v else None,
                     "max_kb": max(v) if v else None}
    if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
        fetch_b = res["FETCH_SIZE"]["mean_kb"] * 1024.0
        write_b = res["WRITE_SIZE"]["mean_kb"] * 1024.0
        res["hbm_bytes_per_launch"] = 2.0 * fetch_b + write_b
        res["correction"] = "2 x FETCH_SIZE (gfx950 half-count of wide reads) + WRITE_SIZE; units KB = 1024 B"
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
