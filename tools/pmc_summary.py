"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of a kernel."""
import csv
import glob
import sys
from collections import defaultdict


def summarise(paths, kernel_substr="interval"):
    vals = defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if kernel_substr in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    pats = sys.argv[1:] or ["gpurun_out/*/run_counter_collection.csv"]
    paths = [p for pat in pats for p in glob.glob(pat)]
    for k, v in sorted(summarise(paths).items()):
        print(f"{k:28s} {v:16.1f}")
