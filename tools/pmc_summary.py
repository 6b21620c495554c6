"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch of a kernel.

  python tools/pmc_summary.py 'gpurun_out/*/run_counter_collection.csv'
  python tools/pmc_summary.py --record BATCH 'gpurun_out/*/run_counter_collection.csv'
      also writes profiles/pmc_traffic.json (counters + the kernel-source hash bench.py checks)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summarise(paths, kernel_substr="interval"):
    vals = defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if kernel_substr in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


if __name__ == "__main__":
    args = sys.argv[1:]
    batch = None
    if args and args[0] == "--record":
        batch = int(args[1])
        args = args[2:]
    pats = args or ["gpurun_out/*/run_counter_collection.csv"]
    paths = [p for pat in pats for p in glob.glob(pat, recursive=True)]
    summ = summarise(paths)
    for k, v in sorted(summ.items()):
        print(f"{k:28s} {v:16.1f}")
    if batch is not None:
        sys.path.insert(0, ROOT)
        from bench import kernel_source_hash
        rec = {"batch": batch, "source_hash": kernel_source_hash(),
               "kernel": "ap2_interval_kernel", "units": "FETCH/WRITE_SIZE in kB per dispatch; SQ_* per dispatch",
               "FETCH_SIZE_kB": summ["FETCH_SIZE"], "WRITE_SIZE_kB": summ["WRITE_SIZE"]}
        for k, v in summ.items():
            if k.startswith("SQ_"):
                rec[k] = v
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fh:
            json.dump(rec, fh, indent=1, sort_keys=True)
        print("wrote profiles/pmc_traffic.json")
