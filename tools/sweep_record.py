"""Sweep GPU-utilisation record: from a rocprofv3 ``--kernel-trace --stats`` summary of the bench's
sweep block and the bench's JSON line, write {wall time, GPU kernel time, busy fraction, the top
kernels with their share} for bench.py to attach to BENCH.sweep / BENCH.dual_sweep while the
solver and evaluator sources are unchanged (hash).

    python tools/sweep_record.py --stats gpurun_out/sprof/.../kernel_stats.csv \
        --bench gpurun_out/sweep_ap2_prof.log --arch ap2 --out profiles/r05/sweep/sweep_profile_ap2.json
"""
import argparse
import csv
import hashlib
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOLVER_SOURCES = ["awebox_amd/ipm.py", "awebox_amd/btd.py", "awebox_amd/batched_lu.py", "awebox_amd/csrc/batched_lu.hip",
                  "awebox_amd/sweep.py", "awebox_amd/trajectory.py", "awebox_amd/homotopy.py"]
EVAL_SOURCES = {"ap2": ["awebox_amd/csrc/awegpu.hip", "awebox_amd/csrc/ap2_model.hpp", "awebox_amd/csrc/ap2_tables.hpp"],
                "dual": ["awebox_amd/csrc/awedual.hip", "awebox_amd/csrc/dual_model.hpp", "awebox_amd/csrc/dual_tables.hpp",
                         "awebox_amd/csrc/dual_hess_tables.hpp", "awebox_amd/dual_homotopy.py"]}


def sources_hash(arch: str) -> str:
    h = hashlib.sha256()
    for rel in SOLVER_SOURCES + EVAL_SOURCES[arch]:
        with open(os.path.join(ROOT, rel), "rb") as fh:
            h.update(rel.encode() + fh.read())
    return h.hexdigest()[:16]


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if "(" in name else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--bench", required=True, help="the bench log whose JSON line holds the sweep block")
    ap.add_argument("--arch", choices=["ap2", "dual"], required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--top", type=int, default=8)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.stats)))
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    line = None
    for ln in open(args.bench):
        ln = ln.strip()
        if ln.startswith("{") and '"metric"' in ln:
            line = json.loads(ln)
    key = "sweep" if args.arch == "ap2" else "dual_sweep"
    blk = line[key]
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    top = [{"kernel": short(r["Name"]), "calls": int(r["Calls"]), "total_s": float(r["TotalDurationNs"]) * 1e-9,
            "avg_ms": float(r["AverageNs"]) * 1e-6, "share_of_gpu_time": float(r["TotalDurationNs"]) / total_ns}
           for r in rows[:args.top]]
    rec = {"arch": args.arch, "points_per_gpu": blk["points_per_gpu"], "wall_s": blk["wall_s"],
           "trials_per_s": blk["value"], "gpu_kernel_s": total_ns * 1e-9,
           "gpu_busy_frac": total_ns * 1e-9 / blk["wall_s"], "launches": sum(int(r["Calls"]) for r in rows),
           "top_kernels": top, "source_hash": sources_hash(args.arch),
           "stats_file": os.path.relpath(args.stats, ROOT),
           "note": "rocprofv3 --kernel-trace --stats of the bench run with only this sweep block (plus one "
                   "small evaluation step); GPU busy = summed kernel time / the sweep's wall time (an upper "
                   "bound: the few kernels outside the sweep block are included)"}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps({k: rec[k] for k in ("wall_s", "gpu_kernel_s", "gpu_busy_frac")}), top[0])


if __name__ == "__main__":
    main()
