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


def record_configs(fetch_dir, write_dir, *sq_dirs, only=None, hashes=None):
    """profiles/pmc_traffic_configs.json: FETCH/WRITE_SIZE (and, from further counter directories,
    the SQ_* FP64 / VALU / wave-state counters) per dispatch of the config-3 (dual kites, B = 128)
    and config-5 (tracking MPC, B = 256) interval kernels of tools/pmc_kernels.py.  ``only`` limits
    the update to some kernels (the others keep their entries); ``hashes`` overrides the source
    hash of a kernel (records taken on committed sources that have changed in the tree since)."""
    sys.path.insert(0, ROOT)
    from bench import sources_hash
    path = os.path.join(ROOT, "profiles", "pmc_traffic_configs.json")
    try:
        out = json.load(open(path))
    except (OSError, ValueError):
        out = {}
    # the kernels of one evaluation on the generated instance-minor paths the bench measures
    configs = (("dual", ("transpose_in_kernel", "dual_gen_node_kernel", "dual_gen_interval_kernel",
                         "dual_gen_finalize_kernel"), 128),
               ("mpc", ("transpose_in_kernel", "mpc_gen_node_kernel", "mpc_gen_finalize_kernel"), 256))
    for which, kerns, batch in configs:
        if only is not None and which not in only:
            continue
        rec = {"batch": batch, "kernel": " + ".join(kerns),
               "source_hash": (hashes or {}).get(which) or sources_hash(which),
               "units": "FETCH/WRITE_SIZE in kB, SQ_* counts: per evaluation (the kernels' means per dispatch, "
                        "summed); 5 evaluations (tools/pmc_kernels.py, tools/gpu_pmc_configs.sh)",
               "per_kernel": {}}
        ok = True
        for kern in kerns:
            pk = {}
            for d in (fetch_dir.format(which=which), write_dir.format(which=which)) + tuple(x.format(which=which) for x in sq_dirs):
                pk.update(summarise(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True), kern))
            if "FETCH_SIZE" not in pk or "WRITE_SIZE" not in pk:
                ok = False
                break
            rec["per_kernel"][kern] = pk
            for k, v in pk.items():
                key = k + "_kB" if k in ("FETCH_SIZE", "WRITE_SIZE") else k
                rec[key] = rec.get(key, 0.0) + v
        if ok:
            out[which] = rec
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print("wrote profiles/pmc_traffic_configs.json", sorted(out))


def record_hess(dirs, batch=256):
    """profiles/pmc_hess.json: counters per dispatch of ap2_hess_kernel<4> (tools/pmc_kernels.py --hess)."""
    sys.path.insert(0, ROOT)
    from bench import kernel_source_hash
    paths = [p for d in dirs for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)]
    summ = summarise(paths, "ap2_hess_kernel")
    rec = {"batch": batch, "kernel": "ap2_hess_kernel<4>", "source_hash": kernel_source_hash(),
           "units": "FETCH/WRITE_SIZE in kB per dispatch; SQ_* per dispatch"}
    for k, v in summ.items():
        rec[k + ("_kB" if k in ("FETCH_SIZE", "WRITE_SIZE") else "")] = v
    with open(os.path.join(ROOT, "profiles", "pmc_hess.json"), "w") as fh:
        json.dump(rec, fh, indent=1, sort_keys=True)
    print("wrote profiles/pmc_hess.json")


def record_gen(batch, dirs):
    """profiles/pmc_traffic.json for the generated evaluation path: counters per dispatch of
    ap2_node_kernel<4> and ap2_gather_kernel<4>, and their sum (one evaluation) at the top level,
    which bench.py reads (FETCH_SIZE x 2 + WRITE_SIZE = HBM bytes per evaluation launch)."""
    sys.path.insert(0, ROOT)
    from bench import kernel_source_hash
    paths = [p for d in dirs for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)]
    rec = {"batch": batch, "source_hash": kernel_source_hash(), "path": "generated",
           "kernel": "ap2_node_kernel + ap2_gather_kernel", "kernels": {},
           "units": "FETCH/WRITE_SIZE in kB per dispatch; SQ_* per dispatch; mean over 5 dispatches "
                    "(tools/pmc_kernels.py --ap2, tools/gpu_pmc_gen.sh)"}
    tot = defaultdict(float)
    for kern in ("ap2_node_kernel", "ap2_gather_kernel"):
        summ = summarise(paths, kern)
        rec["kernels"][kern] = {k + ("_kB" if k in ("FETCH_SIZE", "WRITE_SIZE") else ""): v for k, v in summ.items()}
        for k, v in summ.items():
            tot[k + ("_kB" if k in ("FETCH_SIZE", "WRITE_SIZE") else "")] += v
    rec["kernel"] = " + ".join(rec["kernels"])
    rec.update(tot)
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fh:
        json.dump(rec, fh, indent=1, sort_keys=True)
    print("wrote profiles/pmc_traffic.json", json.dumps({k: v for k, v in tot.items()}))


SOA_KERNELS = ("ap2_soa_in_kernel", "ap2_soa_shoot_kernel", "ap2_soa_radau_kernel", "ap2_soa_interval_kernel",
               "ap2_finalize_kernel")   # ap2_soa_in_kernel only runs with per-instance inputs


def record_soa(batch, dirs):
    """profiles/pmc_traffic.json for the instance-minor evaluation path: counters per dispatch of each
    of its kernels (tools/gpu_pmc_soa.sh) and their sum over one evaluation at the top level, which
    bench.py reads (FETCH_SIZE x 2 + WRITE_SIZE = HBM bytes per evaluation, the gfx950 correction)."""
    sys.path.insert(0, ROOT)
    from bench import kernel_source_hash
    paths = [p for d in dirs for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)]
    rec = {"batch": batch, "source_hash": kernel_source_hash(), "path": "soa", "input_layout": "instance-minor",
           "kernels": {},
           "units": "FETCH/WRITE_SIZE in kB per dispatch; SQ_* per dispatch; mean over 5 dispatches "
                    "(tools/pmc_kernels.py --ap2, tools/gpu_pmc_soa.sh)"}
    tot = defaultdict(float)
    for kern in SOA_KERNELS:
        summ = summarise(paths, kern)
        if not summ:
            continue
        rec["kernels"][kern] = {k + ("_kB" if k in ("FETCH_SIZE", "WRITE_SIZE") else ""): v for k, v in summ.items()}
        for k, v in summ.items():
            tot[k + ("_kB" if k in ("FETCH_SIZE", "WRITE_SIZE") else "")] += v
    rec["kernel"] = " + ".join(rec["kernels"])
    rec.update(tot)
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fh:
        json.dump(rec, fh, indent=1, sort_keys=True)
    print("wrote profiles/pmc_traffic.json", json.dumps({k: v for k, v in tot.items()}))


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--record-soa":
        record_soa(int(args[1]), args[2:])
        sys.exit(0)
    if args and args[0] == "--record-gen":
        record_gen(int(args[1]), args[2:])
        sys.exit(0)
    if args and args[0] == "--record-configs":
        record_configs(*args[1:])
        sys.exit(0)
    if args and args[0] == "--record-hess":
        record_hess(args[1:])
        sys.exit(0)
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
