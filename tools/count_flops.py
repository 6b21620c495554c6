"""Algorithmic flop count of one AP2 NLP evaluation: compile and run
tools/flops/ap2_flops.cpp (the node model on an op-counting scalar, the assembly counted from
the kernel's loops) and write the record bench.py divides by the measured kernel time.

    python tools/count_flops.py [--n-k 40] [--d 4] [--out profiles/r03/flops_ap2.json]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
MODEL_SOURCES = [os.path.join(ROOT, "awebox_amd", "csrc", f) for f in ("ap2_model.hpp", "ap2_tables.hpp", "scalar.hpp")]


def source_hash() -> str:
    h = hashlib.sha256()
    for p in MODEL_SOURCES + [os.path.join(ROOT, "tools", "flops", "ap2_flops.cpp")]:
        h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def count(n_k=40, d=4) -> dict:
    import numpy as np

    from awebox_amd import problem as pb
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    with tempfile.TemporaryDirectory() as tmp:
        exe = os.path.join(tmp, "ap2_flops")
        subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "awebox_amd", "csrc"), "-I",
                        os.path.join(ROOT, "include"), os.path.join(ROOT, "tools", "flops", "ap2_flops.cpp"),
                        "-o", exe], check=True)
        cfile = os.path.join(tmp, "consts.txt")
        np.savetxt(cfile, consts.consts)
        out = subprocess.run([exe, str(n_k), str(d), cfile], check=True, capture_output=True, text=True)
    rec = json.loads(out.stdout)
    rec["source_hash"] = source_hash()
    rec["method"] = ("node model on an op-counting scalar carrying its colour-dependency set (value ops once per "
                     "node, tangent ops per structurally nonzero colour), assembly from the kernel's loops; "
                     "tools/flops/ap2_flops.cpp")
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-k", type=int, default=40)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03", "flops_ap2.json"))
    args = ap.parse_args()
    rec = count(args.n_k, args.d)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
