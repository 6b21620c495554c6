"""Profile the batched homotopy (trajectory.optimize_batch) of B wind speeds at AP2 N=40 d=4:
phase timings of the interior-point solver (IpmOptions(profile=True)) per homotopy step."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--n-k", type=int, default=40)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--out", default="gpurun_out/batch_profile.json")
    args = ap.parse_args()
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize_batch
    consts = pb.build_constants(pb.Ap2Config(n_k=args.n_k, d=4))
    u = np.linspace(5.0, 8.0, args.batch)
    ev = Ap2Evaluator(consts, batch=args.batch)
    t0 = time.perf_counter()
    V, summary, outs, res = optimize_batch(consts, ev, u, IpmOptions(max_iter=1000, profile=args.profile))
    wall = time.perf_counter() - t0
    rec = {"batch": args.batch, "wall_s": wall, "steps": [dict(r, iterations=r["iterations"]) for r in summary],
           "timing": {k: round(v, 3) for k, v in res[0].timing.items()},
           "avg_power_W": [o["avg_power_W"] for o in outs], "period_s": [o["period_s"] for o in outs]}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1, default=float)
    print(json.dumps({"wall_s": wall, "timing": rec["timing"],
                      "iters": [max(r["iterations"]) for r in summary]}, default=float))


if __name__ == "__main__":
    main()
