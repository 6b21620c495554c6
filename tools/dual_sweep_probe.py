"""Config-4 shard on one GPU with progress output: the dual-kite fan sweep (homotopy for the first
point, batched warm start for the rest) at N=20 d=4, printing per point the iterations, KKT solves,
dense fallbacks and wall time.  Used to A/B the separator linear algebra.

    python tools/dual_sweep_probe.py [--points 8] [--first 0] [--mode fan]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=8)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--mode", default="fan")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--max-m", type=int, default=None,
                    help="largest separator stage for the fused kernels (48: the block recursion for m = 100)")
    args = ap.parse_args()
    import numpy as np

    from awebox_amd import batched_lu
    if args.max_m is not None:
        batched_lu.BTD_MAX_M = args.max_m

    from awebox_amd.dual_homotopy import make_evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    u = np.linspace(5.0, 8.0, 64)[args.first:args.first + args.points]
    t0 = time.perf_counter()
    res = run_sweep(u, n_k=20, d=4, make_evaluator=lambda c, b=1: make_evaluator(c, batch=b), device="cuda",
                    opts=IpmOptions(max_iter=3000), arch="dual", mode=args.mode, verbose=args.verbose)
    el = time.perf_counter() - t0
    out = {k: res.get(k) for k in ("iterations", "avg_power_W", "period_s", "ok", "wall_s")}
    for k in ("kkt_solves", "kkt_dense", "timing"):
        if k in res:
            out[k] = res[k]
    out["elapsed_s"] = el
    out["separator"] = "fused" if batched_lu.BTD_MAX_M >= 100 else "block recursion"
    out["trials_per_s"] = len(u) / el
    print(json.dumps(out, default=str), flush=True)


if __name__ == "__main__":
    main()
