"""Config 4 in full on one GPU: the 64 points of u_ref = linspace(5, 8, 64) (the dual-kite power
curve, examples/dual_kites_power_curve.py:48 range, N=20 d=4) as the 8 ranks' shards of 8 points,
run one after the other with awebox_amd.sweep.run_sweep (the code each rank runs).  Writes one JSON
line per shard (powers, periods, iterations, convergence, wall) and a summary line with the whole
power curve and its monotonicity.

    python tools/config4_full.py --mode fan --shards 0-7
    python tools/config4_full.py --global-chain     # the reference's order: one chain over all 64 points

--global-chain runs the 64 points as ONE chain on one GPU (the homotopy at 5 m/s, then every next
point warm-started from the previous one: awebox/sweep.py:150-172 with the example's
apply_sweeping_warmstart), the order the reference's sweep solves them in; the optimal V of every
point goes to gpurun_out/config4_global_chain_V.npz.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="fan", choices=["fan", "chain", "batch"])
    ap.add_argument("--shards", default="0-7")
    ap.add_argument("--n-k", type=int, default=20)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "config4_full.jsonl"))
    ap.add_argument("--global-chain", action="store_true")
    args = ap.parse_args()
    from awebox_amd.dual_homotopy import make_evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    lo, hi = (int(x) for x in args.shards.split("-"))
    grid = np.linspace(5.0, 8.0, 64)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    if args.global_chain:
        t0 = time.perf_counter()
        res = run_sweep(grid, n_k=args.n_k, d=4, make_evaluator=lambda c, b=1: make_evaluator(c, batch=b),
                        device="cuda", opts=IpmOptions(max_iter=3000), arch="dual", mode="chain", verbose=True)
        p = np.asarray(res["avg_power_W"], dtype=float)
        rec = {"global_chain": True, "n_k": args.n_k, "u_ref": [round(float(x), 5) for x in res["u_ref"]],
               "avg_power_W": [round(float(x), 2) for x in p],
               "period_s": [round(float(t), 3) for t in res["period_s"]],
               "iterations": [int(i) for i in res["iterations"]], "ok": [bool(o) for o in res["ok"]],
               "wall_s": time.perf_counter() - t0, "trials_per_s": res["trials_per_s"],
               "all_converged": bool(all(res["ok"])), "power_monotone": bool(np.all(np.diff(p) > 0)),
               "min_step_W": float(np.min(np.diff(p)))}
        print(json.dumps(rec), flush=True)
        out = os.path.join(os.path.dirname(args.out), "config4_global_chain.jsonl")
        with open(out, "a") as fh:
            fh.write(json.dumps(rec) + "\n")
        np.savez_compressed(os.path.join(os.path.dirname(args.out), "config4_global_chain_V.npz"),
                            u_ref=np.asarray(res["u_ref"]), V=np.asarray(res["V_opt"]))
        return
    curve = {}
    t_all = time.perf_counter()
    for r in range(lo, hi + 1):
        u = grid[8 * r:8 * r + 8]
        t0 = time.perf_counter()
        res = run_sweep(u, n_k=args.n_k, d=4, make_evaluator=lambda c, b=1: make_evaluator(c, batch=b),
                        device="cuda", opts=IpmOptions(max_iter=3000), arch="dual", mode=args.mode, verbose=True)
        rec = {"shard": r, "mode": args.mode, "n_k": args.n_k, "u_ref": [round(float(x), 5) for x in res["u_ref"]],
               "avg_power_W": [round(float(p), 2) for p in res["avg_power_W"]],
               "period_s": [round(float(t), 3) for t in res["period_s"]],
               "iterations": [int(i) for i in res["iterations"]], "ok": [bool(o) for o in res["ok"]],
               "wall_s": time.perf_counter() - t0, "trials_per_s": res["trials_per_s"]}
        print(json.dumps(rec), flush=True)
        with open(args.out, "a") as fh:
            fh.write(json.dumps(rec) + "\n")
        for uu, p, ok in zip(rec["u_ref"], rec["avg_power_W"], rec["ok"]):
            curve[uu] = (p, ok)
    us = sorted(curve)
    p = np.array([curve[x][0] for x in us])
    summary = {"summary": True, "mode": args.mode, "points": len(us), "all_converged": all(curve[x][1] for x in us),
               "power_monotone": bool(np.all(np.diff(p) > 0)), "min_step_W": float(np.min(np.diff(p))) if len(p) > 1 else None,
               "p_first_W": float(p[0]), "p_last_W": float(p[-1]), "wall_s": time.perf_counter() - t_all}
    print(json.dumps(summary), flush=True)
    with open(args.out, "a") as fh:
        fh.write(json.dumps(summary) + "\n")


if __name__ == "__main__":
    main()
