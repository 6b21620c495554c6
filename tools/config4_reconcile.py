"""Config 4 in the reference's order from 8 shards, on one GPU.

The dual-kite power curve (u_ref = linspace(5, 8, 64), N=20 d=4; examples/dual_kites_power_curve.py)
three ways, and the comparison the round-5 verdict asks for:

1. the reference's order: ONE chain over the 64 points (the homotopy at 5 m/s, then every point
   warm-started from the previous one; awebox/sweep.py:148-172);
2. the 8 shards of 8 points as 8 ranks run them (sweep.run_sweep mode "chain": each shard's homotopy,
   then its own chain), one after the other;
3. the shards joined by sweep.reconcile_shard in rank order, exactly as _reconcile_ranks does across
   ranks: shard r re-solves its first point warm-started from shard r-1's last solution (the
   speculative re-solve from shard r-1's own last point, re-done only if shard r-1 changed), keeps its
   chain when the re-solved point is the same optimum, re-chains otherwise.

Per point: power, period, family (interior orbit or at the example's t_f bound of 20 s), relative
power difference to the single chain, whether the V is bitwise the chain's.  Summary: points within
0.1 %, family differences, and the 8-GPU wall time of the sharded sweep modelled from the measured
per-shard times (parallel phase = slowest shard + its speculative re-solve; then the re-chains in rank
order).

    python tools/config4_reconcile.py [--out gpurun_out/config4_reconcile.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fam(t):
    return "tf_bound" if t >= 19.99 else "interior"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-k", type=int, default=20)
    ap.add_argument("--points", type=int, default=64)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "config4_reconcile.json"))
    ap.add_argument("--no-watchdog", action="store_true", help="IPOPT's watchdog off (A/B against records before it)")
    args = ap.parse_args()
    from awebox_amd.dual_homotopy import make_evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import reconcile_shard, run_sweep, speculate, warm_point_solver
    grid = np.linspace(5.0, 8.0, 64)[:args.points]
    opts = IpmOptions(max_iter=3000, watchdog_shortened_iter_trigger=0 if args.no_watchdog else 10)
    mk = lambda c, b=1: make_evaluator(c, batch=b)  # noqa: E731
    t0 = time.perf_counter()
    glob = run_sweep(grid, n_k=args.n_k, d=4, make_evaluator=mk, device="cuda", opts=opts, arch="dual",
                     mode="chain", verbose=True)
    t_glob = time.perf_counter() - t0
    print(json.dumps({"global_chain_s": t_glob}), flush=True)
    per = len(grid) // args.shards
    shards = []
    for r in range(args.shards):
        us = grid[per * r:per * (r + 1)]
        t1 = time.perf_counter()
        res = run_sweep(us, n_k=args.n_k, d=4, make_evaluator=mk, device="cuda", opts=opts, arch="dual", mode="chain",
                        verbose=True, return_states=True)
        res["wall"] = time.perf_counter() - t1
        shards.append(res)
        print(json.dumps({"shard": r, "wall_s": res["wall"], "P": [round(p, 1) for p in res["avg_power_W"]]}),
              flush=True)
    prob, v0 = shards[0]["problem"], shards[0]["v0"]
    ev = mk(prob.consts)
    solve_warm = warm_point_solver(prob, ev, opts, "cuda", v0)
    spec_s, seq_s, changed_prev, decisions = [0.0], 0.0, False, ["start"]
    spec_last = [s["states"][-1] for s in shards]             # each shard's own last solution
    for r in range(1, args.shards):
        s = shards[r]
        us = list(s["u_ref"])
        outs = [{"avg_power_W": p, "period_s": t} for p, t in zip(s["avg_power_W"], s["period_s"])]
        t1 = time.perf_counter()
        spec = speculate(solve_warm, us, spec_last[r - 1])          # the parallel speculative re-solves
        spec_s.append(time.perf_counter() - t1)
        t1 = time.perf_counter()
        pred_final = shards[r - 1]["states"][-1]
        changed = reconcile_shard(solve_warm, us, s["states"], outs, s["iterations"], s["ok"], pred_final,
                                  changed_prev, spec=spec)
        seq_s += time.perf_counter() - t1
        decisions.append(("re-chained" if changed and len(us) > 2 else "kept")
                         + (" (predecessor changed)" if changed_prev else ""))
        s["avg_power_W"] = [o["avg_power_W"] for o in outs]
        s["period_s"] = [o["period_s"] for o in outs]
        s["V_opt"] = np.stack([st[0] for st in s["states"]])
        changed_prev = changed
        print(json.dumps({"reconcile": r, "decision": decisions[-1], "P": [round(p, 1) for p in s["avg_power_W"]]}),
              flush=True)
    # comparison with the single chain
    rows = []
    Vg = np.asarray(glob["V_opt"])
    for i, u in enumerate(grid):
        r, j = divmod(i, per)
        s = shards[r]
        pg, tg = glob["avg_power_W"][i], glob["period_s"][i]
        ps, ts = s["avg_power_W"][j], s["period_s"][j]
        rows.append({"i": i, "u_ref": float(u), "shard": r, "global": {"P": pg, "T": tg, "family": fam(tg)},
                     "reconciled": {"P": ps, "T": ts, "family": fam(ts), "dP_rel": (ps - pg) / pg,
                                    "bitwise": bool(np.array_equal(np.asarray(s["V_opt"][j]), Vg[i])),
                                    "ok": bool(s["ok"][j])}})
    d = [r["reconciled"] for r in rows]
    t_par = max(s["wall"] + sp for s, sp in zip(shards, spec_s))
    summ = {"points": len(rows), "within_0.1pct": sum(abs(x["dP_rel"]) <= 1e-3 for x in d),
            "bitwise_equal_chain": sum(x["bitwise"] for x in d),
            "family_differs": [r["i"] for r in rows if r["reconciled"]["family"] != r["global"]["family"]],
            "max_abs_dP_rel": max(abs(x["dP_rel"]) for x in d), "all_converged": all(x["ok"] for x in d),
            "decisions": decisions,
            "global_chain": {"wall_s": t_glob, "trials_per_s": len(grid) / t_glob,
                             "power_monotone": bool(np.all(np.diff(glob["avg_power_W"]) > 0))},
            "sharded_8gpu_model": {"parallel_phase_s": t_par, "sequential_reconcile_s": seq_s,
                                   "wall_s": t_par + seq_s, "trials_per_s": len(grid) / (t_par + seq_s)},
            "reconciled_power_monotone": bool(np.all(np.diff([x["P"] for x in d]) > 0))}
    out = {"summary": summ, "points": rows}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1, default=lambda o: o.item() if hasattr(o, "item") else str(o))
    print(json.dumps(summ, default=lambda o: o.item() if hasattr(o, "item") else str(o)), flush=True)


if __name__ == "__main__":
    main()
