"""Which AP2 N=40 wind speeds give sweep points whose period is not on a t_f bound (20 or 70 s)?
Runs the bench's fan-mode shard (8 points, batched warm start) at a few u_ref ranges and prints
periods, powers and trials/s.

    python tools/sweep_interior_probe.py [--ranges 8.5:10,10:12]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranges", default="8.5:10,10:12")
    a = ap.parse_args()
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    consts = pb.build_constants()
    # warm the solver and evaluator kernels once (the bench's earlier blocks do this)
    run_sweep([5.0, 5.05], n_k=consts.cfg.n_k, d=consts.cfg.d, make_evaluator=lambda c, b=1: Ap2Evaluator(c, batch=b),
              dist=None, device="cuda", opts=IpmOptions(max_iter=1000), mode="fan")
    for rg in a.ranges.split(","):
        lo, hi = (float(x) for x in rg.split(":"))
        u = list(np.linspace(lo, hi, 8))
        res = run_sweep(u, n_k=consts.cfg.n_k, d=consts.cfg.d, make_evaluator=lambda c, b=1: Ap2Evaluator(c, batch=b),
                        dist=None, device="cuda", opts=IpmOptions(max_iter=1000), mode="fan")
        print(json.dumps({"u": [round(x, 3) for x in u], "trials_per_s": res["trials_per_s"], "wall_s": res["wall_s"],
                          "period_s": [round(t, 2) for t in res["period_s"]], "avg_power_W": [round(p, 1) for p in res["avg_power_W"]],
                          "iterations": res["iterations"], "ok": [bool(x) for x in res["ok"]]}), flush=True)


if __name__ == "__main__":
    main()
