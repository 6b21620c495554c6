"""Sensitivity of the default AP2 N=40 homotopy's end point to roundoff-level changes: the full
homotopy on the generated, the colour and the instance-minor evaluation path, and on the colour path from initial
guesses perturbed by a relative 1e-13 / 1e-10 (seeded).  Prints one JSON line per run: steps,
iterations, final objective, average power and period.

    python tools/homotopy_branch.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    rng = np.random.default_rng(7)
    noise = rng.standard_normal(v0.shape)
    runs = [("generated", 0.0), ("colour", 0.0), ("colour", 1e-13), ("colour", 1e-10), ("generated", 1e-13),
            ("soa", 0.0)]
    for path, eps in runs:
        ev = Ap2Evaluator(consts, batch=1)
        ev.path = path
        V, summary, out, _ = optimize(consts, ev, IpmOptions(max_iter=2000), v_init=v0 * (1.0 + eps * noise),
                                      eval_path=None)
        print(json.dumps({"path": path, "hess": ev.hess_path, "perturbation": eps,
                          "iterations": [r["iterations"] for r in summary],
                          "status": [r["status"] for r in summary], "f": summary[-1]["f"],
                          "avg_power_W": out["avg_power_W"], "period_s": out["period_s"]}, default=float), flush=True)


if __name__ == "__main__":
    main()
