"""Do identical instances stay identical through a batched homotopy?  The AP2 N=40 default homotopy
for B identical instances in one batch (the steps of trajectory.optimize_batch, colour path), with
every step's members compared bitwise to member 0 and to a B = 1 run.

    python tools/batch_members.py [--B 128] [--probe]
--probe wraps the solver's building blocks as tools/batch_consistency_probe.py does (first operation
that gives identical inputs different outputs)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--probe", action="store_true")
    args = ap.parse_args()
    from awebox_amd import homotopy as hm
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import IpmOptions, solve_batch
    from awebox_amd.trajectory import hippo_options
    if args.probe:
        import batch_consistency_probe as bp
        bp.install()
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    steps = hm.schedule(consts, lay, v0)
    lbg, ubg = lay.g_bounds()
    runs = {}
    for B in (1, args.B):
        ev = Ap2Evaluator(consts, batch=B)
        ev.path = "colour"
        x = np.tile(v0, (B, 1))
        lam = zl = zu = None
        recs = []
        for st in steps:
            P = np.tile(pb.pack_p(lay, consts, v0, step=st.cost_step), (B, 1))
            try:
                res = solve_batch(ev, P, x, st.lbx, st.ubx, lbg, ubg, lam0=lam, zl0=zl, zu0=zu,
                                  opts=hippo_options(st.label, IpmOptions(max_iter=2000)))
            except Exception as e:                        # the probe's report
                print(json.dumps({"B": B, "step": st.label, "stopped": str(e)[:2000]}), flush=True)
                return
            x = np.stack([r.x for r in res])
            lam = np.stack([r.lam_g for r in res])
            zl = np.stack([r.zl for r in res])
            zu = np.stack([r.zu for r in res])
            differ = [b for b in range(B) if not np.array_equal(x[b], x[0])]
            recs.append({"step": st.label, "iters": sorted(set(r.iterations for r in res)), "differ": differ[:20],
                         "n_differ": len(differ), "x0": x[0].copy()})
        runs[B] = recs
        out = hm.outputs(consts, lay, x[0])
        print(json.dumps({"B": B, "period_s": out["period_s"],
                          "steps": [{k: v for k, v in r.items() if k != "x0"} for r in recs]}), flush=True)
    for r1, rb in zip(runs[1], runs[args.B]):
        print(json.dumps({"step": r1["step"], "member0_equals_B1": bool(np.array_equal(r1["x0"], rb["x0"]))}), flush=True)


if __name__ == "__main__":
    main()
