"""Identical instances through the batched final homotopy step: the power1 point of the default AP2
N=40 homotopy (B = 1), then the final step for B identical instances in one batch, `--repeat` times;
prints how many members differ from member 0 (V bitwise) and their iteration counts per repeat."""
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
    ap.add_argument("--repeat", type=int, default=2)
    args = ap.parse_args()
    from awebox_amd import homotopy as hm
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import IpmOptions, solve_batch
    from awebox_amd.trajectory import hippo_options, optimize
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    ev1 = Ap2Evaluator(consts, batch=1)
    _, _, _, res = optimize(consts, ev1, IpmOptions(max_iter=2000), final_step="power1")
    st = hm.schedule(consts, lay, v0)[-1]
    lbg, ubg = lay.g_bounds()
    P = pb.pack_p(lay, consts, v0, step=st.cost_step)
    ev = Ap2Evaluator(consts, batch=args.B)
    ev.path = "colour"
    B = args.B
    for rep in range(args.repeat):
        out = solve_batch(ev, np.tile(P, (B, 1)), np.tile(res.x, (B, 1)), st.lbx, st.ubx, lbg, ubg,
                          lam0=np.tile(res.lam_g, (B, 1)), zl0=np.tile(res.zl, (B, 1)), zu0=np.tile(res.zu, (B, 1)),
                          opts=hippo_options("final", IpmOptions(max_iter=2000)))
        differ = [b for b in range(B) if not np.array_equal(out[b].x, out[0].x)]
        print(json.dumps({"rep": rep, "env": {k: v for k, v in os.environ.items() if k.startswith("AWE_")},
                          "iters": sorted(set(r.iterations for r in out)), "differ": differ[:20],
                          "n_differ": len(differ), "seconds": out[0].seconds}), flush=True)


if __name__ == "__main__":
    main()
