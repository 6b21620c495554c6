"""Which separator path the dual-kite KKT takes (block-tridiagonal or dense Schur complement), and
the dual homotopy's per-step KKT statistics (dense fallbacks, phase seconds) at N=20 d=4, u_ref = 5."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from awebox_amd import dual as du
    from awebox_amd import dual_homotopy as dh
    from awebox_amd.ipm import DeviceNlp, IpmOptions, StructuredKKT
    mc = du.build_constants(du.MultiConfig(n_k=20, d=4))
    lay = du.layout_for(mc)
    ev = dh.make_evaluator(mc, batch=1)
    v0 = du.initial_guess(mc, lay)
    st = dh.schedule(mc, lay, v0)[0]
    lbg, ubg = lay.g_bounds()
    nlp = DeviceNlp(ev, du.pack_p(lay, mc, v0, step=st.cost_step), st.lbx, st.ubx, lbg, ubg, "cuda")
    sk = StructuredKKT(nlp, ev.layout, "cuda", separators="btd")
    print(json.dumps({"n_k": lay.n_k, "btd": sk.btd is not None, "nS": sk.nS, "nI": sk.nI, "N": sk.N}), flush=True)
    _, summary, out, _ = dh.optimize(mc, ev, IpmOptions(max_iter=3000, profile=True), u_ref=5.0)
    for r in summary:
        print(json.dumps({k: r[k] for k in ("step", "iterations", "seconds", "kkt_solves", "kkt_dense", "timing")}),
              flush=True)


if __name__ == "__main__":
    main()
