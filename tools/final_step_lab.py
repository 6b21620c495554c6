"""Solver lab (CPU port, test harness): run the AP2 homotopy up to power1 once, cache the warm
start, then re-run only the final step with given IpmOptions and print iteration statistics."""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-k", type=int, default=40)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--cache", default="/tmp/final_lab_cache.npz")
    ap.add_argument("--opts", default="{}", help="IpmOptions overrides as JSON")
    ap.add_argument("--out", default="/tmp/final_lab.json")
    ap.add_argument("--btd", action="store_true", help="block-tridiagonal separators (the GPU's path)")
    ap.add_argument("--save", default=None, help="write the solution (V, multipliers) to this .npz")
    args = ap.parse_args()
    from awebox_amd import homotopy as hm
    from awebox_amd import problem as pb
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import IpmOptions, solve
    from awebox_amd.trajectory import hippo_options, optimize
    from oracle.cpu_device import CpuDeviceEvaluator
    consts = pb.build_constants(pb.Ap2Config(n_k=args.n_k, d=args.d))
    lay = pb.NlpLayout(args.n_k, args.d)
    ev = CpuDeviceEvaluator(consts)
    v0 = initial_guess(consts, lay)
    if not os.path.exists(args.cache):
        V, summary, out, res = optimize(consts, ev, IpmOptions(max_iter=1000), device="cpu", final_step="power1")
        np.savez(args.cache, x=res.x, lam=res.lam_g, zl=res.zl, zu=res.zu)
    c = np.load(args.cache)
    st = hm.schedule(consts, lay, v0)[-1]
    lbg, ubg = lay.g_bounds()
    P = pb.pack_p(lay, consts, v0, step=st.cost_step)
    opts = hippo_options("final", dataclasses.replace(IpmOptions(max_iter=1500, verbose=False), **json.loads(args.opts)))
    t0 = time.perf_counter()
    import awebox_amd.ipm as ipm_mod
    if args.btd:                     # the GPU's separator path (block sweep) on the host
        orig = ipm_mod.StructuredKKT.__init__

        def init(self, *a, **kw):
            orig(self, *a, **kw)
            self.force_btd = True
        ipm_mod.StructuredKKT.__init__ = init
    res = solve(ev, P, c["x"], st.lbx, st.ubx, lbg, ubg, lam0=c["lam"], zl0=c["zl"], zu0=c["zu"], opts=opts, device="cpu")
    out = hm.outputs(consts, lay, res.x)
    log = res.log
    a = np.array([r["alpha"] for r in log])
    am = np.array([r.get("alpha_max", np.nan) for r in log])
    bt = np.array([r.get("backtracks", 0) for r in log])
    print(json.dumps({"status": res.status, "iterations": res.iterations, "seconds": time.perf_counter() - t0,
                      "power_W": float(out["avg_power_W"]), "period_s": out["period_s"], "f": res.f,
                      "alpha_lt_0.1": int((a < 0.1).sum()), "ftb_lt_0.1": int((am < 0.1).sum()),
                      "backtracks_total": int(bt.sum())}))
    with open(args.out, "w") as fh:
        json.dump(log, fh, default=float)
    if args.save:
        np.savez_compressed(args.save, V=res.x, lam_g=res.lam_g, zl=res.zl, zu=res.zu, f=res.f,
                            avg_power_W=out["avg_power_W"], period_s=out["period_s"])


if __name__ == "__main__":
    main()
