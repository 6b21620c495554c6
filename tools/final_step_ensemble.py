"""Branch statistics of the AP2 N=40 homotopy's final step.

Runs the default homotopy up to power1 once (B = 1, the product path), then solves the final step
for K members at once (ipm.solve_batch, one IPOPT iteration per member): member 0 starts from the
power1 point itself, member b > 0 from it times (1 + eps N(0,1)) (seeded), with the power1
multipliers.  Prints one JSON line per solver variant: per member the status, iterations,
period, average power and objective, and the histogram of the period branches.  With --trace the
per-iteration logs of members 0 and 1 are written too (first divergence of their iterates).

    python tools/final_step_ensemble.py --k 16 --eps 1e-13 --variants '[{}, {"watchdog": false}]'
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def branch(period: float) -> str:
    for name, lo, hi in (("35.9", 33.0, 40.0), ("51.7", 50.0, 53.5), ("58.4", 56.0, 61.0), ("70", 69.0, 70.5)):
        if lo <= period <= hi:
            return name
    return f"other:{period:.1f}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--eps", type=float, default=1e-13)
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--path", default="generated", choices=["generated", "colour", "soa", "cpu"])
    ap.add_argument("--hess", default="follow", choices=["follow", "generated", "hyperdual"],
                    help="Hessian kernel (default: the one the evaluation path selects)")
    ap.add_argument("--variants", default="[{}]", help="JSON list of IpmOptions overrides")
    ap.add_argument("--cache", default=os.path.join(ROOT, "gpurun_out", "power1_{path}.npz"))
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "final_step_ensemble.jsonl"))
    ap.add_argument("--trace", default=None, help="write the logs of members 0 and 1 to this JSON file")
    args = ap.parse_args()
    from awebox_amd import homotopy as hm
    from awebox_amd import problem as pb
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import IpmOptions, solve_batch
    from awebox_amd.trajectory import hippo_options, optimize
    consts = pb.build_constants(pb.Ap2Config())
    lay = pb.NlpLayout(consts.cfg.n_k, consts.cfg.d)
    v0 = initial_guess(consts, lay)

    def make_ev(batch):
        if args.path == "cpu":
            from oracle.cpu_device import CpuDeviceEvaluator
            return CpuDeviceEvaluator(consts), "cpu"
        from awebox_amd.evaluator import Ap2Evaluator
        ev = Ap2Evaluator(consts, batch=batch)
        ev.path = args.path
        ev.hess_path = args.hess
        return ev, "cuda"

    cache = args.cache.format(path=f"{args.path}_{args.hess}")
    if not os.path.exists(cache):
        ev1, dev = make_ev(1)
        t0 = time.perf_counter()
        _, summ, _, res = optimize(consts, ev1, IpmOptions(max_iter=2000), device=dev, final_step="power1",
                                   eval_path=None)
        os.makedirs(os.path.dirname(cache), exist_ok=True)
        np.savez(cache, x=res.x, lam=res.lam_g, zl=res.zl, zu=res.zu)
        print(json.dumps({"power1": [s["iterations"] for s in summ], "seconds": time.perf_counter() - t0}), flush=True)
    c = np.load(cache)
    st = hm.schedule(consts, lay, v0)[-1]
    lbg, ubg = lay.g_bounds()
    P = pb.pack_p(lay, consts, v0, step=st.cost_step)
    K = args.k
    rng = np.random.default_rng(args.seed)
    noise = rng.standard_normal((K, lay.n_v))
    noise[0] = 0.0
    X0 = c["x"][None, :] * (1.0 + args.eps * noise)
    ev, dev = make_ev(K)
    i_tf = int(lay.theta()[1])
    s_tf = float(consts.scaling[pb.W_TH0 + 1])
    for var in json.loads(args.variants):
        # per iteration: the period of every member and the largest scaled distance of member b's
        # V from member 0's (the growth of a 1e-13 difference along the iteration)
        periods, dist = [], []

        def cb(it, V, stepped):
            Vh = V.detach().cpu().numpy() if hasattr(V, "detach") else np.asarray(V)
            periods.append((Vh[:, i_tf] * s_tf).round(4).tolist())
            dist.append(np.abs(Vh - Vh[0:1]).max(axis=1).tolist())
        opts = hippo_options("final", dataclasses.replace(IpmOptions(max_iter=3000, callback=cb), **var))
        t0 = time.perf_counter()
        res = solve_batch(ev, np.tile(P, (K, 1)), X0, st.lbx, st.ubx, lbg, ubg,
                          lam0=np.tile(c["lam"], (K, 1)), zl0=np.tile(c["zl"], (K, 1)), zu0=np.tile(c["zu"], (K, 1)),
                          opts=opts, device=dev)
        secs = time.perf_counter() - t0
        members = []
        hist = {}
        for r in res:
            out = hm.outputs(consts, lay, r.x)
            br = branch(out["period_s"])
            hist[br] = hist.get(br, 0) + 1
            members.append({"status": r.status, "it": r.iterations, "T": round(out["period_s"], 3),
                            "P": round(out["avg_power_W"], 1), "f": r.f, "branch": br})
        rec = {"variant": var, "path": args.path, "hess": getattr(ev, "hess_path", "fd"), "k": K, "eps": args.eps, "seconds": secs, "hist": hist,
               "members": members}
        line = json.dumps(rec, default=float)
        print(line, flush=True)
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "a") as fh:
            fh.write(line + "\n")
        if args.trace:
            with open(args.trace, "w") as fh:
                json.dump({"variant": var, "logs": [r.log for r in res], "periods": periods, "dist": dist}, fh,
                          default=float)


if __name__ == "__main__":
    main()
