"""Where a sweep block's time goes: runs bench.py's sweep block recipe (run_sweep, fan mode) with
every interior-point call recorded (batch, iterations, KKT solves, dense-LU fallbacks, phase
timings with IpmOptions(profile=True)) and the dense fallback's library solves timed.

    python tools/sweep_phase_probe.py --arch ap2 --points 8 [--profile] --out gpurun_out/sweep_phases.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", choices=["ap2", "dual"], default="ap2")
    ap.add_argument("--points", type=int, default=8)
    ap.add_argument("--profile", action="store_true", help="synchronised phase timings (slower)")
    ap.add_argument("--refine", type=int, default=None, help="StructuredKKT.REFINE_STEPS override")
    ap.add_argument("--awelu-solve", action="store_true", help="btd.BorderedBtd.AWELU_SOLVE (block recursion)")
    ap.add_argument("--out", default="gpurun_out/sweep_phases.json")
    args = ap.parse_args()
    import torch

    import awebox_amd.ipm as ipm
    import awebox_amd.sweep as sw
    import awebox_amd.trajectory as tr

    if args.refine is not None:
        ipm.StructuredKKT.REFINE_STEPS = args.refine
    if args.awelu_solve:
        import awebox_amd.btd as btd
        btd.BorderedBtd.AWELU_SOLVE = True
    calls = []
    dense = {"n": 0, "s": 0.0}
    orig_sb = ipm.solve_batch

    def rec_solve_batch(*a, **k):
        t0 = time.perf_counter()
        out = orig_sb(*a, **k)
        torch.cuda.synchronize()
        calls.append({"B": len(out), "s": time.perf_counter() - t0, "iterations": [r.iterations for r in out],
                      "kkt_solves": out[0].kkt_solves, "kkt_dense": out[0].kkt_dense,
                      "timing": {q: round(v, 4) for q, v in out[0].timing.items()}})
        print(json.dumps(calls[-1]), flush=True)
        return out

    orig_se = torch.linalg.solve_ex

    def rec_solve_ex(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = orig_se(*a, **k)
        torch.cuda.synchronize()
        dense["n"] += 1
        dense["s"] += time.perf_counter() - t0
        return out

    ipm.solve_batch = rec_solve_batch
    tr.solve_batch = rec_solve_batch
    sw.solve_batch = rec_solve_batch
    torch.linalg.solve_ex = rec_solve_ex
    dev = torch.device("cuda:0")
    u = np.linspace(5.0, 8.0, 64)[:args.points]
    opts = ipm.IpmOptions(max_iter=1000 if args.arch == "ap2" else 3000, profile=args.profile)
    if args.arch == "ap2":
        from awebox_amd.evaluator import Ap2Evaluator
        mk = lambda c, b=1: Ap2Evaluator(c, batch=b)  # noqa: E731
        kw = dict(n_k=40, d=4)
    else:
        from awebox_amd.dual_homotopy import make_evaluator
        mk = lambda c, b=1: make_evaluator(c, device=str(dev), batch=b)  # noqa: E731
        kw = dict(n_k=20, d=4, arch="dual")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = sw.run_sweep(u, make_evaluator=mk, device=str(dev), opts=opts, mode="fan", **kw)
    wall = time.perf_counter() - t0
    phases = {}
    for c in calls:
        for q, v in c["timing"].items():
            phases[q] = phases.get(q, 0.0) + v
    rec = {"arch": args.arch, "points": args.points, "profile": args.profile, "wall_s": wall,
           "refine_steps": ipm.StructuredKKT.REFINE_STEPS,
           "trials_per_s": res["trials_per_s"], "iterations": res["iterations"],
           "avg_power_W": [round(p, 3) for p in res["avg_power_W"]], "dense_fallbacks": dense["n"],
           "dense_fallback_s": dense["s"], "phase_s": {q: round(v, 3) for q, v in phases.items()}, "calls": calls}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps({k: rec[k] for k in ("wall_s", "trials_per_s", "iterations", "dense_fallbacks",
                                          "dense_fallback_s", "phase_s")}), flush=True)


if __name__ == "__main__":
    main()
