"""Run the dual-kite power-cycle homotopy (examples/dual_kites_power_curve.py options) with the GPU
interior-point solver, the HIP dual-kite evaluator and the coloured central-difference Hessian;
write per-step summaries and outputs to gpurun_out/solve_dual.json."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-k", type=int, default=20)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--u-ref", type=float, default=10.0)
    ap.add_argument("--max-iter", type=int, default=500)
    ap.add_argument("--final-step", default=None)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "solve_dual.json"))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()
    import torch
    from awebox_amd import dual as du
    from awebox_amd import dual_homotopy as dh
    from awebox_amd.build import build
    from awebox_amd.ipm import IpmOptions
    build()
    mc = du.build_constants(du.MultiConfig(n_k=args.n_k, d=args.d, u_ref=args.u_ref))
    ev = dh.make_evaluator(mc)
    t0 = time.perf_counter()
    V, summary, out, _ = dh.optimize(mc, ev, IpmOptions(max_iter=args.max_iter, verbose=args.verbose, profile=args.profile),
                                     verbose=True, final_step=args.final_step)
    rec = {"n_k": args.n_k, "d": args.d, "u_ref": args.u_ref, "seconds": time.perf_counter() - t0,
           "steps": summary, "outputs": out, "device": torch.cuda.get_device_name(0)}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1, default=float)
    print(json.dumps({"outputs": out, "seconds": rec["seconds"]}, default=float))


if __name__ == "__main__":
    main()
