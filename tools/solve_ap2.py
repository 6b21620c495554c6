"""Run the AP2 power-cycle homotopy with the GPU interior-point solver and the HIP evaluator;
write per-step summaries and the trajectory outputs to gpurun_out/solve_ap2.json."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-k", type=int, default=40)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--u-ref", type=float, default=10.0)
    ap.add_argument("--max-iter", type=int, default=1000)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "solve_ap2.json"))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="the CPU port behind the device interface (test harness)")
    ap.add_argument("--iter-log", action="store_true", help="keep every step's per-iteration log in the output")
    ap.add_argument("--opts", default="{}", help="IpmOptions overrides as JSON")
    args = ap.parse_args()
    import torch
    from awebox_amd import problem as pb
    from awebox_amd.build import build
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize
    consts = pb.build_constants(pb.Ap2Config(n_k=args.n_k, d=args.d, u_ref=args.u_ref))
    if args.cpu:
        from oracle.cpu_device import CpuDeviceEvaluator
        ev, device = CpuDeviceEvaluator(consts), "cpu"
    else:
        build()
        ev, device = Ap2Evaluator(consts, batch=1), "cuda"
    t0 = time.perf_counter()
    import dataclasses
    base = dataclasses.replace(IpmOptions(max_iter=args.max_iter, verbose=args.verbose), **json.loads(args.opts))
    V, summary, out, _ = optimize(consts, ev, base,
                               verbose=True, device=device, keep_logs=args.iter_log)
    rec = {"n_k": args.n_k, "d": args.d, "u_ref": args.u_ref, "seconds": time.perf_counter() - t0,
           "steps": summary, "outputs": out, "device": torch.cuda.get_device_name(0) if device == "cuda" else "cpu"}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(rec, fh, indent=1, default=float)
    print(json.dumps({"outputs": out, "seconds": rec["seconds"]}, default=float))


if __name__ == "__main__":
    main()
