"""A/B of the fused interior-point measures (AWE_IPM_FUSED=1, libawelu awelu_ipm_measures) against
the torch composition (AWE_IPM_FUSED=0) in one process: the converged MPC (config 5, B loops, the
bench's pmpc_block loop) and the AP2 N=40 default homotopy at B=1.  Reports the time per sampling
time / per homotopy and whether every iterate is bitwise the same.

    python tools/ipm_fused_ab.py [--loops 64] [--steps 3] [--no-ap2] [--out gpurun_out/ipm_fused_ab.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pmpc(fused, loops, steps):
    os.environ["AWE_IPM_FUSED"] = "1" if fused else "0"
    from awebox_amd import kite3 as k3
    from awebox_amd.mpc_solve import BatchedPmpc
    c = k3.build_constants()
    r = BatchedPmpc(c, loops, device="cuda")
    r.start(seed=99)
    r.simulate_reference(1 + steps + c.cfg.n_k + 1)
    r.step()
    torch.cuda.synchronize()
    Vs, its, ts = [], [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        out = r.step()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        Vs.append(r.V.cpu().numpy().copy())
        its.append(np.asarray(out["iterations"]).tolist())
    return Vs, its, ts


def ap2(fused):
    os.environ["AWE_IPM_FUSED"] = "1" if fused else "0"
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize
    consts = pb.build_constants()
    ev = Ap2Evaluator(consts, batch=1)
    t0 = time.perf_counter()
    _, _, _, res = optimize(consts, ev, IpmOptions(max_iter=2000))
    torch.cuda.synchronize()
    return res, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loops", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-ap2", action="store_true")
    ap.add_argument("--out", default="gpurun_out/ipm_fused_ab.json")
    a = ap.parse_args()
    rec = {}
    V0, it0, t0 = pmpc(False, a.loops, a.steps)
    V1, it1, t1 = pmpc(True, a.loops, a.steps)
    rec["pmpc"] = {"loops": a.loops, "ms_per_step_torch": [1e3 * t for t in t0], "ms_per_step_fused": [1e3 * t for t in t1],
                   "iterations_equal": it0 == it1,
                   "bitwise_equal": all(np.array_equal(x, y) for x, y in zip(V0, V1))}
    print(json.dumps(rec["pmpc"]), flush=True)
    if not a.no_ap2:
        r0, s0 = ap2(False)
        r1, s1 = ap2(True)
        rec["ap2"] = {"s_torch": s0, "s_fused": s1, "iterations": [r0.iterations, r1.iterations],
                      "bitwise_equal": bool(np.array_equal(r0.x, r1.x) and np.array_equal(r0.lam_g, r1.lam_g)),
                      "f": [r0.f, r1.f]}
        print(json.dumps(rec["ap2"]), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
