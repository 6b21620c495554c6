"""Config 5 closed loop on one GPU: B tracking-MPC loops advanced by batched real-time iterations
(awebox_amd/rti.py), with a per-phase time breakdown (linearisation + KKT solve, plant, shift).

    python tools/mpc_closed_loop.py --batch 256 --steps 40 --out gpurun_out/mpc_rti.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--n-k", type=int, default=20)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--out", default=None)
    ap.add_argument("--plant", choices=["collocation", "rk4root"], default="collocation")
    a = ap.parse_args()
    import numpy as np
    import torch

    from awebox_amd import kite3 as k3
    from awebox_amd.rti import BatchedRti

    c = k3.build_constants(k3.Kite3Config(n_k=a.n_k, d=a.d))
    r = BatchedRti(c, a.batch, device="cuda", plant=a.plant)
    r.start()
    sync = torch.cuda.synchronize
    phases = {"iterate": [], "plant": [], "shift": []}
    hist = []
    for s in range(a.steps):
        sync()
        t0 = time.perf_counter()
        eq, path = r.iterate()
        r.u0 = r.V[:, r.u0_idx].clone()
        sync()
        t1 = time.perf_counter()
        x1, pres = r._plant() if a.plant == "collocation" else r._rk4root()
        sync()
        t2 = time.perf_counter()
        r._shift(x1)
        r.step_count += 1
        sync()
        t3 = time.perf_counter()
        for k, v in zip(phases, (t1 - t0, t2 - t1, t3 - t2)):
            phases[k].append(v * 1e3)
        x_ref = r.P[:, r.lay.p_ref + r.lay.x(0)[0]:r.lay.p_ref + r.lay.x(0)[0] + k3.NX]
        trk = (x1 - x_ref).norm(dim=1)
        hist.append({"step": s, "eq_residual_max": float(eq.max()), "eq_residual_median": float(eq.median()),
                     "path_max": float(path.max()), "plant_residual_max": float(pres.max()),
                     "tracking_error_median": float(trk.median()), "tracking_error_max": float(trk.max()),
                     "finite": bool(torch.isfinite(r.V).all())})
        print(json.dumps(hist[-1]), flush=True)
    # un-synchronised timing of whole RTI steps
    sync()
    t0 = time.perf_counter()
    n = 10
    for _ in range(n):
        r.step()
    sync()
    el = (time.perf_counter() - t0) / n
    skip = min(2, a.steps - 1)
    res = {"batch": a.batch, "n_k": a.n_k, "d": a.d, "plant": a.plant, "ms_per_rti_step": el * 1e3,
           "loop_steps_per_s": a.batch / el,
           "phase_ms_median": {k: float(np.median(v[skip:])) for k, v in phases.items()},
           "kkt": {"interval_block": r.nI, "separator_block": r.nS, "coupling": r.L},
           "history": hist}
    print(json.dumps({k: v for k, v in res.items() if k != "history"}))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
