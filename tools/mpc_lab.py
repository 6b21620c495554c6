"""GPU lab: converged tracking MPC (mpc_solve.BatchedPmpc) on config 5's instances.

    python tools/mpc_lab.py --batch 4 --ref sim|circle [--verbose] [--steps S]

Prints per-loop status / iterations / solve time, the active bounds at the solution and the
distance to ten Gauss-Newton iterations (the RTI at fixed P) from the same start.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from awebox_amd import kite3 as k3  # noqa: E402
from awebox_amd.ipm import IpmOptions  # noqa: E402
from awebox_amd.mpc_solve import CONSISTENT_X0, BatchedPmpc, simulated_reference  # noqa: E402
from awebox_amd.rti import BatchedRti  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--ref", default="sim", choices=["sim", "circle"])
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--steps", type=int, default=0, help="closed-loop steps after the first solve")
    ap.add_argument("--no-homotopy", action="store_true")
    a = ap.parse_args()
    c = k3.build_constants()
    B = a.batch
    pm = BatchedPmpc(c, B, device="cuda", opts=IpmOptions(verbose=a.verbose),
                     homotopy_warmstart=not a.no_homotopy)
    pm.start()
    lay = pm.lay
    if a.ref == "sim":
        xs = pm.P[:, lay.p_ref + lay.x(0)[0]:lay.p_ref + lay.x(0)[0] + k3.NX].clone()
        t = time.perf_counter()
        R = simulated_reference(pm, xs)
        print(f"simulated reference {time.perf_counter() - t:.2f} s", flush=True)
        gen = torch.Generator().manual_seed(11)
        pm.P[:, lay.p_ref:lay.p_ref + lay.n_v] = R
        noise = torch.zeros(B, k3.NX, dtype=torch.float64)
        noise[:, list(CONSISTENT_X0)] = 0.01 * torch.randn(B, len(CONSISTENT_X0), generator=gen, dtype=torch.float64)
        pm.P[:, lay.p_x0:lay.p_x0 + k3.NX] = xs + noise.cuda()
        pm.V.copy_(R)
    V_init = pm.V.clone()
    pm.ev.eval_nlp_device(pm.V, pm.P, pm.f, pm.g, pm.grad, pm.jac)
    gp = pm.g[:, pm.path_t].view(B, lay.n_k, -1).cpu().numpy()
    print("initial path rows (k, row) max:", gp.max(axis=(0,)).round(3).tolist(), flush=True)
    v = pm.V.cpu().numpy()
    bad = [np.where((v[b] < pm.lbx - 1e-9) | (v[b] > pm.ubx + 1e-9))[0][:10].tolist() for b in range(B)]
    print("initial bound violations:", bad, flush=True)
    for _ in range(10):
        eq, pmax = BatchedRti.iterate(pm)
    torch.cuda.synchronize()
    Vr = pm.V.cpu().numpy()
    print("rti eq", eq.cpu().numpy(), "path max", pmax.cpu().numpy(), flush=True)
    pm.V.copy_(V_init)
    t = time.perf_counter()
    res = pm.solve()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"solve {dt:.2f} s", [(r.status, r.iterations, f"{r.kkt_error:.1e}") for r in res], flush=True)
    Vp = pm.V.cpu().numpy()
    free = pm.free
    lb, ub = pm.lbx[free], pm.ubx[free]
    for b in range(B):
        gl, gu = Vp[b, free] - lb, ub - Vp[b, free]
        act = free[(gl < 1e-4) | (gu < 1e-4)]
        viol_r = free[(Vr[b, free] < lb - 1e-6) | (Vr[b, free] > ub + 1e-6)]
        print(f"loop {b}: f={res[b].f:.4e} active bounds {len(act)} {act[:8].tolist()} "
              f"rti violations {len(viol_r)} max|Vp-Vr|={np.abs(Vp[b, free] - Vr[b, free]).max():.3e}", flush=True)
    for b in range(B):
        if res[b].status != "solve_succeeded":
            print(f"loop {b} log:", res[b].log[-3:], flush=True)
    for s in range(a.steps):
        t = time.perf_counter()
        out = pm.step()
        torch.cuda.synchronize()
        print(f"step {s}: {time.perf_counter() - t:.2f} s status {out['status']} it {out['iterations'].tolist()} "
              f"track {out['tracking_error'].cpu().numpy().round(3).tolist()}", flush=True)


if __name__ == "__main__":
    main()
