"""GPU lab: the rk4root plant against the collocation plant, per loop, over closed-loop steps.

    python tools/plant_lab.py [--batch 256] [--steps 3] [--n-fe 20] [--all-x0]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from awebox_amd import kite3 as k3  # noqa: E402
from awebox_amd.rti import BatchedRti  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--n-fe", type=int, default=20)
    ap.add_argument("--all-x0", action="store_true", help="x0 noise on every state (SURVEY spec)")
    ap.add_argument("--circle", action="store_true", help="track the synthetic circle")
    a = ap.parse_args()
    c = k3.build_constants()
    r = BatchedRti(c, a.batch, device="cuda", n_fe=a.n_fe)
    r.start(x0_entries=None if a.all_x0 else (6, 7, 10))
    if not a.circle:
        r.simulate_reference(a.steps + c.cfg.n_k + 1)
    for s in range(a.steps):
        r.iterate()
        x0 = r.P[:, :k3.NX].clone()
        x_c, res_c = r._plant()
        x_r, res_r = r._rk4root()
        step = (x_c - x0).abs().amax(dim=1)
        gap = (x_c - x_r).abs().amax(dim=1)
        ratio = gap / step
        q = torch.quantile(ratio, torch.tensor([0.5, 0.9, 0.99, 1.0], dtype=torch.float64, device="cuda"))
        w = int(ratio.argmax())
        print(f"step {s}: gap/step quantiles (50/90/99/max) {q.cpu().numpy()} worst loop {w}: gap {float(gap[w]):.3e} "
              f"step {float(step[w]):.3e} res_c {float(res_c[w]):.1e} res_r {float(res_r[w]):.1e} "
              f"worst per-state {(x_c[w] - x_r[w]).abs().cpu().numpy()}", flush=True)
        r._shift(x_c)
        r.step_count += 1


if __name__ == "__main__":
    main()
