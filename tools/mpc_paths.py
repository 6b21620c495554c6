"""Tracking-MPC evaluator paths on the GPU: the dual-number kernel (awempc_eval_nlp) against the
generated instance-minor path (awempc_eval_nlp_im) at the bench's batch -- kernel times from HIP events
and wall-clock evaluations/s of a timed loop.  One JSON line per path.

    python tools/mpc_paths.py [--batch 256] [--steps 200]
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
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import torch

    from awebox_amd import kite3 as k3
    from awebox_amd.mpc import MpcEvaluator

    c = k3.build_constants()
    lay = k3.MpcLayout(c.cfg.n_k, c.cfg.d)
    B = args.batch
    orbit = k3.CircularOrbit(c.cfg)
    inst = [k3.batch_instance(c, lay, i, B, orbit=orbit) for i in range(B)]
    dev = torch.device("cuda", 0)
    V = torch.tensor(np.stack([v for v, _ in inst]), device=dev)
    P = torch.tensor(np.stack([p for _, p in inst]), device=dev)
    ev = MpcEvaluator(c, batch=B)
    f = torch.empty(B, dtype=torch.float64, device=dev)
    g = torch.empty(B, ev.n_g, dtype=torch.float64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for im in (False, True):
        gr, jac = ev.alloc_grad(dev, instance_minor=im), ev.alloc_jac(dev, instance_minor=im)
        for _ in range(5):
            ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        parts = []
        for _ in range(20):
            ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
            parts.append(ev.last_kernel_ms_im() if im else ev.last_kernel_ms())
        parts = np.mean(parts, axis=0).tolist()
        print(json.dumps({"path": "generated_im" if im else "dual", "batch": B, "wall_ms_per_eval": el / args.steps * 1e3,
                          "evals_per_s_wall": B * args.steps / el, "kernel_ms": parts,
                          "evals_per_s_kernel": B / (sum(parts) * 1e-3),
                          "finite": bool(torch.isfinite(jac).all().item())}), flush=True)


if __name__ == "__main__":
    main()
