"""Dual-kite evaluator paths on the GPU: the colour kernel (adl_eval_nlp) against the generated
instance-minor path (adl_eval_nlp_im) at the bench's config-3 batch (N=60 d=4, 128 instances) --
kernel times from HIP events, wall-clock evaluations/s of a timed loop, output checksums.

    python tools/dual_paths.py [--batch 128] [--n-k 60] [--steps 50] [--lib path]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--n-k", type=int, default=60)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch

    from awebox_amd import dual as du
    from awebox_amd import dual_evaluator as de

    if args.lib:
        de.load_library(args.lib)
    mc = du.build_constants(du.MultiConfig(n_k=args.n_k, d=4))
    lay = du.layout_for(mc)
    v0 = du.initial_guess(mc, lay)
    B = args.batch
    V = torch.tensor(np.stack([du.batch_member(v0, lay, b) for b in range(B)]), device="cuda")
    P = torch.tensor(np.stack([du.pack_p(lay, mc, v0, u_ref=5.0 + 3.0 * b / max(B - 1, 1)) for b in range(B)]),
                     device="cuda")
    ev = de.DualEvaluator(mc, batch=B)
    f = torch.empty(B, dtype=torch.float64, device="cuda")
    g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for im in (False, True):
        if im and not ev.generated_available:
            print(json.dumps({"path": "generated_im", "available": False}), flush=True)
            continue
        gr, jac = ev.alloc_grad("cuda", instance_minor=im), ev.alloc_jac("cuda", instance_minor=im)
        for _ in range(3):
            ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        parts = []
        for _ in range(10):
            ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
            parts.append(ev.last_kernel_ms_im() if im else ev.last_kernel_ms())
        parts = np.median(np.array(parts), axis=0).tolist()
        print(json.dumps({"path": "generated_im" if im else "colour", "batch": B, "n_k": args.n_k,
                          "wall_ms_per_eval": el / args.steps * 1e3, "evals_per_s_wall": B * args.steps / el,
                          "kernel_ms": parts, "evals_per_s_kernel": B / (sum(parts) * 1e-3),
                          "jac_sum": float(jac.sum()), "g_sum": float(g.sum()), "grad_sum": float(gr.sum()),
                          "f_sum": float(f.sum()), "finite": bool(torch.isfinite(jac).all().item())}), flush=True)


if __name__ == "__main__":
    main()
