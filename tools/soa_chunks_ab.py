"""A/B of the instance-minor path's Radau / interval chunking (AWE_SOA_CHUNKS, read at awe_create):
the bench's AP2 evaluation (B = 2048, V and P instance-minor) timed per setting in one process, the
outputs compared bitwise with the unchunked launch.

    python tools/soa_chunks_ab.py [--reps 50]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--B", type=int, default=2048)
    ap.add_argument("--settings", default="1,2,4,8,1,4")
    args = ap.parse_args()
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import batch_member, initial_guess
    B = args.B
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device="cuda")
    P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0)] * B), device="cuda")
    ref = None
    for c in [int(x) for x in args.settings.split(",")]:
        os.environ["AWE_SOA_CHUNKS"] = str(c)
        ev = Ap2Evaluator(consts, batch=B)
        VT, PT = ev.alloc_inputs("cuda")
        VT.copy_(V)
        PT.copy_(P)
        f = torch.empty(B, dtype=torch.float64, device="cuda")
        g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
        gr, jac = ev.alloc_grad("cuda"), ev.alloc_jac("cuda")
        for _ in range(5):
            ev.eval_nlp_device(VT, PT, f, g, gr, jac)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ev.eval_nlp_device(VT, PT, f, g, gr, jac)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.reps * 1e3
        out = [x.cpu().numpy().copy() for x in (f, g, gr, jac)]
        same = None if ref is None else all(np.array_equal(a, b) for a, b in zip(ref, out))
        if ref is None:
            ref = out
        ks = ev.last_kernel_ms_soa()
        print(json.dumps({"chunks": c, "ms": ms, "evals_per_s": B / ms * 1e3, "bitwise_vs_first": same,
                          "events_ms": [round(x, 4) for x in ks]}), flush=True)
        del ev


if __name__ == "__main__":
    main()
