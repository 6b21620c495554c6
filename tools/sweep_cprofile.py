"""Host profile of the bench's sweep blocks (AP2 N=40 fan shard of 8 points; optionally the dual-kite
N=20 fan shard): wall time and cProfile's top functions, to find the host-side cost per iteration.

    python tools/sweep_cprofile.py [--arch ap2|dual] [--points 8] [--out gpurun_out/sweep_cprofile_ap2.txt]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ap2")
    ap.add_argument("--points", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch

    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    u = list(np.linspace(5.0, 8.0, 64)[:a.points])
    if a.arch == "ap2":
        from awebox_amd import problem as pb
        from awebox_amd.evaluator import Ap2Evaluator
        consts = pb.build_constants()
        kw = dict(n_k=consts.cfg.n_k, d=consts.cfg.d, make_evaluator=lambda c, b=1: Ap2Evaluator(c, batch=b),
                  opts=IpmOptions(max_iter=1000))
    else:
        from awebox_amd.dual_homotopy import make_evaluator
        kw = dict(n_k=20, d=4, make_evaluator=lambda c, b=1: make_evaluator(c, device="cuda", batch=b),
                  opts=IpmOptions(max_iter=3000), arch="dual")
    prof = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prof.enable()
    res = run_sweep(u, dist=None, device="cuda", mode="fan", **kw)
    torch.cuda.synchronize()
    prof.disable()
    wall = time.perf_counter() - t0
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats("tottime").print_stats(45)
    st.sort_stats("cumulative").print_stats(45)
    text = f"wall {wall:.3f} s trials/s {res['trials_per_s']:.4f} iterations {res['iterations']}\n" + s.getvalue()
    out = a.out or os.path.join(ROOT, "gpurun_out", f"sweep_cprofile_{a.arch}.txt")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as fh:
        fh.write(text)
    print(text[:3000])


if __name__ == "__main__":
    main()
