"""Host-side profile (cProfile) of the batched homotopy of 8 AP2 wind speeds at N=40 d=4 on the GPU:
where the interior-point solver's wall time goes outside the device kernels (Python orchestration,
torch launches, host syncs).  Writes gpurun_out/solver_pstats.txt (top functions by own time and
by cumulative time)."""
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize_batch
    consts = pb.build_constants(pb.Ap2Config(n_k=40, d=4))
    u = np.linspace(5.0, 8.0, 8)
    ev = Ap2Evaluator(consts, batch=8)
    optimize_batch(consts, ev, u[:1].repeat(8), IpmOptions(max_iter=3))      # warm-up: kernels, tables
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    _, summary, outs, _ = optimize_batch(consts, ev, u, IpmOptions(max_iter=1000))
    pr.disable()
    wall = time.perf_counter() - t0
    out = io.StringIO()
    out.write(f"wall {wall:.2f} s, iterations per step {[max(r['iterations']) for r in summary]}\n")
    for key in ("tottime", "cumulative"):
        st = pstats.Stats(pr, stream=out)
        st.sort_stats(key).print_stats(45)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/solver_pstats.txt", "w") as fh:
        fh.write(out.getvalue())
    print(f"wall {wall:.2f} s", flush=True)


if __name__ == "__main__":
    main()
