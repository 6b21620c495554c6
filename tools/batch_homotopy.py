"""Batch-size independence of the AP2 N=40 homotopy: the default homotopy of one
instance (trajectory.optimize) against the same problem inside a batch of B identical instances
(trajectory.optimize_batch), both on the homotopy drivers' pinned evaluation path.  Prints one JSON
line: iterations, period and power of the single run, and for the batch whether every member's V is
bitwise the single run's.

    python tools/batch_homotopy.py [B]
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")


def main():
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize, optimize_batch
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    consts = pb.build_constants()
    t0 = time.perf_counter()
    V1, s1, o1, _ = optimize(consts, Ap2Evaluator(consts, batch=1), IpmOptions(max_iter=2000))
    t1 = time.perf_counter()
    ev = Ap2Evaluator(consts, batch=B)
    VB, sB, oB, _ = optimize_batch(consts, ev, [10.0] * B, IpmOptions(max_iter=2000))
    t2 = time.perf_counter()
    same = [bool(np.array_equal(VB[b], V1)) for b in range(B)]
    print(json.dumps({"batch": B, "path": ev.path, "hess": ev.hess_path,
                      "single": {"iterations": [r["iterations"] for r in s1], "period_s": o1["period_s"],
                                 "avg_power_W": o1["avg_power_W"], "seconds": t1 - t0},
                      "batch_iterations_member0": [r["iterations"][0] for r in sB],
                      "batch_periods": sorted({round(o["period_s"], 6) for o in oB}),
                      "members_bitwise_equal_single": int(sum(same)), "seconds_batch": t2 - t1}), flush=True)


if __name__ == "__main__":
    main()
