"""Is the batched inertia kernel deterministic?  The interval blocks (awelu sym_inertia, blocked
kernel, n ~ 250) and the separator pivot blocks (unblocked kernel, m = 46) of the AP2 N=40 KKT at a
final-step iterate, each block replicated over a batch of 128 instances, counted `--repeat` times:
every copy of a block must get the same counts every time.  Also the LU factor and the block sweep."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--repeat", type=int, default=40)
    ap.add_argument("--iters", type=int, default=60)
    args = ap.parse_args()
    from awebox_amd import ipm
    from awebox_amd import problem as pb
    from awebox_amd.batched_lu import btd_factor, lu_factor, sym_inertia
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize
    grabbed = {}
    orig = ipm.StructuredKKT.inertia

    def grab(self):
        grabbed["KII"] = self.KII.clone()
        if self.use_btd and self.btd.fused:
            grabbed["D"] = self.btd.Tf[0][:, :, 1].clone()
            grabbed["T"] = None
        return orig(self)
    ipm.StructuredKKT.inertia = grab
    consts = pb.build_constants()
    ev1 = Ap2Evaluator(consts, batch=1)
    optimize(consts, ev1, IpmOptions(max_iter=args.iters), final_step="final0")
    ipm.StructuredKKT.inertia = orig
    KII = grabbed["KII"]                                      # [n_k, nI, nI]
    D = grabbed["D"][0]                                       # [nb, m, m]
    n_k, nI = KII.shape[0], KII.shape[1]
    B = args.B
    big = KII.repeat(B, 1, 1).contiguous()
    bigD = D.repeat(B, 1, 1).contiguous()
    ref = sym_inertia(KII, ztol=ipm.ZERO_PIVOT).cpu()
    refD = sym_inertia(D.contiguous(), ztol=ipm.ZERO_PIVOT).cpu()
    bad = {"blocked": 0, "unblocked": 0, "lu": 0}
    first = {}
    LU0, _ = lu_factor(KII)
    LU0 = LU0.cpu()
    for rep in range(args.repeat):
        c = sym_inertia(big, ztol=ipm.ZERO_PIVOT).cpu().view(B, n_k, 3)
        diff = (c != ref[None]).any(-1).nonzero().tolist()
        if diff:
            bad["blocked"] += 1
            first.setdefault("blocked", (rep, diff[:5]))
        cD = sym_inertia(bigD, ztol=ipm.ZERO_PIVOT).cpu().view(B, -1, 3)
        diffD = (cD != refD[None]).any(-1).nonzero().tolist()
        if diffD:
            bad["unblocked"] += 1
            first.setdefault("unblocked", (rep, diffD[:5]))
        if rep % 8 == 0:
            LU, _ = lu_factor(big)
            LUc = LU.cpu().view(B, n_k, nI, nI)
            dl = (LUc != LU0[None]).flatten(2).any(-1).nonzero().tolist()
            if dl:
                bad["lu"] += 1
                first.setdefault("lu", (rep, dl[:5]))
    print(json.dumps({"n_k": n_k, "nI": nI, "m": D.shape[-1], "B": B, "repeat": args.repeat, "bad_repeats": bad,
                      "first": first, "ref_counts_sum": ref.sum(0).tolist()}), flush=True)


if __name__ == "__main__":
    main()
