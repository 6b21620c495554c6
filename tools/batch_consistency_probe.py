"""Which operation of the batched solve gives identical instances different bits?

Runs the AP2 N=40 final homotopy step for K identical instances in one batch (ipm.solve_batch) with
the solver's building blocks wrapped: whenever every instance enters an operation with the same
inputs, the operation's outputs must be the same for every instance; the first operation that breaks
this is reported (its name, the call count, which instances differ) and the run stops.

    python tools/batch_consistency_probe.py [--K 64] [--path colour]
"""
import argparse
import functools
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class Broken(Exception):
    pass


CALLS = {}


def rows_equal(t):
    if t is None or not torch.is_tensor(t) or t.dim() == 0 or t.shape[0] < 2:
        return True, []
    t2 = t.reshape(t.shape[0], -1)
    eq = (t2 == t2[0:1]) | (torch.isnan(t2) & torch.isnan(t2[0:1]))
    bad = (~eq.all(1)).nonzero().flatten().tolist()
    return not bad, bad


def blocks_equal(t, B):
    """[B * n_k, ...] tensors: instance-major blocks."""
    if t is None or not torch.is_tensor(t) or t.shape[0] % B:
        return True, []
    return rows_equal(t.reshape(B, -1))


def wrap(cls, name, in_fn, out_fn):
    orig = getattr(cls, name)

    @functools.wraps(orig)
    def w(self, *a, **k):
        key = f"{cls.__name__}.{name}"
        CALLS[key] = CALLS.get(key, 0) + 1
        ins = in_fn(self, a, k)
        same_in = all(rows_equal(t)[0] for t in ins)
        r = orig(self, *a, **k)
        if same_in:
            for label, t, blk in out_fn(self, r, a, k):
                ok, bad = blocks_equal(t, blk) if blk else rows_equal(t)
                if not ok:
                    raise Broken(json.dumps({"op": key, "call": CALLS[key], "output": label, "instances": bad[:20],
                                             "n_bad": len(bad), "calls": CALLS}))
        return r
    setattr(cls, name, w)


def install():
    """Wrap the solver's building blocks (see the module docstring)."""
    from awebox_amd import ipm
    wrap(ipm.DeviceNlp, "eval_all", lambda s, a, k: [a[0]],
         lambda s, r, a, k: [("f", r[0], 0), ("grad", r[1], 0), ("g", r[2], 0), ("jv", r[3], 0)])
    wrap(ipm.DeviceNlp, "eval_fg", lambda s, a, k: [a[0]], lambda s, r, a, k: [("f", r[0], 0), ("g", r[1], 0)])
    wrap(ipm.DeviceNlp, "hess", lambda s, a, k: [a[0], a[1]], lambda s, r, a, k: [("H", r, 0)])
    wrap(ipm.StructuredKKT, "factor", lambda s, a, k: [a[0], a[1], a[2]],
         lambda s, r, a, k: [("KII", s.KII, s.B), ("LU_I", s.LU_I, s.B), ("X", s.X, s.B), ("vals", s.vals, 0),
                             ("Tf0", s.btd.Tf[0] if s.use_btd and s.btd.fused else None, 0),
                             ("Tf1", s.btd.Tf[1] if s.use_btd and s.btd.fused else None, 0),
                             ("Z", s.btd.Z if s.use_btd and s.btd.nG else None, 0),
                             ("Cf", s.btd.Cf[0] if s.use_btd and s.btd.nG else None, 0)])
    wrap(ipm.StructuredKKT, "_solve", lambda s, a, k: [a[0]], lambda s, r, a, k: [("sol", r, 0)])
    wrap(ipm.StructuredKKT, "matvec", lambda s, a, k: [a[0]], lambda s, r, a, k: [("Kx", r, 0)])
    wrap(ipm.StructuredKKT, "inertia", lambda s, a, k: [], lambda s, r, a, k: [("inertia", r, 0)])



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--path", default="colour")
    args = ap.parse_args()
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import final_step_ensemble, optimize
    install()
    consts = pb.build_constants()
    ev1 = Ap2Evaluator(consts, batch=1)
    _, summary, _, res = optimize(consts, ev1, IpmOptions(max_iter=2000), final_step="power1", eval_path=args.path)
    ev = Ap2Evaluator(consts, batch=args.K)
    ev.path = args.path
    try:
        members, hist = final_step_ensemble(consts, ev, (res.x, res.lam_g, res.zl, res.zu), args.K, eps=0.0)
        print(json.dumps({"result": "no divergence", "hist": hist, "iterations": [m["iterations"] for m in members],
                          "calls": CALLS}))
    except Broken as e:
        print(json.dumps({"result": "divergence", **json.loads(str(e))}))


if __name__ == "__main__":
    main()
