"""Find the operation that gives identical instances different bits, without changing the solver's
timing: every wrapped operation compares its inputs and outputs across the batch's instances ON THE
DEVICE (no host synchronisation) and appends a 0-d flag "inputs equal and outputs differ"; after the
run the flags come back in one copy and the first raised one names the operation and call.

    python tools/lazy_probe.py [--B 128] [--runs 3] [--final-only]
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

FLAGS = []          # (label, call, flag tensor, differing-instance mask tensor)
CNT = {}
B_ = [1]


def _rows(t):
    B = B_[0]
    if not torch.is_tensor(t) or not t.is_cuda or t.numel() == 0 or t.dim() == 0 or t.shape[0] % B:
        return None
    return t.reshape(B, -1)


def _eq_rows(t):
    """[B] bool: row b equals row 0 (NaN equal to NaN), or None when t has no batch rows."""
    r = _rows(t)
    if r is None:
        return None
    same = (r == r[0:1]) | (torch.isnan(r) & torch.isnan(r[0:1])) if r.is_floating_point() else (r == r[0:1])
    return same.all(1)


def _all_eq(ts):
    f = None
    for t in ts:
        e = _eq_rows(t)
        if e is not None:
            f = e.all() if f is None else (f & e.all())
    return f


def wrap_fn(mod, name, ins, outs):
    orig = getattr(mod, name)

    @functools.wraps(orig)
    def w(*a, **k):
        label = f"{getattr(mod, '__name__', mod)}.{name}"
        CNT[label] = CNT.get(label, 0) + 1
        same_in = _all_eq(ins(a, k))
        r = orig(*a, **k)
        if same_in is not None:
            for ol, t in outs(r, a, k):
                e = _eq_rows(t)
                if e is not None:
                    FLAGS.append((f"{label}:{ol}", CNT[label], same_in & ~e.all(), ~e))
        return r
    setattr(mod, name, w)


def install():
    from awebox_amd import batched_lu, det, ipm
    T = lambda *xs: list(xs)  # noqa: E731
    wrap_fn(batched_lu, "lu_factor", lambda a, k: T(a[0]), lambda r, a, k: [("LU", r[0]), ("piv", r[1])])
    wrap_fn(batched_lu, "lu_solve", lambda a, k: T(a[0], a[1], a[2]), lambda r, a, k: [("X", r)])
    wrap_fn(batched_lu, "btd_factor", lambda a, k: T(a[0]), lambda r, a, k: [("F", r[0]), ("Dinv", r[1])])
    wrap_fn(batched_lu, "btd_solve", lambda a, k: T(a[0], a[1], a[2]), lambda r, a, k: [("X", r)])
    wrap_fn(batched_lu, "sym_inertia", lambda a, k: T(a[0]), lambda r, a, k: [("counts", r)])
    wrap_fn(det, "row_sum", lambda a, k: T(a[0]), lambda r, a, k: [("s", r)])
    wrap_fn(det, "bmm", lambda a, k: T(a[0], a[1]), lambda r, a, k: [("C", r)])

    def wrap_m(cls, name, ins, outs):
        orig = getattr(cls, name)

        @functools.wraps(orig)
        def w(self, *a, **k):
            label = f"{cls.__name__}.{name}"
            CNT[label] = CNT.get(label, 0) + 1
            same_in = _all_eq(ins(self, a, k))
            r = orig(self, *a, **k)
            if same_in is not None:
                for ol, t in outs(self, r, a, k):
                    e = _eq_rows(t)
                    if e is not None:
                        FLAGS.append((f"{label}:{ol}", CNT[label], same_in & ~e.all(), ~e))
            return r
        setattr(cls, name, w)
    wrap_m(ipm.DeviceNlp, "eval_all", lambda s, a, k: [a[0]],
           lambda s, r, a, k: [("f", r[0]), ("grad", r[1]), ("g", r[2]), ("jv", r[3])])
    wrap_m(ipm.DeviceNlp, "eval_fg", lambda s, a, k: [a[0]], lambda s, r, a, k: [("f", r[0]), ("g", r[1])])
    wrap_m(ipm.DeviceNlp, "hess", lambda s, a, k: [a[0], a[1]], lambda s, r, a, k: [("H", r)])
    wrap_m(ipm.StructuredKKT, "factor", lambda s, a, k: [a[0], a[1], a[2]],
           lambda s, r, a, k: [("vals", s.vals), ("KII", s.KII)])
    wrap_m(ipm.StructuredKKT, "_solve", lambda s, a, k: [a[0]], lambda s, r, a, k: [("sol", r)])
    wrap_m(ipm.StructuredKKT, "matvec", lambda s, a, k: [a[0]], lambda s, r, a, k: [("Kx", r)])
    wrap_m(ipm.StructuredKKT, "inertia", lambda s, a, k: [s.KII], lambda s, r, a, k: [("inertia", r)])
    orig_sc = ipm._ScatterSum.add_into_sel

    def sc_sel(self, out, vals, sel):
        CNT["add_into_sel"] = CNT.get("add_into_sel", 0) + 1
        same_in = _all_eq([out, vals])
        r = orig_sc(self, out, vals, sel)
        e = _eq_rows(r)
        if same_in is not None and e is not None:
            FLAGS.append(("_ScatterSum.add_into_sel", CNT["add_into_sel"], same_in & ~e.all(), ~e))
        return r
    ipm._ScatterSum.add_into_sel = sc_sel


def report():
    if not FLAGS:
        return {"flags": 0}
    fl = torch.stack([f[2] for f in FLAGS]).cpu().numpy()
    hit = np.where(fl)[0]
    if not len(hit):
        return {"flags": len(FLAGS), "divergence": None}
    i = hit[0]
    lab, call, _, mask = FLAGS[i]
    return {"flags": len(FLAGS), "first": {"op": lab, "call": int(call), "index": int(i),
                                          "instances": mask.nonzero().flatten().tolist()[:10]},
            "next": [(FLAGS[j][0], int(FLAGS[j][1])) for j in hit[1:6]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=128)
    ap.add_argument("--runs", type=int, default=3)
    args = ap.parse_args()
    from awebox_amd import homotopy as hm
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import IpmOptions, solve_batch
    from awebox_amd.trajectory import hippo_options, optimize
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    ev1 = Ap2Evaluator(consts, batch=1)
    _, _, _, res = optimize(consts, ev1, IpmOptions(max_iter=2000), final_step="power1")
    st = hm.schedule(consts, lay, v0)[-1]
    lbg, ubg = lay.g_bounds()
    P = pb.pack_p(lay, consts, v0, step=st.cost_step)
    B = B_[0] = args.B
    ev = Ap2Evaluator(consts, batch=B)
    ev.path = "colour"
    install()
    for run in range(args.runs):
        FLAGS.clear()
        CNT.clear()
        out = solve_batch(ev, np.tile(P, (B, 1)), np.tile(res.x, (B, 1)), st.lbx, st.ubx, lbg, ubg,
                          lam0=np.tile(res.lam_g, (B, 1)), zl0=np.tile(res.zl, (B, 1)), zu0=np.tile(res.zu, (B, 1)),
                          opts=hippo_options("final", IpmOptions(max_iter=2000)))
        differ = [b for b in range(B) if not np.array_equal(out[b].x, out[0].x)]
        print(json.dumps({"run": run, "iters": sorted(set(r.iterations for r in out)), "differ": differ[:10],
                          **report()}), flush=True)


if __name__ == "__main__":
    main()
