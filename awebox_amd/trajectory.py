"""Trajectory optimisation of the AP2 power cycle on the GPU: the homotopy loop of
awebox/opti/optimization.py:273-382 (solve_homotopy -> solve_specific_homotopy_step ->
solve_general_homotopy_step) around the GPU interior-point solver (ipm.py) and the HIP
evaluator.  Each step updates P's cost vector and the variable bounds (homotopy.schedule) and
warm-starts from the previous solution and multipliers.
"""
from __future__ import annotations

import time

import numpy as np

from . import homotopy as hm
from . import problem as pb
from .initial_guess import initial_guess
from .ipm import IpmOptions, solve, solve_batch


def hippo_options(label: str, base: IpmOptions | None = None) -> IpmOptions:
    """awebox's hippo strategy (preparation.py:285-323, default.py:324-351): the initial and
    intermediate homotopy steps stop at the barrier parameter mu_target = 1e-2 with tol 1e-4
    (initial: mu_init 1, cold start; middle: mu_init 1e-2, warm start); the final step starts at
    mu_init 1e-2 and converges to tol 1e-8 (mu_target 0).  The hippo steps set IPOPT's
    acceptable_iter to 5 (acceptable_iter_hippo); the final step keeps IPOPT's default 15."""
    import dataclasses
    base = base or IpmOptions()
    if label.startswith("initial"):
        return dataclasses.replace(base, mu_init=1.0, mu_target=1e-2, tol=1e-4, acceptable_iter=5)
    if label.startswith("final"):
        return dataclasses.replace(base, mu_init=1e-2, mu_target=0.0, tol=1e-8)
    return dataclasses.replace(base, mu_init=1e-2, mu_target=1e-2, tol=1e-4, acceptable_iter=5)


# Evaluation path of the homotopy drivers.  The final homotopy step crosses a
# non-convex region in which the regularised Newton map expands roundoff ~1.2x per iteration, so the
# local optimum it ends on depends on the last bits of the evaluation (35.9 / 51.7 / 53.6 / 70 s
# branches under 1e-13 perturbations, profiles/r06/ensemble/).  The drivers run one path for every
# batch size -- the colour kernel with the hyper-dual Hessian -- because each evaluation path rounds
# differently; together with the solver's batch-invariant sums and products (det.py) and race-free
# inertia kernels, a problem solved alone or inside a batch of any size then follows the same iterates
# bitwise (tests/test_regression.py::test_ap2_n40_batched_homotopy_b128, tests/test_det_gpu.py).
# Which branch the default run lands on is still a matter of its rounding (round 6: the t_f bound).
# eval_path=None keeps the evaluator's own path.
HOMOTOPY_EVAL_PATH = "colour"


class _pinned_path:
    """Run the evaluator on ``eval_path`` (with the Hessian following it) inside the block and
    restore the caller's path and Hessian mode afterwards (None: leave the evaluator alone)."""

    def __init__(self, ev, eval_path):
        self.ev, self.eval_path = ev, eval_path

    def __enter__(self):
        ev = self.ev
        self.saved = None
        if self.eval_path is not None and hasattr(ev, "path"):
            self.saved = (ev.path, getattr(ev, "hess_mode", None))
            ev.path = self.eval_path
            if hasattr(ev, "hess_path"):
                ev.hess_path = "follow"
        return ev

    def __exit__(self, *exc):
        if self.saved is not None:
            path, hmode = self.saved
            self.ev.path = path
            if hmode is not None:
                self.ev.hess_path = hmode
        return False


def optimize(consts: pb.Ap2Constants, ev, opts: IpmOptions | None = None, device="cuda",
             v_init: np.ndarray | None = None, final_step: str | None = None, verbose=False,
             u_ref: float | None = None, keep_logs=False, eval_path: str | None = HOMOTOPY_EVAL_PATH):
    """Run the homotopy; returns (V_opt, per-step summaries, outputs, last IpmResult).
    ``u_ref`` overrides the wind reference speed in P (the sweep parameter); ``eval_path`` is the
    evaluation path the homotopy runs on (HOMOTOPY_EVAL_PATH; None: the evaluator's own)."""
    with _pinned_path(ev, eval_path):
        return _optimize(consts, ev, opts, device, v_init, final_step, verbose, u_ref, keep_logs)


def _optimize(consts, ev, opts, device, v_init, final_step, verbose, u_ref, keep_logs):
    lay = pb.NlpLayout(consts.cfg.n_k, consts.cfg.d)
    v0 = initial_guess(consts, lay) if v_init is None else v_init
    steps = hm.schedule(consts, lay, v0)
    lbg, ubg = lay.g_bounds()
    x, lam, zl, zu = v0.copy(), None, None, None
    summary = []
    for st in steps:
        P = pb.pack_p(lay, consts, v0, step=st.cost_step, u_ref=u_ref)
        t0 = time.perf_counter()
        res = solve(ev, P, x, st.lbx, st.ubx, lbg, ubg, lam0=lam, zl0=zl, zu0=zu,
                    opts=hippo_options(st.label, opts), device=device)
        out = hm.outputs(consts, lay, res.x)
        rec = dict(step=st.label, status=res.status, iterations=res.iterations, f=res.f,
                   kkt_error=res.kkt_error, constr_viol=res.constr_viol, seconds=time.perf_counter() - t0,
                   **out)
        if res.timing:
            rec["timing"] = {k: round(v, 3) for k, v in res.timing.items()}
        if keep_logs:
            rec["log"] = res.log
        summary.append(rec)
        if verbose:
            print(rec, flush=True)
        x, lam, zl, zu = res.x, res.lam_g, res.zl, res.zu
        if final_step is not None and st.label == final_step:
            break
    return x, summary, hm.outputs(consts, lay, x), res


def optimize_batch(consts: pb.Ap2Constants, ev, u_refs, opts: IpmOptions | None = None, device="cuda",
                   v_init: np.ndarray | None = None, verbose=False, eval_path: str | None = HOMOTOPY_EVAL_PATH):
    """The homotopy for B = len(u_refs) wind speeds at once (ev.batch == B): every step is one
    batched interior-point solve (ipm.solve_batch) in which each instance keeps its own IPOPT
    iteration; all instances share the layout, bounds and schedule, and differ in P's u_ref.
    Returns (V [B, n_v], per-step summaries (lists over instances), outputs per instance, results)."""
    with _pinned_path(ev, eval_path):
        return _optimize_batch(consts, ev, u_refs, opts, device, v_init, verbose)


def _optimize_batch(consts, ev, u_refs, opts, device, v_init, verbose):
    lay = pb.NlpLayout(consts.cfg.n_k, consts.cfg.d)
    v0 = initial_guess(consts, lay) if v_init is None else v_init
    B = len(u_refs)
    steps = hm.schedule(consts, lay, v0)
    lbg, ubg = lay.g_bounds()
    x = np.tile(v0, (B, 1))
    lam = zl = zu = None
    summary = []
    res = None
    for st in steps:
        P = np.stack([pb.pack_p(lay, consts, v0, step=st.cost_step, u_ref=u) for u in u_refs])
        t0 = time.perf_counter()
        res = solve_batch(ev, P, x, st.lbx, st.ubx, lbg, ubg, lam0=lam, zl0=zl, zu0=zu,
                          opts=hippo_options(st.label, opts), device=device)
        rec = dict(step=st.label, status=[r.status for r in res], iterations=[r.iterations for r in res],
                   f=[r.f for r in res], seconds=time.perf_counter() - t0)
        summary.append(rec)
        if verbose:
            print(rec, flush=True)
        x = np.stack([r.x for r in res])
        lam = np.stack([r.lam_g for r in res])
        zl = np.stack([r.zl for r in res])
        zu = np.stack([r.zu for r in res])
    return x, summary, [hm.outputs(consts, lay, x[b]) for b in range(B)], res


# period branches of the AP2 N=40 final step
AP2_BRANCHES = (("35.9", 33.0, 40.0), ("51.7", 50.0, 53.0), ("53.6", 53.0, 55.0), ("58.4", 56.0, 61.0),
                ("66-70", 64.0, 70.5))


def period_branch(period_s: float) -> str:
    for name, lo, hi in AP2_BRANCHES:
        if lo <= period_s <= hi:
            return name
    return f"other:{period_s:.1f}"


def final_step_ensemble(consts: pb.Ap2Constants, ev, start, K: int, eps: float = 1e-13, seed: int = 11,
                        opts: IpmOptions | None = None, device="cuda"):
    """Branch statistics of the homotopy's final step: K final-step solves from
    the power1 point ``start`` = (x, lam_g, zl, zu) at once (ipm.solve_batch, ev.batch == K), member 0
    from the point itself, member b > 0 from x (1 + eps N(0, 1)) (seeded), all with its multipliers.
    Returns (per-member records {status, iterations, f, period_s, avg_power_W, branch}, histogram)."""
    import dataclasses
    lay = pb.NlpLayout(consts.cfg.n_k, consts.cfg.d)
    v0 = initial_guess(consts, lay)
    st = hm.schedule(consts, lay, v0)[-1]
    lbg, ubg = lay.g_bounds()
    P = pb.pack_p(lay, consts, v0, step=st.cost_step)
    x1, lam1, zl1, zu1 = start
    noise = np.random.default_rng(seed).standard_normal((K, lay.n_v))
    noise[0] = 0.0
    X0 = x1[None, :] * (1.0 + eps * noise)
    o = hippo_options("final", dataclasses.replace(opts or IpmOptions(), max_iter=3000))
    res = solve_batch(ev, np.tile(P, (K, 1)), X0, st.lbx, st.ubx, lbg, ubg, lam0=np.tile(lam1, (K, 1)),
                      zl0=np.tile(zl1, (K, 1)), zu0=np.tile(zu1, (K, 1)), opts=o, device=device)
    members, hist = [], {}
    for r in res:
        out = hm.outputs(consts, lay, r.x)
        br = period_branch(out["period_s"])
        hist[br] = hist.get(br, 0) + 1
        members.append(dict(status=r.status, iterations=r.iterations, f=r.f, period_s=out["period_s"],
                            avg_power_W=out["avg_power_W"], branch=br))
    return members, hist
