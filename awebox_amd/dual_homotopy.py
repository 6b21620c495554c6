"""Bounds, homotopy schedule, outputs and the trajectory driver of the dual-kite power cycle
(config 3/4: examples/dual_kites_power_curve.py, phase_fix 'single_reelout').

Restates for the multi-kite layout of ``dual.py``:

* ``variable_bounds``: ``ocp/var_bounds.py:42-103`` with the 'single_reelout' phase fix of
  ``assign_phase_fix_bounds`` (``:105-200``): dl_t free at x[0], >= 0 on the reel-out control
  nodes, 0 at the switching node, <= 0 on the reel-in nodes; t_f components only >= 0 (the period
  is bounded by the two t_f rows of g); model bounds of every node (q_z >= 100 m, omega, delta,
  lambda >= 0) and the example's l_t in [0, 1000];
* ``schedule``: the power-cycle homotopy (``scheduling.py:37-104, 161-240, 424-470``) with
  ``set_initial_bounds`` (``preparation.py:150-227``): theta fixed at the initialization values,
  fictitious controls free, and -- because t_f has two components -- dl_t and l_t freed until the
  first power step restores their (phase-fix) bounds;
* ``outputs``: average power over the phase-fixed period (``ocp_outputs.py:118-140``).
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass

import numpy as np

from . import dual as du
from . import problem as pb

INF = math.inf


def _model_bounds_si(mc: du.MultiConstants) -> dict:
    """(var_type, name) -> (lb, ub) SI bounds of the model variables (system.define_bounds with
    default.py:186-215, ampyx_ap2_settings.py:43-60 and the example's l_t bounds)."""
    cfg, m = mc.cfg, mc.model
    om = 50.0 * math.pi / 180.0
    out = {}
    for (vt, n), (o, s) in m.off.items():
        base = pb.split_name(n)
        if vt == "x" and base == "q":
            out[(vt, n)] = (np.array([-INF, -INF, 100.0]), np.array([INF, INF, INF]))
        elif vt == "x" and base == "omega":
            out[(vt, n)] = (np.full(3, -om), np.full(3, om))
        elif vt == "x" and base == "delta":
            out[(vt, n)] = (-np.asarray(cfg.delta_max), np.asarray(cfg.delta_max))
        elif vt == "u" and base == "ddelta":
            out[(vt, n)] = (-np.asarray(cfg.ddelta_max), np.asarray(cfg.ddelta_max))
        elif vt == "z":
            out[(vt, n)] = (np.zeros(1), np.full(1, INF))
    out[("x", "l_t")] = (np.array([cfg.l_t_bounds[0]]), np.array([cfg.l_t_bounds[1]]))
    out[("x", "dl_t")] = (np.array([-15.0]), np.array([20.0]))
    out[("u", "ddl_t")] = (np.array([cfg.ddl_t_bounds[0]]), np.array([cfg.ddl_t_bounds[1]]))
    out[("theta", "diam_t")] = (np.array([cfg.diam_t_fixed]), np.array([cfg.diam_t_fixed]))
    out[("theta", "l_s")] = (np.array([1.0e-2]), np.array([1.0e3]))
    out[("theta", "diam_s")] = (np.array([1.0e-4]), np.array([1.0e-1]))
    return out


def variable_bounds(mc: du.MultiConstants, lay: du.MultiLayout):
    m, s = mc.model, mc.scaling
    lb = np.full(lay.n_v, -INF)
    ub = np.full(lay.n_v, INF)
    for (vt, name), (l_si, u_si) in _model_bounds_si(mc).items():
        o, n = m.off[(vt, name)]
        sc = s[o:o + n]
        ls, us = l_si / sc, u_si / sc
        if vt == "x":
            for k in range(lay.n_k):                  # zoh + periodic: x[0..n_k-1]
                idx = lay.x(k)[o:o + n]
                lb[idx], ub[idx] = ls, us
        elif vt == "u":
            for k in range(lay.n_k):
                idx = lay.u(k)[o - m.w_u0:o - m.w_u0 + n]
                lb[idx], ub[idx] = ls, us
        elif vt == "z":
            for k in range(lay.n_k):
                idx = lay.z(k)[o - m.w_z0:o - m.w_z0 + n]
                lb[idx], ub[idx] = ls, us
        elif vt == "theta":
            i = lay.theta_index(name)
            lb[i], ub[i] = ls[0], us[0]
    if lay.single_reelout:
        for nm in ("t_f0", "t_f1"):                   # var_bounds.py:84-89
            lb[lay.theta_index(nm)], ub[lay.theta_index(nm)] = 0.0, INF
        o, _ = m.off[("x", "dl_t")]
        dmax, dmin = 20.0 / s[o], -15.0 / s[o]
        for k in range(lay.n_k + 1):                  # assign_phase_fix_bounds
            i = lay.x(k)[o]
            if k == 0:
                lb[i], ub[i] = -INF, INF
            elif k == lay.n_k or k == lay.nk_reelout:
                lb[i], ub[i] = 0.0, 0.0
            elif k < lay.nk_reelout:
                lb[i], ub[i] = 0.0, dmax
            else:
                lb[i], ub[i] = dmin, 0.0
    lb[lay.v_xi:lay.v_xi + 2] = ub[lay.v_xi:lay.v_xi + 2] = 0.0
    return lb, ub


@dataclass
class Step:
    label: str
    cost_step: str
    lbx: np.ndarray
    ubx: np.ndarray


def _bound_updates(mc: du.MultiConstants):
    """scheduling.define_bounds_to_update for a lift-mode power cycle."""
    theta_sorted = sorted(n for n, _ in mc.model.TH)
    fict = sorted(n for n, _ in mc.model.U if "fict" in n)
    return [("initial", 0, [(n, "theta") for n in theta_sorted] * 2 + [("ddl_t", "u")] * 2),
            ("fictitious", 0, [("gamma", "phi")]),
            ("fictitious", 1, [("gamma", "phi")] + [(n, "u") for n in fict for _ in range(2)]),
            ("power", 0, [("psi", "phi")] + [("dl_t", "x")] * 2 + [("l_t", "x")] * 2),
            ("power", 1, [("psi", "phi")]),
            ("final", 0, [])]


def schedule(mc: du.MultiConstants, lay: du.MultiLayout, v_init: np.ndarray) -> list[Step]:
    m = mc.model
    lb0, ub0 = variable_bounds(mc, lay)
    lb, ub = lb0.copy(), ub0.copy()
    updates = _bound_updates(mc)
    upd_phi = {n for _, _, ups in updates for n, vt in ups if vt == "phi"}
    for i, name in enumerate(pb.PHI_NAMES):
        lb[lay.phi()[i]] = ub[lay.phi()[i]] = 1.0 if name in upd_phi else 0.0
    init_si = {"diam_t": mc.cfg.diam_t_init, "l_s": mc.cfg.l_s_init, "diam_s": mc.cfg.diam_s_init}
    for name, val in init_si.items():                 # preparation.py:176-182
        i = lay.theta_index(name)
        lb[i] = ub[i] = val / mc.scaling[m.off[("theta", name)][0]]
    tf_idx = [lay.theta_index(n) for n in lay.theta_names if n.startswith("t_f")]
    for i in tf_idx:
        lb[i] = ub[i] = v_init[i]
    for name in (n for n, _ in m.U if "fict" in n):
        o, n = m.off[("u", name)]
        for k in range(lay.n_k):
            idx = lay.u(k)[o - m.w_u0:o - m.w_u0 + n]
            lb[idx], ub[idx] = -INF, INF
    if lay.single_reelout:                            # preparation.py:203-214
        for name in ("dl_t", "l_t"):
            o, _ = m.off[("x", name)]
            for k in range(lay.n_k + 1):
                lb[lay.x(k)[o]], ub[lay.x(k)[o]] = -INF, INF

    def idx_of(name, vt):
        if vt == "phi":
            return [lay.phi()[pb.PHI_NAMES.index(name)]]
        if vt == "theta":
            return tf_idx if name == "t_f" else [lay.theta_index(name)]
        o, n = m.off[(vt, name)]
        out = []
        for k in range(lay.n_k + (1 if vt == "x" else 0)):
            if vt == "u":
                out.extend(lay.u(k)[o - m.w_u0:o - m.w_u0 + n])
            else:
                out.extend(lay.x(k)[o:o + n])
        return out

    counter: dict = {}
    steps = []
    for step, part, ups in updates:
        for name, vt in ups:
            counter[name] = counter.get(name, 0) + 1
            which = "lb" if counter[name] % 2 == 1 else "ub"
            for i in idx_of(name, vt):
                if which == "lb":
                    lb[i] = 0.0 if vt == "phi" else lb0[i]
                else:
                    ub[i] = 0.0 if vt == "phi" else ub0[i]
        steps.append(Step(f"{step}{part}", f"{step}{part}", lb.copy(), ub.copy()))
    return steps


def outputs(mc: du.MultiConstants, lay: du.MultiLayout, V: np.ndarray) -> dict:
    """Average power [W] over the phase-fixed period, the period [s] and the two t_f."""
    m, s = mc.model, mc.scaling
    w = np.asarray(pb.collocation(lay.d)[3], dtype=float)
    o_l = m.off[("x", "l_t")][0]
    o_dl = m.off[("x", "dl_t")][0]
    o_lam = m.off[("z", "lambda10")][0]
    energy = 0.0
    for k in range(lay.n_k):
        tf = float(V[lay.tf_index(k)])
        for j in range(lay.d):
            cx = V[lay.coll_x(k, j)]
            lam = float(V[lay.coll_z(k, j)[0]]) * s[o_lam]
            energy += tf / lay.n_k * w[j] * lam * cx[o_l] * s[o_l] * cx[o_dl] * s[o_dl]
    if lay.single_reelout:
        t0, t1 = float(V[lay.theta_index("t_f0")]), float(V[lay.theta_index("t_f1")])
        T = t0 * lay.nk_reelout / lay.n_k + t1 * (lay.n_k - lay.nk_reelout) / lay.n_k
    else:
        t0 = t1 = T = float(V[lay.theta_index("t_f")])
    return {"avg_power_W": energy / T, "period_s": T, "energy_J": energy, "t_f": [t0, t1]}


def make_evaluator(mc: du.MultiConstants, device="cuda", batch: int = 1, hessian: str = "exact"):
    """Dual-kite evaluator of `batch` instances.  ``hessian='exact'`` (IPOPT's default,
    opts/default.py:323): nlp_hess_l from the hyper-dual kernel (awedual.hip, dual_hess_kernel);
    ``'fd'``: coloured central differences of the exact HIP gradient (fd_hessian.py)."""
    from .dual_evaluator import DualEvaluator
    ev = DualEvaluator(mc, batch=batch)
    if hessian == "exact":
        return ev
    if hessian != "fd":
        raise ValueError(f"unknown Hessian mode {hessian!r}")
    from .fd_hessian import FdHessian
    return FdHessian(ev, lambda B: DualEvaluator(mc, batch=B), ev.layout, device=device)


def optimize(mc: du.MultiConstants, ev, opts=None, device="cuda", v_init=None, verbose=False,
             u_ref: float | None = None, final_step: str | None = None):
    """The homotopy of optimization.py:273-382 on the GPU interior-point solver; returns
    (V_opt, per-step summaries, outputs, last result)."""
    from .ipm import solve
    from .trajectory import hippo_options
    lay = du.layout_for(mc)
    v0 = du.initial_guess(mc, lay) if v_init is None else v_init
    steps = schedule(mc, lay, v0)
    lbg, ubg = lay.g_bounds()
    x, lam, zl, zu = v0.copy(), None, None, None
    summary = []
    res = None
    for st in steps:
        P = du.pack_p(lay, mc, v0, step=st.cost_step, u_ref=u_ref)
        t0 = time.perf_counter()
        res = solve(ev, P, x, st.lbx, st.ubx, lbg, ubg, lam0=lam, zl0=zl, zu0=zu,
                    opts=hippo_options(st.label, opts), device=device)
        out = outputs(mc, lay, res.x)
        rec = dict(step=st.label, status=res.status, iterations=res.iterations, f=res.f, kkt_error=res.kkt_error,
                   constr_viol=res.constr_viol, seconds=time.perf_counter() - t0, kkt_solves=res.kkt_solves,
                   kkt_dense=res.kkt_dense, timing={k: round(v, 3) for k, v in res.timing.items()}, **out)
        summary.append(rec)
        if verbose:
            print(rec, flush=True)
        x, lam, zl, zu = res.x, res.lam_g, res.zl, res.zu
        if final_step is not None and st.label == final_step:
            break
    return x, summary, outputs(mc, lay, x), res


def optimize_batch(mc: du.MultiConstants, ev, u_refs, opts=None, device="cuda", v_init=None, verbose=False):
    """The homotopy for B = len(u_refs) wind speeds at once (ev.batch == B), one batched
    interior-point solve per step (ipm.solve_batch); returns (V [B, n_v], per-step summaries,
    outputs per instance, results)."""
    from .ipm import solve_batch
    from .trajectory import hippo_options
    lay = du.layout_for(mc)
    v0 = du.initial_guess(mc, lay) if v_init is None else v_init
    B = len(u_refs)
    steps = schedule(mc, lay, v0)
    lbg, ubg = lay.g_bounds()
    x = np.tile(v0, (B, 1))
    lam = zl = zu = None
    summary = []
    res = None
    for st in steps:
        P = np.stack([du.pack_p(lay, mc, v0, step=st.cost_step, u_ref=u) for u in u_refs])
        t0 = time.perf_counter()
        res = solve_batch(ev, P, x, st.lbx, st.ubx, lbg, ubg, lam0=lam, zl0=zl, zu0=zu,
                          opts=hippo_options(st.label, opts), device=device)
        rec = dict(step=st.label, status=[r.status for r in res], iterations=[r.iterations for r in res],
                   f=[r.f for r in res], seconds=time.perf_counter() - t0,
                   timing={k: round(v, 3) for k, v in res[0].timing.items()})
        summary.append(rec)
        if verbose:
            print(rec, flush=True)
        x = np.stack([r.x for r in res])
        lam = np.stack([r.lam_g for r in res])
        zl = np.stack([r.zl for r in res])
        zu = np.stack([r.zu for r in res])
    return x, summary, [outputs(mc, lay, x[b]) for b in range(B)], res
