"""Variable bounds, the homotopy schedule and trajectory outputs of the AP2 power-cycle problem.

Host-side data formats either side of the evaluator:

* ``variable_bounds``: the model's scaled variable bounds on V (``ocp/var_bounds.py:42-103``) for
  the AP2 options (``ampyx_ap2_settings.py:17-60``, ``opts/default.py:190-210``,
  ``opts/model_funcs.py:300-310,418``): x bounds on the shooting states x[0..n_k-1] only (zoh,
  periodic), z and u bounds on the interval variables, theta bounds, the 'simple' lift-mode phase
  fix dl_t(x[0]) = 0 (``var_bounds.py:204-209``).
* ``schedule``: the homotopy of a power cycle without induction -- initial, fictitious (2 parts),
  power (2 parts), final (``opti/scheduling.py:37-104``) -- each step with the cost vector
  (``problem.COST_UPDATES``) and the bounds after ``set_initial_bounds``
  (``preparation.py:150-227``) and the step's ``update_bounds`` (``scheduling.py:155-230,
  330-398``).  Homotopy parameters use the 'penalty' method (``default.py:339-341``): a free
  phi in [0, 1] with a linear cost, fixed to 0 by the step's final bound update.
* ``outputs``: average power and period (``dynamics.py:318-330``, ``collocation.py:272-316``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import problem as pb

INF = math.inf


def _model_bounds_si(cfg: pb.Ap2Config) -> dict:
    """(var_type, name) -> (lb, ub) SI arrays for every bounded model variable (system.define_bounds)."""
    om = 50.0 * math.pi / 180.0
    return {
        ("x", "q10"): (np.array([-INF, -INF, 100.0]), np.array([INF, INF, INF])),
        ("x", "omega10"): (np.full(3, -om), np.full(3, om)),
        ("x", "delta10"): (-np.asarray(cfg.delta_max), np.asarray(cfg.delta_max)),
        ("x", "l_t"): (np.array([10.0]), np.array([700.0])),
        ("x", "dl_t"): (np.array([-15.0]), np.array([20.0])),
        ("u", "ddelta10"): (-np.asarray(cfg.ddelta_max), np.asarray(cfg.ddelta_max)),
        ("u", "ddl_t"): (np.array([cfg.ddl_t_bounds[0]]), np.array([cfg.ddl_t_bounds[1]])),
        ("z", "lambda10"): (np.array([0.0]), np.array([INF])),
        ("theta", "diam_t"): (np.array([cfg.diam_t_fixed]), np.array([cfg.diam_t_fixed])),
        ("theta", "t_f"): (np.array([20.0]), np.array([70.0])),
    }


def _node_offset(vt: str, name: str) -> tuple[int, int]:
    return pb.W_OFF[(vt, name)]


def variable_bounds(consts: pb.Ap2Constants, lay: pb.NlpLayout):
    """Model bounds nlp.V_bounds (scaled) as (lbx, ubx); phi and xi at their schedule-free values."""
    cfg = consts.cfg
    s = consts.scaling
    lb = np.full(lay.n_v, -INF)
    ub = np.full(lay.n_v, INF)
    for (vt, name), (l_si, u_si) in _model_bounds_si(cfg).items():
        o, n = _node_offset(vt, name)
        sc = s[o:o + n]
        ls, us = l_si / sc, u_si / sc
        if vt == "x":
            for k in range(lay.n_k):                      # zoh + periodic: x[0..n_k-1] only
                idx = lay.x(k)[o:o + n]
                lb[idx], ub[idx] = ls, us
        elif vt == "u":
            for k in range(lay.n_k):
                idx = lay.u(k)[o - pb.W_U0:o - pb.W_U0 + n]
                lb[idx], ub[idx] = ls, us
        elif vt == "z":
            for k in range(lay.n_k):
                idx = lay.z(k)
                lb[idx], ub[idx] = ls, us
        elif vt == "theta":
            idx = lay.theta()[o - pb.W_TH0:o - pb.W_TH0 + n]
            lb[idx], ub[idx] = ls, us
    # lift-mode 'simple' phase fix: dl_t at the first control node (var_bounds.py:204-209)
    o, _ = _node_offset("x", "dl_t")
    lb[lay.x(0)[o]] = ub[lay.x(0)[o]] = 0.0
    # xi: power cycles fix both at 0 (formulation.py:152-153)
    lb[lay.v_xi:lay.v_xi + 2] = ub[lay.v_xi:lay.v_xi + 2] = 0.0
    return lb, ub


@dataclass
class Step:
    label: str          # e.g. "fictitious0"
    cost_step: str      # key into consts.cost_steps
    lbx: np.ndarray
    ubx: np.ndarray


# bound updates per (step, part) of the power-cycle schedule (scheduling.py:155-230):
# (bound name, var_type) updated in order; each update moves the next schedule entry
# [1] lb -> final, [2] ub -> final
_BOUND_UPDATES = [("initial", 0, [("diam_t", "theta"), ("t_f", "theta")] * 2 + [("ddl_t", "u")] * 2),
                  ("fictitious", 0, [("gamma", "phi")]),
                  ("fictitious", 1, [("gamma", "phi"), ("f_fict10", "u"), ("f_fict10", "u"),
                                     ("m_fict10", "u"), ("m_fict10", "u")]),
                  ("power", 0, [("psi", "phi")]),
                  ("power", 1, [("psi", "phi")]),
                  ("final", 0, [])]


def schedule(consts: pb.Ap2Constants, lay: pb.NlpLayout, v_init: np.ndarray) -> list[Step]:
    """The homotopy steps with their cost vector and bounds."""
    lb0, ub0 = variable_bounds(consts, lay)
    lb, ub = lb0.copy(), ub0.copy()
    # set_initial_bounds: phi = 1 for the scheduled parameters, 0 for the rest
    updated = {n for _, _, ups in _BOUND_UPDATES for n, vt in ups if vt == "phi"}
    for i, name in enumerate(pb.PHI_NAMES):
        v = 1.0 if name in updated else 0.0
        lb[lay.phi()[i]] = ub[lay.phi()[i]] = v
    # theta fixed at the initial values (diam_t from the initialization options, t_f from V_init)
    it = lay.theta()
    lb[it[0]] = ub[it[0]] = v_init[it[0]]
    lb[it[1]] = ub[it[1]] = v_init[it[1]]
    # fictitious controls unbounded
    for name in ("f_fict10", "m_fict10"):
        o, n = _node_offset("u", name)
        for k in range(lay.n_k):
            idx = lay.u(k)[o - pb.W_U0:o - pb.W_U0 + n]
            lb[idx], ub[idx] = -INF, INF

    counter: dict[str, int] = {}
    steps = []

    def idx_of(name, vt):
        if vt == "phi":
            return [lay.phi()[pb.PHI_NAMES.index(name)]]
        if vt == "theta":
            return [it[0] if name == "diam_t" else it[1]]
        o, n = _node_offset(vt, name)
        out = []
        for k in range(lay.n_k):
            out.extend(lay.u(k)[o - pb.W_U0:o - pb.W_U0 + n])
        return out

    for step, part, ups in _BOUND_UPDATES:
        for name, vt in ups:
            counter[name] = counter.get(name, 0) + 1
            which = "lb" if counter[name] == 1 else "ub"
            ii = idx_of(name, vt)
            target = 0.0 if vt == "phi" else None          # update_final_bounds
            for i in ii:
                if which == "lb":
                    lb[i] = target if target is not None else lb0[i]
                else:
                    ub[i] = target if target is not None else ub0[i]
        steps.append(Step(f"{step}{part}", f"{step}{part}", lb.copy(), ub.copy()))
    return steps


def outputs(consts: pb.Ap2Constants, lay: pb.NlpLayout, V: np.ndarray) -> dict:
    """Average power [W] over the period and the period t_f [s] (integral output e of
    dynamics.py:318-330 integrated by collocation.py:272-316)."""
    s = consts.scaling
    w = np.asarray(pb.collocation(lay.d)[3], dtype=float)
    tf = V[lay.theta()[1]] * s[pb.W_TH0 + 1]
    o_l, _ = _node_offset("x", "l_t")
    o_dl, _ = _node_offset("x", "dl_t")
    o_lam, _ = _node_offset("z", "lambda10")
    energy = 0.0
    for k in range(lay.n_k):
        for j in range(lay.d):
            cx = V[lay.coll_x(k, j)]
            lam = V[lay.coll_z(k, j)][0] * s[o_lam]
            p = lam * cx[o_l] * s[o_l] * cx[o_dl] * s[o_dl]
            energy += tf / lay.n_k * w[j] * float(p)
    return {"avg_power_W": energy / tf, "period_s": float(tf), "energy_J": energy}


def power_integrand(consts: pb.Ap2Constants):
    """The power integral output's integrand p = lambda10 l_t dl_t [W] (dynamics.py:318-330) from
    scaled states x [B, 23] and algebraic variables z [B, 1] (torch tensors)."""
    s = consts.scaling
    o_l, _ = _node_offset("x", "l_t")
    o_dl, _ = _node_offset("x", "dl_t")
    o_lam, _ = _node_offset("z", "lambda10")
    c = float(s[o_lam] * s[o_l] * s[o_dl])

    def p(x, z):
        return c * z[:, 0] * x[:, o_l] * x[:, o_dl]
    return p


def interval_energy(consts: pb.Ap2Constants, lay: pb.NlpLayout, V: np.ndarray, k: int) -> float:
    """Energy [J] of interval k: the integral output's increment over the interval
    (collocation.py:272-316), the reference integrators' ``qf``."""
    s = consts.scaling
    w = np.asarray(pb.collocation(lay.d)[3], dtype=float)
    tf = V[lay.theta()[1]] * s[pb.W_TH0 + 1]
    o_l, _ = _node_offset("x", "l_t")
    o_dl, _ = _node_offset("x", "dl_t")
    o_lam, _ = _node_offset("z", "lambda10")
    e = 0.0
    for j in range(lay.d):
        cx = V[lay.coll_x(k, j)]
        e += tf / lay.n_k * w[j] * V[lay.coll_z(k, j)][0] * s[o_lam] * cx[o_l] * s[o_l] * cx[o_dl] * s[o_dl]
    return float(e)
