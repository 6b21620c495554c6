"""Standard circular-orbit initial guess for the AP2 single-kite power cycle.

Restates ``awebox/opti/initialization_dir/initialization.py:72-104`` and
``standard_scenario.py:72-149, 253-458`` + ``tools.py:39-379`` for architecture {1: 0}, kite_dof 6,
``kite_dcm='aero_validity'``, ``normal_vector_model='tether_parallel'``, clockwise rotation,
``psi0_rad=0``.  Produces the *scaled* decision vector V0 (``struct_op.si_to_scaled``) and the
synthetic batch members of SURVEY.md section 8(d).
"""
from __future__ import annotations

import math

import numpy as np

from . import problem as pb


def _normalize(v):
    return v / np.linalg.norm(v)


def _normed_cross(a, b):
    return _normalize(np.cross(a, b))


class _Precompute:
    def __init__(self, cfg: pb.Ap2Config):
        # standard_scenario.precompute_path_parameters with init_clipping (no clip triggers for AP2)
        self.hypotenuse = cfg.l_t_init
        self.radius = self.hypotenuse * math.sin(cfg.cone_deg * math.pi / 180.0)
        self.groundspeed = cfg.groundspeed
        for _ in range(3):
            self.winding_period = 2. * math.pi * self.radius / self.groundspeed
            self.groundspeed = 2. * math.pi * self.radius / self.winding_period
        self.time_final = cfg.windings * self.winding_period
        self.height = (self.hypotenuse ** 2. - self.radius ** 2.) ** 0.5
        self.angular_speed = self.groundspeed / self.radius


def guess_values_at_time(t: float, cfg: pb.Ap2Config, pre: _Precompute) -> dict:
    incl = cfg.inclination_deg * math.pi / 180.
    n_hat = np.array([math.cos(incl), 0.0, math.sin(incl)])       # tools.get_ehat_tether
    xhat = np.array([1.0, 0.0, 0.0])
    y_rot = _normed_cross(n_hat, xhat)                               # tools.get_rotor_reference_frame
    z_rot = _normed_cross(n_hat, y_rot)
    sign = 1.0                                                      # clockwise_rotation_about_xhat
    psi = (0.0 + pre.angular_speed * t) % (2. * math.pi)
    outward = z_rot * math.cos(psi) - sign * y_rot * math.sin(psi)
    e_radial = sign * outward
    e_tangential = _normed_cross(n_hat, e_radial)
    q = outward * pre.radius + n_hat * pre.height
    dq = pre.groundspeed * e_tangential
    ddq = pre.groundspeed ** 2 / pre.radius * (-outward)

    # tools.get_wind_velocity: wind at the fixed altitude l_t * ehat_tether[2]
    zz = cfg.l_t_init * n_hat[2]
    u_inf = cfg.u_ref * (math.sqrt(zz ** 2 + 1.) / cfg.z_ref) ** cfg.exp_ref * xhat
    u_app = u_inf - dq
    e_normal = _normalize(q)                                        # 'tether_parallel'
    e1 = _normalize(u_app)
    e2 = _normed_cross(e_normal, e1)
    e3 = _normed_cross(e1, e2)
    dcm = np.stack([e1, e2, e3], axis=1)
    omega = sign * pre.angular_speed * np.array([0., 0., 1.])
    ddcm = dcm @ np.array([[0., -omega[2], omega[1]], [omega[2], 0., -omega[0]], [-omega[1], omega[0], 0.]])
    return {"q10": q, "dq10": dq, "ddq10": ddq, "omega10": omega, "domega10": np.zeros(3),
            "r10": dcm.reshape(-1, order="F"), "dr10": ddcm.reshape(-1, order="F"),
            "delta10": np.zeros(3), "l_t": np.array([cfg.l_t_init]), "dl_t": np.array([0.0])}


def initial_guess(consts: pb.Ap2Constants, layout: pb.NlpLayout) -> np.ndarray:
    """Scaled V0 (initialization.get_initial_guess)."""
    cfg = consts.cfg
    pre = _Precompute(cfg)
    tf = pre.time_final
    tau, C, D, w = pb.collocation(layout.d)
    n_k, d = layout.n_k, layout.d
    s = consts.scaling
    sx = s[pb.W_X0:pb.W_X0 + pb.NX]
    x_off, _ = pb._offsets(pb.X_VARS)

    def x_vec(ret):
        out = np.zeros(pb.NX)
        for name, (o, sz) in x_off.items():
            out[o:o + sz] = ret[name]
        return out

    V = np.zeros(layout.n_v)
    # theta: diam_t = fixed value, t_f = tf_guess (scaled by 5e-3 and 1)
    V[layout.theta()] = np.array([cfg.diam_t_fixed, tf]) / s[pb.W_TH0:pb.W_TH0 + 2]
    V[layout.phi()] = 1.0
    V[layout.v_xi:layout.v_xi + 2] = 0.0
    for k in range(n_k + 1):
        V[layout.x(k)] = x_vec(guess_values_at_time(k * tf / n_k, cfg, pre)) / sx
        if k < n_k:
            V[layout.z(k)] = 1.0          # multipliers: V(1.) scaled -> s_lambda SI
            for j in range(d):
                t = (k + tau[j + 1]) * tf / n_k
                V[layout.coll_x(k, j)] = x_vec(guess_values_at_time(t, cfg, pre)) / sx
                V[layout.coll_z(k, j)] = 1.0
    # set_xdot: V.xdot[k] = polynomial derivative at tau_0 (initialization.py:239-245)
    h = 1.0 / n_k
    for k in range(n_k):
        X = np.stack([V[layout.x(k)]] + [V[layout.coll_x(k, j)] for j in range(d)])  # [d+1, 23]
        xp = C[:, 0] @ X
        V[layout.xdot(k)] = xp / h / tf
    return V


def batch_member(v0: np.ndarray, layout: pb.NlpLayout, b: int, sigma: float = 0.01,
                 seed_base: int = 20261015) -> np.ndarray:
    """V_b = V0 + 0.01 N(0,1) on all non-fixed entries, rng(20261015 + b)."""
    rng = np.random.default_rng(seed_base + b)
    v = v0.copy()
    noise = sigma * rng.standard_normal(v.shape)
    fixed = np.zeros(v.shape, dtype=bool)
    fixed[layout.theta()[0]] = True          # diam_t is fixed by bounds
    fixed[layout.v_xi:layout.v_xi + 2] = True
    v[~fixed] += noise[~fixed]
    return v
