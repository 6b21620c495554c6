"""Host-side description of the 3-DOF AP2 tracking-MPC NLP (config 5).

The reference builds this NLP in ``awebox/pmpc.py`` from the trial of
``examples/mpc_closed_loop.py``: a single AP2 kite with ``kite_dof = 3`` (roll control through the
``coeff = [CL, psi]`` states, ``three_dof_kite.py``), default options otherwise (log wind with
``u_ref = 5``, ``z_ref = 10``; tether control ``dddl_t``; 'multi' tether drag with 5 elements),
transcribed with radau collocation (``mpc.d = 4``, zoh controls) over a horizon of ``N`` sampling
intervals of ``ts`` seconds (``t_f = N ts`` fixed, pmpc.py:75-82).

This module restates, without CasADi, everything that is *constant* for the evaluator:

* the node-variable layout (``system.py:42-230``: x[11] xdot[11] u[6] z[1] theta[2]);
* the option-derived scaling (``opts/model_funcs.py:227-284, 287-400, 890-1064, 1151-1462``;
  ``mdl/dynamics.py:824-921``) and the fixed parameters theta0 the model reads;
* the MPC NLP layout: ``V`` (``ocp/var_struct.py:39-115``), ``g`` = [initial conditions (11,
  ``ocp/operation.py:303-326``)] + per interval [shooting 12, path 2, collocation d x 12,
  continuity 11] (``ocp/constraints.py:48-145, 210-373``), and the MPC parameter vector
  ``p = [x0, ref (V-shaped), u_ref, Q, R, P]`` (``pmpc.py:166-186``);
* a synthetic periodic reference (the standard circular orbit of
  ``opti/initialization_dir/standard_scenario.py``) and the batch of SURVEY 8(d) config 5.

Row order of the initial conditions: the reference iterates ``set(x_struct.keys())``
(operation.py:311-317), whose order depends on Python's per-process string hashing; any fixed
order is therefore one of the reference's possible orders.  We use the x struct order.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from .collocation import coefficients

# ---------------------------------------------------------------------------------------
# model variables (system.py:42-230; kite_dof 3 -> coeff/dcoeff, tether control 'dddl_t' ->
# ddl_t is a state and dddl_t a control; integral_outputs -> no energy state)
# ---------------------------------------------------------------------------------------
X_VARS = [("q10", 3), ("dq10", 3), ("coeff10", 2), ("l_t", 1), ("dl_t", 1), ("ddl_t", 1)]
XDOT_VARS = [("d" + n, s) for n, s in X_VARS]          # dq10 ddq10 dcoeff10 dl_t ddl_t dddl_t
U_VARS = [("f_fict10", 3), ("dcoeff10", 2), ("dddl_t", 1)]
Z_VARS = [("lambda10", 1)]
THETA_VARS = [("diam_t", 1), ("t_f", 1)]
VAR_TYPES = [("x", X_VARS), ("xdot", XDOT_VARS), ("u", U_VARS), ("z", Z_VARS), ("theta", THETA_VARS)]

NX, NU, NZ, NTH = 11, 6, 1, 2
NW = 2 * NX + NU + NZ + NTH            # 31 node variables
NPHI, NXI = 7, 2
N_EQ, N_INEQ = 12, 2

W_OFF = {}
_p = 0
for _vt, _ents in VAR_TYPES:
    for _n, _s in _ents:
        W_OFF[(_vt, _n)] = (_p, _s)
        _p += _s
assert _p == NW

# model rows: dynamics_translation (3), dynamics_constraint (1), trivial kinematics in the sorted
# order of the xdot names that also live in x or u (lagr_dyn.py:141-169): dcoeff10 (2), dddl_t,
# ddl_t, dl_t, dq10 (3); inequalities: tether_stress10, acceleration10 (dynamics.py:106-129)
EQ_NAMES = (["dynamics_translation"] * 3 + ["dynamics_constraint"] + ["trivial_dcoeff10"] * 2
            + ["trivial_dddl_t", "trivial_ddl_t", "trivial_dl_t"] + ["trivial_dq10"] * 3)
INEQ_NAMES = ["tether_stress10", "acceleration10"]

# ---------------------------------------------------------------------------------------
# model constants vector; mirrors K3_C_* in include/awempc.h
# ---------------------------------------------------------------------------------------
CONST_NAMES = (["n_k", "d", "g", "t_ref", "rho_ref", "gamma_air", "r_air", "z_ref", "z0_air", "kappa",
                "rho_tether", "cd_tether", "stress_max", "m_k", "s_ref", "ar", "cd0", "acc_max",
                "scaling_length", "scaling_diam", "g_scaling", "q_scaling_mean", "lambda_scaling",
                "n_elements"] + [f"scaling{i}" for i in range(NW)])
NCONST = len(CONST_NAMES)
CONST_IDX = {n: i for i, n in enumerate(CONST_NAMES)}


@dataclass
class Kite3Config:
    """Options of examples/mpc_closed_loop.py (+ awebox defaults, opts/default.py)."""
    n_k: int = 20                 # MPC horizon N (SURVEY config 5)
    d: int = 4                    # mpc.d
    ts: float = 0.1               # sampling time (mpc_closed_loop.py:59)
    u_ref: float = 5.0            # user_options.wind.u_ref
    z_ref: float = 10.0           # params.wind.z_ref
    z0_air: float = 0.1           # params.wind.log_wind.z0_air
    groundspeed: float = 20.0     # solver.initialization.*
    inclination_deg: float = 40.0
    cone_deg: float = 25.0
    l_t_init: float = 500.0
    windings: int = 1
    diam_t_init: float = 5e-3     # solver.initialization.theta.diam_t (scaling)
    diam_t: float = 5e-3          # the fixed tether diameter of the MPC trial (pmpc.py:77-80)
    tether_rho: float = 970.0
    tether_cd: float = 1.0
    kappa: float = 10.0
    max_stress: float = 3.6e9
    stress_safety_factor: float = 1.5
    tether_force_limits: tuple = (1e0, 2e3)
    acc_max: float = 12.0
    g_scaling: float = 9.81
    ddl_t_bounds: tuple = (-100.0, 100.0)
    dddl_t_bounds: tuple = (-100.0, 100.0)
    coeff_max: tuple = (2.0, 80.0 * math.pi / 180.0)
    coeff_min: tuple = (0.0, -80.0 * math.pi / 180.0)
    dcoeff_max: tuple = (5.0, 80.0 * math.pi / 180.0)
    n_elements: int = 5
    # ampyx_data.py:46-237
    m_k: float = 36.8
    b_ref: float = 5.5
    s_ref: float = 3.0
    cx0: float = -0.0293
    alpha_max_deg: float = 9.0
    # reference orbit of the synthetic tracking problem (CL, roll angle)
    coeff_ref: tuple = (1.0, 0.0)


@dataclass
class Kite3Constants:
    cfg: Kite3Config
    scaling: np.ndarray            # [31]
    consts: np.ndarray             # [NCONST]
    details: dict = field(default_factory=dict)


def log_wind(u_ref, z_ref, z0, zz):
    """wind.get_speed 'log_wind' with smooth_abs(zz, eps=1) (wind.py:184-208)."""
    z_cropped = math.sqrt(zz ** 2 + 1.0)
    return u_ref * math.log10(z_cropped / z0) / math.log10(z_ref / z0)


def _synthesize(estimates):
    # vector_operations.synthesize_estimate_from_a_list_of_positive_scalar_floats
    return float(np.exp(np.sum(np.log(estimates)) / len(estimates)))


def build_constants(cfg: Kite3Config | None = None) -> Kite3Constants:
    cfg = cfg or Kite3Config()
    g = cfg.g_scaling
    rho_ref = 1.225
    ar = cfg.b_ref / (cfg.s_ref / cfg.b_ref)                     # ampyx_data.py:57
    elevation = cfg.inclination_deg * math.pi / 180.
    altitude = cfg.l_t_init * math.sin(elevation)                # estimate_altitude
    u_alt = log_wind(cfg.u_ref, cfg.z_ref, cfg.z0_air, altitude)
    flight_radius = cfg.groundspeed ** 2 / (cfg.acc_max * g)     # 'centripetal' (model_funcs.py:1151-1180)

    # force scaling 'synthesized' (model_funcs.py:994-1043); 3-DOF CL estimate = coeff max
    # (estimate_CL, :1297-1328)
    CL_est = cfg.coeff_max[0]
    u_app = (u_alt ** 2 + cfg.groundspeed ** 2) ** 0.5
    aero_force = CL_est * (0.5 * rho_ref * u_app ** 2) * cfg.s_ref
    tether_mass = math.pi * (cfg.diam_t_init / 2.) ** 2 * cfg.l_t_init * cfg.tether_rho
    total_mass = cfg.m_k + tether_mass
    tension = (cfg.tether_force_limits[0] + cfg.tether_force_limits[1]) / 2.   # 'average_force'
    tension_per_length = tension / cfg.l_t_init
    estimates = [cfg.m_k * cfg.acc_max * g, tension_per_length * cfg.l_t_init, total_mass * g / 1.0,
                 cfg.m_k * cfg.groundspeed ** 2 / flight_radius, aero_force]
    f_scaling = _synthesize(estimates)
    lambda_scaling = 1.0 * tension_per_length                    # lambda_factor = 1

    sx = {"q10": [flight_radius] * 3, "dq10": [cfg.groundspeed] * 3, "coeff10": list(cfg.coeff_max),
          "l_t": [cfg.l_t_init], "dl_t": [u_alt / 3.], "ddl_t": [max(cfg.ddl_t_bounds) / 2.]}
    su = {"f_fict10": [f_scaling] * 3, "dcoeff10": list(cfg.dcoeff_max),
          "dddl_t": [max(cfg.dddl_t_bounds) / 2.]}
    sz = {"lambda10": [lambda_scaling]}
    sth = {"diam_t": [cfg.diam_t_init], "t_f": [1.0]}
    # xdot scaling = scaling of the integral variable in x (else u) (dynamics.py:886-903)
    sxd = {}
    for n, _ in XDOT_VARS:
        base = n[1:]
        sxd[n] = sx[base] if base in sx else su[base]
    scaling = np.concatenate([np.concatenate([np.array(dct[n], dtype=np.float64) for n, _ in ents])
                              for dct, ents in ((sx, X_VARS), (sxd, XDOT_VARS), (su, U_VARS),
                                                (sz, Z_VARS), (sth, THETA_VARS))])
    assert scaling.shape == (NW,)

    c = np.zeros(NCONST)
    vals = dict(n_k=cfg.n_k, d=cfg.d, g=9.81, t_ref=288.15, rho_ref=rho_ref, gamma_air=6.5e-3,
                r_air=287.053, z_ref=cfg.z_ref, z0_air=cfg.z0_air, kappa=cfg.kappa,
                rho_tether=cfg.tether_rho, cd_tether=cfg.tether_cd,
                stress_max=cfg.max_stress / cfg.stress_safety_factor, m_k=cfg.m_k, s_ref=cfg.s_ref, ar=ar,
                cd0=abs(cfg.cx0), acc_max=cfg.acc_max * g, scaling_length=cfg.l_t_init,
                scaling_diam=cfg.diam_t_init, g_scaling=g, q_scaling_mean=float(np.mean(sx["q10"])),
                lambda_scaling=lambda_scaling, n_elements=cfg.n_elements)
    for k, v in vals.items():
        c[CONST_IDX[k]] = v
    c[CONST_IDX["scaling0"]:CONST_IDX["scaling0"] + NW] = scaling
    details = dict(altitude=altitude, u_alt=u_alt, flight_radius=flight_radius, f_scaling=f_scaling,
                   lambda_scaling=lambda_scaling, estimates=estimates, aero_force=aero_force)
    return Kite3Constants(cfg=cfg, scaling=scaling, consts=c, details=details)


# ---------------------------------------------------------------------------------------
# MPC NLP layout
# ---------------------------------------------------------------------------------------
class MpcLayout:
    """Index maps of V, g and p of the tracking-MPC NLP (radau, zoh, trajectory type 'mpc')."""

    def __init__(self, n_k: int = 20, d: int = 4):
        self.n_k, self.d = n_k, d
        self.nx = NX                                                       # states per shooting node
        self.n_coll_var = NX + NZ
        self.interval_stride = NX + NU + NX + NZ + d * self.n_coll_var      # 77 for d=4
        self.v_theta, self.v_phi, self.v_xi = 0, NTH, NTH + NPHI
        self.v_intervals = NTH + NPHI + NXI                                # 11
        self.n_v = self.v_intervals + n_k * self.interval_stride + NX
        self.rows_per_interval = N_EQ + N_INEQ + d * N_EQ + NX            # 73
        self.g_initial = 0
        self.g_int0 = NX
        self.n_g = NX + n_k * self.rows_per_interval
        # p = [x0 (nx), ref (V), u_ref, Q (nx), R (nu), P (nx)]  (pmpc.py:166-186)
        self.p_x0 = 0
        self.p_ref = NX
        self.p_u_ref = NX + self.n_v
        self.p_Q = self.p_u_ref + 1
        self.p_R = self.p_Q + NX
        self.p_P = self.p_R + NU
        self.n_p = self.p_P + NX

    def x(self, k):
        b = self.v_intervals + k * self.interval_stride
        return np.arange(b, b + NX)

    def u(self, k):
        b = self.v_intervals + k * self.interval_stride + NX
        return np.arange(b, b + NU)

    def xdot(self, k):
        b = self.v_intervals + k * self.interval_stride + NX + NU
        return np.arange(b, b + NX)

    def z(self, k):
        b = self.v_intervals + k * self.interval_stride + 2 * NX + NU
        return np.arange(b, b + NZ)

    def coll_x(self, k, j):
        b = self.v_intervals + k * self.interval_stride + 2 * NX + NU + NZ + j * self.n_coll_var
        return np.arange(b, b + NX)

    def coll_z(self, k, j):
        b = self.v_intervals + k * self.interval_stride + 2 * NX + NU + NZ + j * self.n_coll_var + NX
        return np.arange(b, b + NZ)

    def theta(self):
        return np.arange(0, NTH)

    def phi(self):
        return np.arange(self.v_phi, self.v_phi + NPHI)

    def xi(self):
        return np.arange(self.v_xi, self.v_xi + NXI)

    def g_init(self):
        return np.arange(0, NX)

    def g_shooting(self, k):
        b = NX + k * self.rows_per_interval
        return np.arange(b, b + N_EQ)

    def g_path(self, k):
        b = NX + k * self.rows_per_interval + N_EQ
        return np.arange(b, b + N_INEQ)

    def g_coll(self, k, j):
        b = NX + k * self.rows_per_interval + N_EQ + N_INEQ + j * N_EQ
        return np.arange(b, b + N_EQ)

    def g_continuity(self, k):
        b = NX + k * self.rows_per_interval + N_EQ + N_INEQ + self.d * N_EQ
        return np.arange(b, b + NX)

    def g_bounds(self):
        lb, ub = np.zeros(self.n_g), np.zeros(self.n_g)
        for k in range(self.n_k):
            lb[self.g_path(k)] = -np.inf
        ub[self.g_path(0)] = np.inf          # path constraints at k = 0 released (pmpc.py:128-134)
        return lb, ub


MPC_P_ENTRIES = ("x0", "ref", "u_ref", "Q", "R", "P")   # pmpc.py:166-186 (tracking cost), in order


def pack_p_from_reference(get, lay: MpcLayout) -> np.ndarray:
    """The MPC parameter vector in this library's flat layout from Pmpc's parameter struct, read
    entry by entry by name: ``p = struct_symMX([x0 (nx), ref (the MPC trial's V struct), u_ref,
    Q (nx), R (nu), P (nx)])`` (pmpc.py:166-186, cost_type 'tracking').  ``get((name,))`` returns
    the entry; with a casadi.tools struct ``p_num``: ``get = lambda path: np.asarray(p_num[path])``.
    A missing name raises KeyError; a wrong size raises ValueError."""
    sizes = {"x0": (lay.p_x0, NX), "ref": (lay.p_ref, lay.n_v), "u_ref": (lay.p_u_ref, 1),
             "Q": (lay.p_Q, NX), "R": (lay.p_R, NU), "P": (lay.p_P, NX)}
    p = np.zeros(lay.n_p)
    for name in MPC_P_ENTRIES:
        off, size = sizes[name]
        v = np.asarray(get((name,)), dtype=np.float64).ravel()
        if v.size != size:
            raise ValueError(f"MPC parameter {name} has {v.size} values, expected {size}")
        p[off:off + size] = v
    return p


def p_fun(p: np.ndarray, lay: MpcLayout) -> dict:
    """Restatement of ``Pmpc.__create_P_fun`` (pmpc.py:641-689): the parameter P of the MPC trial's
    NLP that the MPC constraints ``g = nlp.g_fun(V, P_fun(p))`` (:190) are evaluated with, as
    {entry: value} by the names the reference's loop fills:

    * ``('p', 'ref')``: the trial's V shape, zero except x[0] = p.x0 and x[N] = p.ref's x[N]
      (:660-671) -- x[0] feeds the initial-condition rows (operation.py:303-326);
    * ``('theta0', 'wind', 'u_ref')``: p.u_ref (:675-676); every other theta0 entry is the model
      parameter of p_fix_num (:677-682) -- constant here (``Kite3Constants.consts``);
    * everything else (``('p', 'weights')``, ``('cost', *)``): 0 (:684-685).

    The MPC kernel reads x0 and u_ref from p directly, which is this map composed with g_fun."""
    p = np.asarray(p, dtype=np.float64).ravel()
    ref = np.zeros(lay.n_v)
    ref[lay.x(0)] = p[lay.p_x0:lay.p_x0 + NX]
    ref[lay.x(lay.n_k)] = p[lay.p_ref + lay.x(lay.n_k)]
    return {("p", "ref"): ref, ("p", "weights"): np.zeros(NW), ("theta0", "wind", "u_ref"): p[lay.p_u_ref:lay.p_u_ref + 1]}


def fict_columns(lay: MpcLayout) -> np.ndarray:
    """V indices of the fictitious forces f_fict10 of every interval's zoh control."""
    o = W_OFF[("u", "f_fict10")][0] - NX - NX                      # offset inside u
    return np.concatenate([lay.u(k)[o:o + 3] for k in range(lay.n_k)])


def variable_bounds(consts: Kite3Constants, lay: MpcLayout):
    """Scaled (lbx, ubx) of the MPC NLP.

    ``var_bounds.get_scaled_variable_bounds`` (ocp/var_bounds.py:42-103) for a non-periodic
    ('mpc') trajectory with zoh controls: the model's system bounds (opts/default.py:190-210,
    model_funcs.py:897-914 for the tether control) on the shooting states x[k] of every node
    k = 0..N, on u[k] and z[k]; collocation variables and xdot unbounded; then the MPC
    overrides of pmpc.py: x[0] released (:120-121, the initial-condition rows fix it), phi <= 0
    and xi = 0 (:177-179), f_fict fixed to 0 (:181-190), theta fixed to (diam_t, t_f = N ts)
    (user_options.trajectory.fixed_params, :75-82).  phi's lower bound 0 comes from
    model.parameter_bounds (the homotopy parameters' [0, 1]).  Names carry their node identifier
    in the model (q10, coeff10, lambda10); define_bounds (mdl/system.py:353-383) looks them up
    without it."""
    cfg, s = consts.cfg, consts.scaling
    inf = np.inf
    lb, ub = np.full(lay.n_v, -inf), np.full(lay.n_v, inf)
    x_lb = np.concatenate([[-inf, -inf, 10.0], [-inf] * 3, cfg.coeff_min, [1e-2, -30.0, cfg.ddl_t_bounds[0]]])
    x_ub = np.concatenate([[inf] * 3, [inf] * 3, cfg.coeff_max, [1e3, 30.0, cfg.ddl_t_bounds[1]]])
    dcoeff_max = np.asarray(cfg.dcoeff_max)
    u_lb = np.concatenate([[-inf] * 3, -dcoeff_max, [cfg.dddl_t_bounds[0]]])
    u_ub = np.concatenate([[inf] * 3, dcoeff_max, [cfg.dddl_t_bounds[1]]])
    sx, su, sz = s[:NX], s[2 * NX:2 * NX + NU], s[2 * NX + NU:2 * NX + NU + NZ]
    for k in range(1, lay.n_k + 1):
        lb[lay.x(k)], ub[lay.x(k)] = x_lb / sx, x_ub / sx
    for k in range(lay.n_k):
        lb[lay.u(k)], ub[lay.u(k)] = u_lb / su, u_ub / su
        lb[lay.z(k)], ub[lay.z(k)] = 0.0, inf
    fict = fict_columns(lay)
    lb[fict] = ub[fict] = 0.0
    theta = np.array([cfg.diam_t, lay.n_k * cfg.ts]) / s[2 * NX + NU + NZ:]
    lb[lay.theta()] = ub[lay.theta()] = theta
    lb[lay.phi()] = ub[lay.phi()] = 0.0
    lb[lay.xi()] = ub[lay.xi()] = 0.0
    return lb, ub


# ---------------------------------------------------------------------------------------
# synthetic periodic reference: the standard circular orbit (standard_scenario.py:72-149,
# tools.py:39-379) for the 3-DOF kite, with a constant (CL, psi)
# ---------------------------------------------------------------------------------------
class CircularOrbit:
    def __init__(self, cfg: Kite3Config):
        self.cfg = cfg
        self.radius = cfg.l_t_init * math.sin(cfg.cone_deg * math.pi / 180.0)
        self.groundspeed = cfg.groundspeed
        self.period = cfg.windings * 2. * math.pi * self.radius / self.groundspeed
        self.height = (cfg.l_t_init ** 2 - self.radius ** 2) ** 0.5
        self.angular_speed = self.groundspeed / self.radius

    def state(self, t: float) -> dict:
        cfg = self.cfg
        incl = cfg.inclination_deg * math.pi / 180.
        n_hat = np.array([math.cos(incl), 0.0, math.sin(incl)])
        xhat = np.array([1.0, 0.0, 0.0])
        y_rot = np.cross(n_hat, xhat)
        y_rot /= np.linalg.norm(y_rot)
        z_rot = np.cross(n_hat, y_rot)
        z_rot /= np.linalg.norm(z_rot)
        psi = (self.angular_speed * t) % (2. * math.pi)
        outward = z_rot * math.cos(psi) - y_rot * math.sin(psi)
        e_tan = np.cross(n_hat, outward)
        e_tan /= np.linalg.norm(e_tan)
        q = outward * self.radius + n_hat * self.height
        dq = self.groundspeed * e_tan
        ddq = self.groundspeed ** 2 / self.radius * (-outward)
        return {"q10": q, "dq10": dq, "ddq10": ddq, "coeff10": np.array(cfg.coeff_ref, dtype=np.float64),
                "l_t": np.array([cfg.l_t_init]), "dl_t": np.array([0.0]), "ddl_t": np.array([0.0])}


def x_vector(ret: dict) -> np.ndarray:
    out = np.zeros(NX)
    o = 0
    for n, s in X_VARS:
        out[o:o + s] = ret[n]
        o += s
    return out


def reference_window(consts: Kite3Constants, lay: MpcLayout, t0: float, orbit: CircularOrbit | None = None):
    """Scaled V-shaped reference of the horizon starting at t0 (pmpc.get_reference, :543-604):
    x at the shooting and collocation nodes from the periodic orbit, u = 0 (fictitious forces and a
    constant orbit's dcoeff / dddl_t), xdot = 0, shooting z = 0, collocation z = 1 (scaled),
    theta = (diam_t, t_f = N ts), phi = xi = 0."""
    cfg = consts.cfg
    orbit = orbit or CircularOrbit(cfg)
    s = consts.scaling
    sx = s[:NX]
    tau, _, _, _ = coefficients(lay.d, "radau")
    V = np.zeros(lay.n_v)
    V[lay.theta()] = np.array([cfg.diam_t, lay.n_k * cfg.ts]) / s[2 * NX + NU + NZ:]
    for k in range(lay.n_k + 1):
        V[lay.x(k)] = x_vector(orbit.state((t0 + k * cfg.ts) % orbit.period)) / sx
        if k < lay.n_k:
            for j in range(lay.d):
                t = t0 + (k + tau[j + 1]) * cfg.ts
                V[lay.coll_x(k, j)] = x_vector(orbit.state(t % orbit.period)) / sx
                V[lay.coll_z(k, j)] = 1.0
    return V


def pack_p(lay: MpcLayout, consts: Kite3Constants, x0_scaled, ref, u_ref=None, Q=None, R=None, P=None):
    """The MPC parameter vector (pmpc.py:166-186 tracking, defaults of __generate_objective
    :300-316: unit Q, R, P)."""
    p = np.zeros(lay.n_p)
    p[lay.p_x0:lay.p_x0 + NX] = x0_scaled
    p[lay.p_ref:lay.p_ref + lay.n_v] = ref
    p[lay.p_u_ref] = consts.cfg.u_ref if u_ref is None else u_ref
    p[lay.p_Q:lay.p_Q + NX] = 1.0 if Q is None else Q
    p[lay.p_R:lay.p_R + NU] = 1.0 if R is None else R
    p[lay.p_P:lay.p_P + NX] = 1.0 if P is None else P
    return p


def batch_instance(consts: Kite3Constants, lay: MpcLayout, i: int, batch: int, sigma: float = 0.01,
                   seed: int = 99, orbit: CircularOrbit | None = None):
    """instance i of `batch` starts at phase t_i = i T / batch; x0 = the
    reference state there + 0.01 N(0,1) (scaled), V = the reference window + 0.01 N(0,1) on the
    entries the MPC bounds leave free (theta, phi, xi are fixed)."""
    orbit = orbit or CircularOrbit(consts.cfg)
    t0 = i * orbit.period / batch
    ref = reference_window(consts, lay, t0, orbit)
    rng = np.random.default_rng(seed + i)
    x0 = ref[lay.x(0)] + sigma * rng.standard_normal(NX)
    V = ref + sigma * rng.standard_normal(lay.n_v)
    fixed = np.zeros(lay.n_v, dtype=bool)
    fixed[:lay.v_intervals] = True
    V[fixed] = ref[fixed]
    return V, pack_p(lay, consts, x0, ref)
