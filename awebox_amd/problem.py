"""Host-side description of the Ampyx AP2 single-kite OCP (the north-star NLP).

This module restates, for the AP2 configuration only, the parts of the awebox build pipeline
that *produce constants* for the hot path:

* the model variable layout (``awebox/mdl/system.py:42-230``, order x, xdot, u, z, theta),
* the option-derived scaling vector (``awebox/opts/model_funcs.py:227-320, 993-1183``,
  ``awebox/mdl/dynamics.py:824-921``),
* the fixed parameter tree ``theta0`` (``awebox/opts/default.py``, ``ampyx_data.py``,
  ``ampyx_ap2_settings.py``) packed into a flat vector,
* the NLP decision vector ``V`` and parameter vector ``P``
  (``awebox/ocp/var_struct.py:39-97``, ``awebox/ocp/discretization.py:129-179``),
* the constraint vector ``g`` ordering (``awebox/ocp/constraints.py:48-145, 210-373``),
* the homotopy cost vector of one schedule step (``awebox/opti/scheduling.py``,
  ``awebox/opts/default.py:413-457``) and the regularisation weights
  (``awebox/opti/preparation.py:121-160``).

No CasADi: every index map is explicit.  ``casadi.tools`` tuple entries interleave their
repeated members, so ``V = [theta, phi, xi, (x[k], u[k], xdot[k], z[k], coll_var[k, 0..d-1])_k,
x[n_k]]`` with ``coll_var = {x, z}``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from .collocation import coefficients

# ---------------------------------------------------------------------------------------
# model variables (system.py:42-230 with kite_dof=6, surface_control=1, lift_mode,
# tether control 'ddl_t', integral_outputs=True, architecture {1: 0})
# ---------------------------------------------------------------------------------------
X_VARS = [("q10", 3), ("dq10", 3), ("omega10", 3), ("r10", 9), ("delta10", 3), ("l_t", 1), ("dl_t", 1)]
XDOT_VARS = [("d" + n, s) for n, s in X_VARS]
U_VARS = [("f_fict10", 3), ("m_fict10", 3), ("ddelta10", 3), ("ddl_t", 1)]
Z_VARS = [("lambda10", 1)]
THETA_VARS = [("diam_t", 1), ("t_f", 1)]
PHI_NAMES = ["gamma", "tau", "iota", "psi", "eta", "nu", "upsilon"]  # system.py:435-450
XI_NAMES = ["xi_0", "xi_f"]
COST_NAMES = ["tracking", "u_regularisation", "xdot_regularisation", "gamma", "iota", "psi", "tau",
              "eta", "nu", "upsilon", "fictitious", "power", "power_derivative", "t_f",
              "theta_regularisation", "nominal_landing", "compromised_battery", "transition",
              "beta", "P_max"]  # discretization.py:129-152

VAR_TYPES = [("x", X_VARS), ("xdot", XDOT_VARS), ("u", U_VARS), ("z", Z_VARS), ("theta", THETA_VARS)]


def _offsets(entries):
    out, pos = {}, 0
    for name, size in entries:
        out[name] = (pos, size)
        pos += size
    return out, pos


NX = sum(s for _, s in X_VARS)        # 23
NU = sum(s for _, s in U_VARS)        # 10
NZ = sum(s for _, s in Z_VARS)        # 1
NTH = sum(s for _, s in THETA_VARS)   # 2
NW = 2 * NX + NU + NZ + NTH           # 59 node variables
NPHI = len(PHI_NAMES)
NXI = len(XI_NAMES)
NCOST = len(COST_NAMES)
N_EQ = 24
N_INEQ = 9

# node-variable offsets inside the 59-vector
W_OFF = {}
_pos = 0
for _vt, _ents in VAR_TYPES:
    for _n, _s in _ents:
        W_OFF[(_vt, _n)] = (_pos, _s)
        _pos += _s
assert _pos == NW
W_X0, W_XDOT0, W_U0, W_Z0, W_TH0 = 0, NX, 2 * NX, 2 * NX + NU, 2 * NX + NU + NZ

EQ_NAMES = (["dynamics_translation"] * 3 + ["dynamics_constraint"] + ["rotation_dynamics1"] * 3
            + ["ref_frame_dynamics1"] * 9 + ["trivial_ddelta10"] * 3 + ["trivial_ddl_t"]
            + ["trivial_dl_t"] + ["trivial_dq10"] * 3)
INEQ_NAMES = ["tether_force_max10", "tether_force_min10", "airspeed_max10", "airspeed_min10",
              "alpha_ub1", "alpha_lb1", "beta_ub1", "beta_lb1", "rotation_max10"]

# ---------------------------------------------------------------------------------------
# theta0 packing (our own flat layout of the reference's nested params tree).  Mirrors
# include/awegpu.h AWE_TH_* — keep both in sync.
# ---------------------------------------------------------------------------------------
SD_COEFFS = ["CX", "CY", "CZ", "Cl", "Cm", "Cn"]
SD_INPUTS = ["0", "alpha", "beta", "p", "q", "r", "deltaa", "deltae", "deltar"]
SD_MAXLEN = 3

THETA0_ENTRIES = [
    ("atmosphere.g", 1), ("atmosphere.gamma", 1), ("atmosphere.r", 1), ("atmosphere.t_ref", 1),
    ("atmosphere.p_ref", 1), ("atmosphere.rho_ref", 1), ("atmosphere.gamma_air", 1),
    ("atmosphere.mu_ref", 1), ("atmosphere.c_sutherland", 1),
    ("wind.z_ref", 1), ("wind.log_wind.z0_air", 1), ("wind.power_wind.exp_ref", 1), ("wind.u_ref", 1),
    ("tether.kappa", 1), ("tether.rho", 1), ("tether.cd", 1),
    ("model_bounds.tether_force_limits", 2), ("model_bounds.airspeed_limits", 2),
    ("model_bounds.rot_angles", 3),
    ("kappa_r", 1),
    ("geometry.b_ref", 1), ("geometry.c_ref", 1), ("geometry.s_ref", 1), ("geometry.m_k", 1),
    ("geometry.j", 9),
    ("aero.moment_factor", 1),
    ("aero.stab_derivs", len(SD_COEFFS) * len(SD_INPUTS) * SD_MAXLEN),
]
THETA0_OFF, NTHETA0 = _offsets(THETA0_ENTRIES)

# AP2 stability derivatives (awebox/opts/kite_data/ampyx_data.py:121-223)
AP2_STAB_DERIVS = {
    "CX": {"0": [-0.0293], "alpha": [0.4784, 2.5549], "q": [-0.6029, 4.4124], "deltae": [-0.0106, 0.1115]},
    "CY": {"beta": [-0.1855, -0.0299, 0.0936], "p": [-0.1022, -0.0140, 0.0496], "r": [0.1694, 0.1368],
           "deltaa": [-0.0514, -0.0024, 0.0579], "deltar": [0.10325, 0.0268, -0.1036]},
    "CZ": {"0": [-0.5526], "alpha": [-5.0676, 5.7736], "q": [-7.5560, 0.1251, 6.1486],
           "deltae": [-0.315, -0.0013, 0.2923]},
    "Cl": {"beta": [-0.0630, -0.0003, 0.0312], "p": [-0.5632, -0.0247, 0.2813], "r": [0.1811, 0.6448],
           "deltaa": [-0.2489, -0.0087, 0.2383], "deltar": [0.00436, -0.0013]},
    "Cm": {"0": [-0.0307], "alpha": [-0.6027], "q": [-11.3022, -0.0026, 5.2885],
           "deltae": [-1.0427, -0.0061, 0.9974]},
    "Cn": {"beta": [0.0577, -0.0849], "p": [-0.0565, -0.9137], "r": [-0.0553, 0.0290, 0.0257],
           "deltaa": [0.01903, -0.1147], "deltar": [-0.0404, -0.0117, 0.04089]},
}

# solver weights (default.py:390-411); names not listed get weight 1.0 (preparation.py:130-139)
SOLVER_WEIGHTS = {"q": 1e-1, "dq": 1e-1, "ddq": 1e0, "l_t": 1e-3, "dl_t": 1e-3, "ddl_t": 2e4,
                  "dddl_t": 2e2, "l_s": 1e0, "r": 1e1, "omega": 1e-1, "domega": 5e7, "lambda": 1.,
                  "vortex": 1e-3, "actuator": 1e-3, "a": 1e-3, "delta": 1e-4, "ddelta": 1e2,
                  "dkappa": 1e1, "coeff": 1e-4, "P_max": 0.0, "diam_s": 1e0, "diam_t": 1e0}

# homotopy cost schedule (default.py:413-457); the power entry index 1 is written by
# model_funcs.build_lambda_e_power_scaling (model_funcs.py:1066)
COST_SCHEDULE = {
    "tracking": [1e-1, 1e-3], "u_regularisation": [1e-6], "xdot_regularisation": [1e-8],
    "theta_regularisation": [1e0],
    "gamma": [0., 1e2, 1e-3], "iota": [0., 1e2, 1e-3], "psi": [0., 1e2, 1e-3], "tau": [0., 1e3, 1e-3],
    "eta": [0., 1e3], "nu": [0., 1e3], "upsilon": [0., 1e3],
    "fictitious": [1e3, 1e3, 1e-3], "power": [0., None], "power_derivative": [0., 0.], "t_f": [0.],
    "nominal_landing": [0, 1e-2], "compromised_battery": [0, 1e1, 0], "transition": [0, 1e-1],
    "beta": [1e3], "P_max": [1],
}
# cost updates per (step, sub-step) for a power_cycle schedule (scheduling.py:105-147)
COST_UPDATES = [("initial", 0, None),
                ("fictitious", 0, ["gamma", "fictitious"]), ("fictitious", 1, ["gamma"]),
                ("power", 0, ["power", "psi", "power_derivative", "fictitious"]),
                ("power", 1, ["tracking", "psi"]),
                ("final", 0, [])]


def split_name(name: str) -> str:
    """struct_op.split_name_and_node_identifier (struct_operations.py:1119-1129)."""
    while name and name[-1].isdigit():
        name = name[:-1]
    return name


# ---------------------------------------------------------------------------------------
# option-derived constants
# ---------------------------------------------------------------------------------------
@dataclass
class Ap2Config:
    """User options of examples/ampyx_ap2_trajectory.py + ampyx_ap2_settings.py."""
    n_k: int = 40
    d: int = 4
    u_ref: float = 10.0
    z_ref: float = 100.0
    exp_ref: float = 0.15
    groundspeed: float = 15.0
    inclination_deg: float = 45.0
    cone_deg: float = 15.0
    l_t_init: float = 200.0
    windings: int = 1
    tether_rho: float = 0.0046 * 4.0 / (math.pi * 0.002 ** 2)
    tether_cd: float = 1.2
    diam_t_fixed: float = 2e-3
    tether_force_limits: tuple = (50.0, 1800.0)
    airspeed_limits: tuple = (10.0, 32.0)
    rot_angles: tuple = (80.0 * math.pi / 180., 80.0 * math.pi / 180., 40.0 * math.pi / 180.0)
    delta_max: tuple = (20. * math.pi / 180., 30. * math.pi / 180., 30. * math.pi / 180.)
    ddelta_max: tuple = (2., 2., 2.)
    ddl_t_bounds: tuple = (-2.4, 2.4)
    alpha_max_deg: float = 9.0
    alpha_min_deg: float = -6.0
    beta_max_deg: float = 20.0
    beta_min_deg: float = -20.0


@dataclass
class Ap2Constants:
    """Everything the evaluator needs that does not change between NLP evaluations."""
    cfg: Ap2Config
    scaling: np.ndarray            # [59] SI = scaling * scaled (node variables)
    theta0: np.ndarray             # [NTHETA0] packed fixed parameters
    consts: np.ndarray             # [AWE_NCONST] model constants, see include/awegpu.h
    sd_len: np.ndarray             # [6, 9] int lengths of the stability-derivative stacks
    weights: np.ndarray            # [59] P.p.weights
    cost_steps: dict               # step label -> [20] cost vector
    details: dict = field(default_factory=dict)


def _u_at_altitude(cfg: Ap2Config, zz: float) -> float:
    # wind.get_speed 'power' with smooth_abs(zz, eps=1) (wind.py:184-208)
    z_cropped = math.sqrt(zz ** 2 + 1.0)
    return cfg.u_ref * (z_cropped / cfg.z_ref) ** cfg.exp_ref


def _loyd_phf(CL, CD, elevation):
    # performance_operations.get_loyd_phf (performance_operations.py:43-50)
    eps = 1.e-6
    interior = CD ** 2. / (CL ** 2 + eps ** 2.)
    CR = CL * (1. + interior) ** 0.5
    return 4. / 27. * CR * (CR / CD) ** 2. * math.cos(elevation) ** 3.


def _synthesize(estimates):
    # vector_operations.synthesize_estimate_from_a_list_of_positive_scalar_floats (:833-845)
    return float(np.exp(np.sum(np.log(estimates)) / len(estimates)))


def build_constants(cfg: Ap2Config | None = None) -> Ap2Constants:
    cfg = cfg or Ap2Config()
    g_scaling = 9.81              # model.scaling.other.g
    acc_max = 12.0                # model.model_bounds.acceleration.acc_max
    rho_ref = 1.225
    m_k = 36.8
    b_ref, s_ref = 5.5, 3.0
    c_ref = s_ref / b_ref
    diam_t_init = 5e-3            # solver.initialization.theta.diam_t (scaling, model_funcs.py:282-284)

    # estimates (model_funcs.py:1151-1462)
    elevation = cfg.inclination_deg * math.pi / 180.
    altitude = cfg.l_t_init * math.sin(elevation)
    u_alt = _u_at_altitude(cfg, altitude)
    flight_radius = cfg.groundspeed ** 2. / (acc_max * g_scaling)       # 'centripetal'
    t_f_guess = float((2. * math.pi * cfg.windings * flight_radius) / cfg.groundspeed)
    omega_guess = 2. * math.pi / (t_f_guess / float(cfg.windings))

    alpha = 9.0 * math.pi / 180.  # ampyx aero_validity alpha_max_deg used by estimate_CL/CD
    cosa, sina = math.cos(alpha), math.sin(alpha)
    CXe = -0.0293 + 0.4784 * alpha
    CZe = -0.5526 + -5.0676 * alpha
    rot = (CXe * -cosa + CZe * -sina, CXe * sina + CZe * -cosa)
    CL_est, CD_est = rot[1], rot[0]

    q_alt = 0.5 * rho_ref * u_alt ** 2
    power_density = u_alt * q_alt
    p_loyd = power_density * s_ref * _loyd_phf(CL_est, CD_est, elevation)
    power = 1 * p_loyd * 1. * 0.5   # number_of_kites * p_loyd * induction_eff * dof_eff(6dof)
    energy = power * t_f_guess
    power_cost = 1.0 * (1. / (power / energy))

    tension_per_length = ((cfg.tether_force_limits[0] + cfg.tether_force_limits[1]) / 2.) / cfg.l_t_init
    lambda_scaling = 1.0 * tension_per_length

    tether_mass = math.pi * (diam_t_init / 2.) ** 2. * cfg.l_t_init * cfg.tether_rho
    total_mass = m_k + tether_mass
    u_app = (u_alt ** 2 + cfg.groundspeed ** 2.) ** 0.5
    aero_force = CL_est * (0.5 * rho_ref * u_app ** 2) * s_ref
    estimates = [float(m_k * acc_max * g_scaling), tension_per_length * cfg.l_t_init,
                 total_mass * g_scaling / 1.0, float(m_k * cfg.groundspeed ** 2. / flight_radius),
                 float(aero_force)]
    f_scaling = _synthesize(estimates)
    m_scaling = f_scaling * b_ref / 2.

    airspeed_ref = (cfg.groundspeed ** 2. + u_alt ** 2.) ** 0.5
    ddl_t_scaling = float(np.max(np.array(cfg.ddl_t_bounds)) / 2.)

    # scaling per model variable (dynamics.py:824-921)
    sx = {"q10": [flight_radius] * 3, "dq10": [cfg.groundspeed] * 3, "omega10": [omega_guess] * 3,
          "r10": [1.0] * 9, "delta10": [v / 2. for v in cfg.delta_max], "l_t": [cfg.l_t_init],
          "dl_t": [u_alt / 3.]}
    su = {"f_fict10": [f_scaling] * 3, "m_fict10": [m_scaling] * 3,
          "ddelta10": [v / 2. for v in cfg.ddelta_max], "ddl_t": [ddl_t_scaling]}
    sz = {"lambda10": [lambda_scaling]}
    sth = {"diam_t": [diam_t_init], "t_f": [1.0]}
    # xdot scaling = scaling of the integral variable (dynamics.py:886-903)
    sxd = {"d" + n: v for n, v in sx.items()}
    scaling = np.concatenate([np.concatenate([np.array(d[n], dtype=np.float64) for n, _ in ents])
                              for d, ents in ((sx, X_VARS), (sxd, XDOT_VARS), (su, U_VARS),
                                              (sz, Z_VARS), (sth, THETA_VARS))])
    assert scaling.shape == (NW,)

    # theta0 values
    th = np.zeros(NTHETA0)

    def put(name, val):
        o, s = THETA0_OFF[name]
        th[o:o + s] = np.asarray(val, dtype=np.float64).reshape(-1)

    put("atmosphere.g", 9.81); put("atmosphere.gamma", 1.4); put("atmosphere.r", 287.053)
    put("atmosphere.t_ref", 288.15); put("atmosphere.p_ref", 101325.); put("atmosphere.rho_ref", 1.225)
    put("atmosphere.gamma_air", 6.5e-3); put("atmosphere.mu_ref", 1.789e-5)
    put("atmosphere.c_sutherland", 120.)
    put("wind.z_ref", cfg.z_ref); put("wind.log_wind.z0_air", 0.1)
    put("wind.power_wind.exp_ref", cfg.exp_ref); put("wind.u_ref", cfg.u_ref)
    put("tether.kappa", 10.); put("tether.rho", cfg.tether_rho); put("tether.cd", cfg.tether_cd)
    put("model_bounds.tether_force_limits", cfg.tether_force_limits)
    put("model_bounds.airspeed_limits", cfg.airspeed_limits)
    put("model_bounds.rot_angles", cfg.rot_angles)
    put("kappa_r", 1.)
    put("geometry.b_ref", b_ref); put("geometry.c_ref", c_ref); put("geometry.s_ref", s_ref)
    put("geometry.m_k", m_k)
    put("geometry.j", np.array([[25., 0.0, 0.47], [0.0, 32., 0.0], [0.47, 0.0, 56.]]).reshape(-1, order="F"))
    put("aero.moment_factor", 1.0)
    sd = np.zeros((len(SD_COEFFS), len(SD_INPUTS), SD_MAXLEN))
    sd_len = np.zeros((len(SD_COEFFS), len(SD_INPUTS)), dtype=np.int32)
    for ci, cname in enumerate(SD_COEFFS):
        for ii, iname in enumerate(SD_INPUTS):
            vals = AP2_STAB_DERIVS.get(cname, {}).get(iname)
            if vals:
                sd[ci, ii, :len(vals)] = vals
                sd_len[ci, ii] = len(vals)
    put("aero.stab_derivs", sd.reshape(-1))

    # weights (preparation.py:121-139)
    weights = np.ones(NW)
    for vt, ents in VAR_TYPES:
        for n, s in ents:
            o, _ = W_OFF[(vt, n)]
            base = split_name(n)
            weights[o:o + s] = SOLVER_WEIGHTS.get(base, 1.0)

    # cost schedule (scheduling.py:292-302, update_cost)
    sched = {k: list(v) for k, v in COST_SCHEDULE.items()}
    sched["power"][1] = power_cost
    counter = {k: -1 for k in COST_NAMES}
    cost = np.zeros(NCOST)
    cost_steps = {}
    for step, sub, names in COST_UPDATES:
        names = COST_NAMES if names is None else names
        for n in names:
            counter[n] += 1
            cost[COST_NAMES.index(n)] = sched[n][counter[n]]
        cost_steps[f"{step}{sub}"] = cost.copy()

    consts = pack_consts(cfg=cfg, scaling=scaling, f_scaling=f_scaling, m_scaling=m_scaling,
                         lambda_scaling=lambda_scaling, energy=energy, airspeed_ref=airspeed_ref,
                         diam_t_init=diam_t_init, g_scaling=g_scaling, sd_len=sd_len)
    details = dict(altitude=altitude, u_alt=u_alt, flight_radius=flight_radius, t_f_guess=t_f_guess,
                   omega_guess=omega_guess, CL_est=CL_est, CD_est=CD_est, power=power, energy=energy,
                   power_cost=power_cost, lambda_scaling=lambda_scaling, f_scaling=f_scaling,
                   m_scaling=m_scaling, airspeed_ref=airspeed_ref, estimates=estimates)
    return Ap2Constants(cfg=cfg, scaling=scaling, theta0=th, consts=consts, sd_len=sd_len,
                        weights=weights, cost_steps=cost_steps, details=details)


# layout of the model-constants vector; mirrors AWE_C_* in include/awegpu.h
CONST_NAMES = (
    ["n_k", "d", "scaling_length", "scaling_diam", "g_scaling", "q_scaling_mean", "lambda_scaling",
     "m_aero_scaling", "energy_scaling", "airspeed_ref", "alpha_max", "alpha_min", "beta_max",
     "beta_min", "aero_tightness", "norm_tracking", "norm_u_reg", "norm_theta_reg", "norm_xdot_reg",
     "norm_fictitious", "norm_beta", "n_elements"]
    + [f"scaling{i}" for i in range(NW)]
    + [f"sd_len{i}" for i in range(len(SD_COEFFS) * len(SD_INPUTS))]
)
NCONST = len(CONST_NAMES)
CONST_IDX = {n: i for i, n in enumerate(CONST_NAMES)}


def pack_consts(*, cfg, scaling, f_scaling, m_scaling, lambda_scaling, energy, airspeed_ref,
                diam_t_init, g_scaling, sd_len) -> np.ndarray:
    c = np.zeros(NCONST)
    n_nodes, n_kites = 2, 1
    vals = dict(
        n_k=cfg.n_k, d=cfg.d, scaling_length=cfg.l_t_init, scaling_diam=diam_t_init,
        g_scaling=g_scaling, q_scaling_mean=float(np.mean(scaling[0:3])),
        lambda_scaling=lambda_scaling, m_aero_scaling=m_scaling, energy_scaling=energy,
        airspeed_ref=airspeed_ref,
        alpha_max=cfg.alpha_max_deg * math.pi / 180.0, alpha_min=cfg.alpha_min_deg * math.pi / 180.0,
        beta_max=cfg.beta_max_deg * math.pi / 180.0, beta_min=cfg.beta_min_deg * math.pi / 180.0,
        aero_tightness=1.0,
        # funcs.py:148-153
        norm_tracking=cfg.n_k * n_nodes, norm_u_reg=cfg.n_k * n_kites, norm_theta_reg=cfg.n_k,
        norm_xdot_reg=cfg.n_k * n_nodes, norm_fictitious=cfg.n_k * n_kites, norm_beta=cfg.n_k * n_kites,
        n_elements=5,
    )
    for k, v in vals.items():
        c[CONST_IDX[k]] = v
    c[CONST_IDX["scaling0"]:CONST_IDX["scaling0"] + NW] = scaling
    c[CONST_IDX["sd_len0"]:CONST_IDX["sd_len0"] + sd_len.size] = sd_len.reshape(-1)
    return c


# ---------------------------------------------------------------------------------------
# NLP layout
# ---------------------------------------------------------------------------------------
class NlpLayout:
    """Index maps for V, P and g of the direct-collocation NLP (radau, zoh, phase_fix simple)."""

    def __init__(self, n_k: int = 40, d: int = 4):
        self.n_k, self.d = n_k, d
        self.n_coll_var = NX + NZ
        self.interval_stride = NX + NU + NX + NZ + d * self.n_coll_var      # 153 for d=4
        self.v_theta = 0
        self.v_phi = NTH
        self.v_xi = NTH + NPHI
        self.v_intervals = NTH + NPHI + NXI                                # 11
        self.n_v = self.v_intervals + n_k * self.interval_stride + NX
        self.rows_per_interval = N_EQ + N_INEQ + d * N_EQ + NX            # 152
        self.g_periodic = n_k * self.rows_per_interval
        self.n_g = self.g_periodic + NX
        self.n_p = self.n_v + NW + NCOST + NTHETA0
        self.p_ref, self.p_weights = 0, self.n_v
        self.p_cost, self.p_theta0 = self.n_v + NW, self.n_v + NW + NCOST

    # V indices -------------------------------------------------------------------------
    def x(self, k):
        base = self.v_intervals + k * self.interval_stride
        return np.arange(base, base + NX)

    def u(self, k):
        base = self.v_intervals + k * self.interval_stride + NX
        return np.arange(base, base + NU)

    def xdot(self, k):
        base = self.v_intervals + k * self.interval_stride + NX + NU
        return np.arange(base, base + NX)

    def z(self, k):
        base = self.v_intervals + k * self.interval_stride + 2 * NX + NU
        return np.arange(base, base + NZ)

    def coll_x(self, k, j):
        base = self.v_intervals + k * self.interval_stride + 2 * NX + NU + NZ + j * self.n_coll_var
        return np.arange(base, base + NX)

    def coll_z(self, k, j):
        base = self.v_intervals + k * self.interval_stride + 2 * NX + NU + NZ + j * self.n_coll_var + NX
        return np.arange(base, base + NZ)

    def theta(self):
        return np.arange(self.v_theta, self.v_theta + NTH)

    def phi(self, name=None):
        if name is None:
            return np.arange(self.v_phi, self.v_phi + NPHI)
        return self.v_phi + PHI_NAMES.index(name)

    # g indices -------------------------------------------------------------------------
    def g_shooting(self, k):
        b = k * self.rows_per_interval
        return np.arange(b, b + N_EQ)

    def g_path(self, k):
        b = k * self.rows_per_interval + N_EQ
        return np.arange(b, b + N_INEQ)

    def g_coll(self, k, j):
        b = k * self.rows_per_interval + N_EQ + N_INEQ + j * N_EQ
        return np.arange(b, b + N_EQ)

    def g_continuity(self, k):
        b = k * self.rows_per_interval + N_EQ + N_INEQ + self.d * N_EQ
        return np.arange(b, b + NX)

    def g_periodic_rows(self):
        return np.arange(self.g_periodic, self.g_periodic + NX)

    def g_bounds(self):
        lb = np.zeros(self.n_g)
        ub = np.zeros(self.n_g)
        for k in range(self.n_k):
            lb[self.g_path(k)] = -np.inf
        return lb, ub


# periodicity order: subkeys(...,'x') is sorted (struct_operations.py:51-66, operation.py:245-266)
def periodic_x_order() -> np.ndarray:
    off, _ = _offsets(X_VARS)
    out = []
    for name in sorted(n for n, _ in X_VARS):
        o, s = off[name]
        out.extend(range(o, o + s))
    return np.array(out)


def pack_p(layout: NlpLayout, consts: Ap2Constants, v_ref: np.ndarray, step: str = "power1",
           u_ref: float | None = None) -> np.ndarray:
    p = np.zeros(layout.n_p)
    p[layout.p_ref:layout.p_ref + layout.n_v] = v_ref
    p[layout.p_weights:layout.p_weights + NW] = consts.weights
    p[layout.p_cost:layout.p_cost + NCOST] = consts.cost_steps[step]
    th = consts.theta0.copy()
    if u_ref is not None:
        th[THETA0_OFF["wind.u_ref"][0]] = u_ref
    p[layout.p_theta0:layout.p_theta0 + NTHETA0] = th
    return p


def collocation(d: int = 4):
    return coefficients(d, "radau")


def sd_path(coeff: str, inp: str) -> tuple:
    """P path of a stability derivative: ``('theta0', 'aero', coeff, input)``.  model_funcs.py:
    483-493 appends ('params', 'aero', deriv_name, input_name) for every derivative of the kite
    data (all flagged 's', default.py:599), and stability_derivatives.py:241-243 reads them back
    as ``parameters['theta0', 'aero', coeff_name, input_name]`` -- there is no 'stab_derivs' level."""
    return ("theta0", "aero", coeff, inp)


def stab_derivs_present(get) -> dict:
    """{coeff: [inputs]} of the stability derivatives in the reference's P: the reference keeps only
    the (coeff, input) pairs its kite data define (stability_derivatives.py:230-249 tests the
    label); a pair is absent exactly when ``get`` raises KeyError."""
    out = {}
    for c in SD_COEFFS:
        for i in SD_INPUTS:
            try:
                get(sd_path(c, i))
            except KeyError:
                continue
            out.setdefault(c, []).append(i)
    return out


def pack_p_from_reference(get, layout, stab_derivs_absent: dict | None = None) -> np.ndarray:
    """P in this library's flat layout from the reference's P struct, read entry by entry by name.

    The reference hands IPOPT ``p = P(p_fix_num)`` with ``P = struct([p: [ref (the V struct),
    weights (model.variables)], cost (setup_nlp_cost's 20 entries), theta0 (the params tree)])``
    (ocp/discretization.py:129-179; theta0 = struct_op.generate_nested_dict_struct(options['params']),
    mdl/system.py:417-432).  ``get(path)`` returns the entry at ``path`` as an array, e.g.
    ``get(('p', 'ref'))``, ``get(('cost', 'power'))``, ``get(('theta0', 'wind', 'u_ref'))`` or
    ``get(('theta0', 'aero', 'CX', 'alpha'))`` (``sd_path``); with a casadi.tools struct ``P_num``:
    ``get = lambda path: np.asarray(P_num[path]).ravel()``.  The flat order of the theta0 tree is
    never used, only the names of the entries the evaluator reads.

    ``layout`` is the AP2 ``NlpLayout`` or the multi-kite ``dual.MultiLayout`` (same P structure,
    its own V and weight sizes).  Every entry is required: a missing name raises KeyError --
    except the stability derivatives listed in ``stab_derivs_absent`` ({coeff: [inputs]}), which
    the kite data does not define and which are zero in the model (stability_derivatives.py:
    166-200 sums only the derivatives present).  By default that list is the complement of
    ``AP2_STAB_DERIVS`` (ampyx_data.py:121-223)."""
    if stab_derivs_absent is None:
        stab_derivs_absent = {c: [i for i in SD_INPUTS if i not in AP2_STAB_DERIVS.get(c, {})]
                              for c in SD_COEFFS}
    nw = layout.p_cost - layout.p_weights
    p = np.zeros(layout.n_p)
    p[layout.p_ref:layout.p_ref + layout.n_v] = np.asarray(get(("p", "ref")), dtype=np.float64).ravel()
    w = np.asarray(get(("p", "weights")), dtype=np.float64).ravel()
    if w.size != nw:
        raise ValueError(f"p.weights has {w.size} values, expected {nw}")
    p[layout.p_weights:layout.p_weights + nw] = w
    for i, name in enumerate(COST_NAMES):
        p[layout.p_cost + i] = float(np.asarray(get(("cost", name))).ravel()[0])
    th = np.zeros(NTHETA0)
    for name, size in THETA0_ENTRIES:
        o, _ = THETA0_OFF[name]
        if name == "aero.stab_derivs":
            for ci, cname in enumerate(SD_COEFFS):
                for ii, iname in enumerate(SD_INPUTS):
                    try:
                        v = np.asarray(get(sd_path(cname, iname)), dtype=np.float64).ravel()
                    except KeyError:
                        if iname in stab_derivs_absent.get(cname, ()):
                            continue
                        raise KeyError(f"stability derivative {sd_path(cname, iname)} missing from the "
                                       f"reference P (not listed as absent from the kite data)") from None
                    if len(v) > SD_MAXLEN:
                        raise ValueError(f"stability derivative {cname}.{iname} has {len(v)} > {SD_MAXLEN} terms")
                    b = o + (ci * len(SD_INPUTS) + ii) * SD_MAXLEN
                    th[b:b + len(v)] = v
        else:
            v = np.asarray(get(("theta0",) + tuple(name.split("."))), dtype=np.float64).ravel()
            if v.size != size:
                raise ValueError(f"theta0 entry {name} has {v.size} values, expected {size}")
            th[o:o + size] = v
    p[layout.p_theta0:layout.p_theta0 + NTHETA0] = th
    return p


def reference_p_entries(P: np.ndarray, layout) -> dict:
    """The inverse view: {path: array} of a flat P under the reference's entry names (the paths
    pack_p_from_reference reads); stability derivatives with their used terms only."""
    P = np.asarray(P, dtype=np.float64)
    nw = layout.p_cost - layout.p_weights
    out = {("p", "ref"): P[layout.p_ref:layout.p_ref + layout.n_v].copy(),
           ("p", "weights"): P[layout.p_weights:layout.p_weights + nw].copy()}
    for i, name in enumerate(COST_NAMES):
        out[("cost", name)] = np.array([P[layout.p_cost + i]])
    th = P[layout.p_theta0:layout.p_theta0 + NTHETA0]
    for name, size in THETA0_ENTRIES:
        o, _ = THETA0_OFF[name]
        if name == "aero.stab_derivs":
            for ci, cname in enumerate(SD_COEFFS):
                for ii, iname in enumerate(SD_INPUTS):
                    vals = AP2_STAB_DERIVS.get(cname, {}).get(iname)
                    if vals:
                        b = o + (ci * len(SD_INPUTS) + ii) * SD_MAXLEN
                        out[sd_path(cname, iname)] = th[b:b + len(vals)].copy()
        else:
            out[("theta0",) + tuple(name.split("."))] = th[o:o + size].copy()
    return out
