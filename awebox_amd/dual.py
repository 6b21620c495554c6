"""Host-side description of the multi-kite power-cycle OCP (config 3: dual kites, N=60, d=4).

Restates, for the architectures ``{1: 0}`` (single kite, the AP2 path of ``problem.py``) and
``{1: 0, 2: 1, 3: 1}`` (two kites on secondary tethers below a layer node, the example
``examples/dual_kites_power_curve.py``), the parts of the awebox build pipeline that produce
constants for the hot path:

* the model variables per architecture (``awebox/mdl/system.py:42-230``; order x, xdot, u, z,
  theta; node-major inside each group),
* the option-derived scaling (``awebox/opts/model_funcs.py:227-320, 993-1183, 1358-1470``):
  dq of the layer node scaled by the wind at altitude, the secondary tether length/diameter from
  ``solver.initialization.theta``, the lambda scaling tree (``:1093-1138``), the multi-kite
  total-mass and power estimates,
* the NLP layout with the ``single_reelout`` phase fix (``ocp/var_struct.py:46-49, 99-110``:
  ``theta.t_f`` has two entries; ``ocp/constraints.py:127-170``: two global ``t_f`` bound rows
  after the periodicity rows),
* the standard multi-kite initial guess (``opti/initialization_dir/standard_scenario.py:72-149``,
  ``tools.py:39-330``: layer node on the tether axis, kites on a cone of half-angle
  ``cone_deg`` around it with azimuths offset by 2 pi / 2).

Everything that is shared with the single-kite path (``theta0`` packing, stability derivatives,
solver weights, homotopy costs) is taken from ``problem.py``.
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field

import numpy as np

from . import problem as pb

ARCH_SINGLE = {1: 0}
ARCH_DUAL = {1: 0, 2: 1, 3: 1}


class Architecture:
    """``awebox/mdl/architecture.py:33-120``: kite nodes = nodes without children."""

    def __init__(self, parent_map: dict):
        self.parent_map = dict(parent_map)
        self.number_of_nodes = len(self.parent_map) + 1
        parents = set(self.parent_map.values())
        self.kite_nodes = [n for n in self.parent_map if n not in parents]
        self.number_of_kites = len(self.kite_nodes)
        self.children_map = {}
        for n, p in self.parent_map.items():
            self.children_map.setdefault(p, []).append(n)
        if self.number_of_nodes == 2:
            self.layer_nodes, self.layers = [0], 1
        else:
            self.layer_nodes = sorted(set(self.parent_map.values()) - {0})
            self.layers = len(self.layer_nodes)
        # level siblings (architecture.get_all_level_siblings): kites sharing a parent
        self.level_siblings = {}
        for k in self.kite_nodes:
            self.level_siblings.setdefault(self.parent_map[k], []).append(k)

    def label(self, n: int) -> str:
        return f"{n}{self.parent_map[n]}"


def model_variables(arch: Architecture):
    """(x, xdot, u, z, theta) name/size lists (system.py:42-230; kite_dof 6, surface_control 1,
    lift_mode, tether control 'ddl_t', integral_outputs, no lifted forces)."""
    X, U, Z = [], [], []
    for n in range(1, arch.number_of_nodes):
        lab = arch.label(n)
        if n in arch.kite_nodes:
            X += [(f"q{lab}", 3), (f"dq{lab}", 3), (f"omega{lab}", 3), (f"r{lab}", 9), (f"delta{lab}", 3)]
            U += [(f"f_fict{lab}", 3), (f"m_fict{lab}", 3), (f"ddelta{lab}", 3)]
        else:
            X += [(f"q{lab}", 3), (f"dq{lab}", 3)]
        Z += [(f"lambda{lab}", 1)]
    X += [("l_t", 1), ("dl_t", 1)]
    U += [("ddl_t", 1)]
    XD = [("d" + n, s) for n, s in X]
    TH = [("diam_t", 1), ("t_f", 1)]
    if arch.number_of_nodes - arch.number_of_kites > 1:
        TH += [("l_s", 1), ("diam_s", 1)]
    return X, XD, U, Z, TH


@dataclass
class MultiConfig:
    """User options of examples/dual_kites_power_curve.py + ampyx_ap2_settings.py."""
    parent_map: dict = field(default_factory=lambda: dict(ARCH_DUAL))
    n_k: int = 60
    d: int = 4
    u_ref: float = 10.0
    z_ref: float = 10.0                 # dual_kites_power_curve.py:33
    exp_ref: float = 0.15
    groundspeed: float = 15.0
    inclination_deg: float = 45.0
    cone_deg: float = 15.0
    l_t_init: float = 200.0
    l_s_init: float = 50.0              # default.py:378
    diam_t_init: float = 5e-3           # default.py:380
    diam_s_init: float = 5e-3           # default.py:382
    windings: int = 1
    phase_fix: str = "single_reelout"   # default.py:44 (the example keeps it)
    phase_fix_reelout: float = 0.7      # default.py:294
    t_f_bounds: tuple = (10.0, 20.0)    # dual_kites_power_curve.py:30
    l_t_bounds: tuple = (0.0, 1.0e3)    # dual_kites_power_curve.py:29
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
    anticollision_safety: float = 5.0   # default.py:222

    @property
    def nk_reelout(self) -> int:
        return int(round(self.n_k * self.phase_fix_reelout))


def ap2_single_config(n_k: int = 40, d: int = 4) -> MultiConfig:
    """The AP2 single-kite options of problem.Ap2Config expressed as a MultiConfig."""
    return MultiConfig(parent_map=dict(ARCH_SINGLE), n_k=n_k, d=d, z_ref=100.0, phase_fix="simple")


class Model:
    """Variable layout of one architecture: node-vector offsets, names, row names."""

    def __init__(self, arch: Architecture):
        self.arch = arch
        self.X, self.XD, self.U, self.Z, self.TH = model_variables(arch)
        self.groups = [("x", self.X), ("xdot", self.XD), ("u", self.U), ("z", self.Z), ("theta", self.TH)]
        self.off = {}
        pos = 0
        for vt, ents in self.groups:
            for n, s in ents:
                self.off[(vt, n)] = (pos, s)
                pos += s
        self.nw = pos
        self.nx = sum(s for _, s in self.X)
        self.nu = sum(s for _, s in self.U)
        self.nz = sum(s for _, s in self.Z)
        self.nth = sum(s for _, s in self.TH)
        self.w_x0, self.w_xd0 = 0, self.nx
        self.w_u0 = 2 * self.nx
        self.w_z0 = 2 * self.nx + self.nu
        self.w_th0 = 2 * self.nx + self.nu + self.nz
        kites = arch.kite_nodes
        nodes = range(1, arch.number_of_nodes)
        self.eq_names = ([f"dynamics_translation{n}" for n in nodes for _ in range(3)]
                         + [f"dynamics_constraint{n}" for n in nodes])
        for k in kites:
            self.eq_names += [f"rotation_dynamics{k}"] * 3 + [f"ref_frame_dynamics{k}"] * 9
        for name in self.trivial_names():
            self.eq_names += [f"trivial_{name}"] * self.size(name)
        self.ineq_names = []
        for k in kites:   # tether_constraint_includes['force'] = kite nodes (model_funcs.py:879-880)
            lab = arch.label(k)
            self.ineq_names += [f"tether_force_max{lab}", f"tether_force_min{lab}"]
        for k in kites:
            lab = arch.label(k)
            self.ineq_names += [f"airspeed_max{lab}", f"airspeed_min{lab}"]
        for k in kites:
            self.ineq_names += [f"alpha_ub{k}", f"alpha_lb{k}", f"beta_ub{k}", f"beta_lb{k}"]
        for a, b in itertools.combinations(kites, 2):
            self.ineq_names += [f"anticollision{a}{b}"]
        for k in kites:
            self.ineq_names += [f"rotation_max{arch.label(k)}"]
        self.n_eq = len(self.eq_names)
        self.n_ineq = len(self.ineq_names)

    def size(self, name):
        for vt, ents in self.groups:
            for n, s in ents:
                if n == name:
                    return s
        raise KeyError(name)

    def trivial_names(self):
        """xdot names that also live in x or u, sorted (lagr_dyn.py:141-169)."""
        xs = {n for n, _ in self.X}
        us = {n for n, _ in self.U}
        return sorted(n for n, _ in self.XD if n in xs or n in us)

    def undiff_type(self, name):
        return "x" if name in {n for n, _ in self.X} else "u"

    def sl(self, vt, name):
        o, s = self.off[(vt, name)]
        return slice(o, o + s)

    def periodic_order(self):
        """Sorted x names (struct_op.subkeys, operation.py:245-266) as x-vector indices."""
        xo = {}
        pos = 0
        for n, s in self.X:
            xo[n] = (pos, s)
            pos += s
        out = []
        for n in sorted(xo):
            o, s = xo[n]
            out.extend(range(o, o + s))
        return np.array(out)


@dataclass
class MultiConstants:
    cfg: MultiConfig
    model: Model
    scaling: np.ndarray         # [nw]
    theta0: np.ndarray          # [pb.NTHETA0]
    consts: np.ndarray          # [NCONST] kernel constants (include/awedual.h ADL_C_*)
    sd_len: np.ndarray
    weights: np.ndarray         # [nw]
    cost_steps: dict
    details: dict = field(default_factory=dict)


def _u_at(cfg, zz):
    return cfg.u_ref * (math.sqrt(zz ** 2 + 1.0) / cfg.z_ref) ** cfg.exp_ref


def build_constants(cfg: MultiConfig | None = None) -> MultiConstants:
    cfg = cfg or MultiConfig()
    arch = Architecture(cfg.parent_map)
    model = Model(arch)
    nk_kites = arch.number_of_kites
    g_scaling, acc_max, rho_ref = 9.81, 12.0, 1.225
    m_k, b_ref, s_ref = 36.8, 5.5, 3.0
    elevation = cfg.inclination_deg * math.pi / 180.
    altitude = cfg.l_t_init * math.sin(elevation)                      # estimate_altitude
    u_alt = _u_at(cfg, altitude)
    flight_radius = cfg.groundspeed ** 2. / (acc_max * g_scaling)     # 'centripetal' (:1183-1216)
    t_f_guess = float((2. * math.pi * cfg.windings * flight_radius) / cfg.groundspeed)
    omega_guess = 2. * math.pi / (t_f_guess / float(cfg.windings))

    alpha = 9.0 * math.pi / 180.
    cosa, sina = math.cos(alpha), math.sin(alpha)
    CXe, CZe = -0.0293 + 0.4784 * alpha, -0.5526 + -5.0676 * alpha
    CL_est, CD_est = CXe * sina + CZe * -cosa, CXe * -cosa + CZe * -sina
    q_alt = 0.5 * rho_ref * u_alt ** 2
    p_loyd = u_alt * q_alt * s_ref * pb._loyd_phf(CL_est, CD_est, elevation)
    power = nk_kites * p_loyd * 1.0 * 0.5                               # estimate_power (:1251-1287)
    energy = power * t_f_guess
    power_cost = 1.0 * (1. / (power / energy))

    tension_per_length = ((cfg.tether_force_limits[0] + cfg.tether_force_limits[1]) / 2.) / cfg.l_t_init
    lambda_main = 1.0 * tension_per_length
    rho_t = cfg.tether_rho
    mass_main = math.pi * (cfg.diam_t_init / 2.) ** 2. * cfg.l_t_init * rho_t
    mass_sec = (math.pi * (cfg.diam_s_init / 2.) ** 2. * cfg.l_s_init * rho_t * nk_kites) if nk_kites > 1 else 0.0
    total_mass = m_k * nk_kites + mass_main + mass_sec                  # estimate_total_mass (:1421-1449)
    u_app = (u_alt ** 2 + cfg.groundspeed ** 2.) ** 0.5
    aero_force = CL_est * (0.5 * rho_ref * u_app ** 2) * s_ref
    estimates = [float(m_k * acc_max * g_scaling), tension_per_length * cfg.l_t_init,
                 total_mass * g_scaling / float(nk_kites), float(m_k * cfg.groundspeed ** 2. / flight_radius),
                 float(aero_force)]
    f_scaling = pb._synthesize(estimates)
    m_scaling = f_scaling * b_ref / 2.
    airspeed_ref = (cfg.groundspeed ** 2. + u_alt ** 2.) ** 0.5
    ddl_t_scaling = float(np.max(np.array(cfg.ddl_t_bounds)) / 2.)

    # lambda scaling tree (model_funcs.py:1093-1138): secondary = main tension / n_kites / l_s
    lambda_s = lambda_main * cfg.l_t_init / nk_kites / cfg.l_s_init

    sc = {}
    for n in range(1, arch.number_of_nodes):
        lab = arch.label(n)
        sc[f"q{lab}"] = [flight_radius] * 3
        sc[f"dq{lab}"] = [cfg.groundspeed if n in arch.kite_nodes else u_alt] * 3
        if n in arch.kite_nodes:
            sc[f"omega{lab}"] = [omega_guess] * 3
            sc[f"r{lab}"] = [1.0] * 9
            sc[f"delta{lab}"] = [v / 2. for v in cfg.delta_max]
            sc[f"f_fict{lab}"] = [f_scaling] * 3
            sc[f"m_fict{lab}"] = [m_scaling] * 3
            sc[f"ddelta{lab}"] = [v / 2. for v in cfg.ddelta_max]
        sc[f"lambda{lab}"] = [lambda_main if n == 1 else lambda_s]
    sc.update({"l_t": [cfg.l_t_init], "dl_t": [u_alt / 3.], "ddl_t": [ddl_t_scaling],
               "diam_t": [cfg.diam_t_init], "t_f": [1.0], "l_s": [cfg.l_s_init], "diam_s": [cfg.diam_s_init]})
    scaling = np.zeros(model.nw)
    for (vt, n), (o, s) in model.off.items():
        key = n[1:] if vt == "xdot" else n          # xdot scaled like its integral (dynamics.py:886-903)
        scaling[o:o + s] = sc[key]

    cfg_ap2 = pb.Ap2Config(n_k=cfg.n_k, d=cfg.d, u_ref=cfg.u_ref, z_ref=cfg.z_ref, exp_ref=cfg.exp_ref)
    base = pb.build_constants(cfg_ap2)              # theta0 packing, stability derivatives
    theta0 = base.theta0.copy()
    weights = np.ones(model.nw)
    for (vt, n), (o, s) in model.off.items():
        weights[o:o + s] = pb.SOLVER_WEIGHTS.get(pb.split_name(n), 1.0)
    sched = {k: list(v) for k, v in pb.COST_SCHEDULE.items()}
    sched["power"][1] = power_cost
    counter = {k: -1 for k in pb.COST_NAMES}
    cost = np.zeros(pb.NCOST)
    cost_steps = {}
    for step, sub, names in pb.COST_UPDATES:
        for n in (pb.COST_NAMES if names is None else names):
            counter[n] += 1
            cost[pb.COST_NAMES.index(n)] = sched[n][counter[n]]
        cost_steps[f"{step}{sub}"] = cost.copy()

    vals = dict(
        n_k=cfg.n_k, d=cfg.d, nk_reelout=cfg.nk_reelout if cfg.phase_fix == "single_reelout" else cfg.n_k,
        single_reelout=1.0 if cfg.phase_fix == "single_reelout" else 0.0,
        phase_fix_reelout=cfg.phase_fix_reelout, tf_lb=cfg.t_f_bounds[0], tf_ub=cfg.t_f_bounds[1],
        scaling_length_t=cfg.l_t_init, scaling_length_s=cfg.l_s_init,
        scaling_diam_t=cfg.diam_t_init, scaling_diam_s=cfg.diam_s_init, g_scaling=g_scaling,
        m_aero_scaling=m_scaling, energy_scaling=energy, airspeed_ref=airspeed_ref,
        alpha_max=cfg.alpha_max_deg * math.pi / 180.0, alpha_min=cfg.alpha_min_deg * math.pi / 180.0,
        beta_max=cfg.beta_max_deg * math.pi / 180.0, beta_min=cfg.beta_min_deg * math.pi / 180.0,
        aero_tightness=1.0,
        norm_tracking=cfg.n_k * arch.number_of_nodes, norm_u_reg=cfg.n_k * nk_kites, norm_theta_reg=cfg.n_k,
        norm_xdot_reg=cfg.n_k * arch.number_of_nodes, norm_fictitious=cfg.n_k * nk_kites,
        norm_beta=cfg.n_k * nk_kites, n_elements=5,
        anticollision_dist_min=cfg.anticollision_safety * b_ref,
    )
    consts = np.zeros(NCONST)
    for k, v in vals.items():
        consts[CONST_IDX[k]] = v
    consts[CONST_IDX["scaling0"]:CONST_IDX["scaling0"] + model.nw] = scaling
    consts[CONST_IDX["sd_len0"]:CONST_IDX["sd_len0"] + base.sd_len.size] = base.sd_len.reshape(-1)
    details = dict(altitude=altitude, u_alt=u_alt, flight_radius=flight_radius, t_f_guess=t_f_guess,
                   omega_guess=omega_guess, power=power, energy=energy, power_cost=power_cost,
                   lambda_main=lambda_main, lambda_s=lambda_s, f_scaling=f_scaling, m_scaling=m_scaling,
                   airspeed_ref=airspeed_ref, estimates=estimates, total_mass=total_mass)
    return MultiConstants(cfg=cfg, model=model, scaling=scaling, theta0=theta0, consts=consts,
                          sd_len=base.sd_len, weights=weights, cost_steps=cost_steps, details=details)


# kernel constants (mirrors ADL_C_* in include/awedual.h)
CONST_NAMES = (
    ["n_k", "d", "nk_reelout", "single_reelout", "phase_fix_reelout", "tf_lb", "tf_ub",
     "scaling_length_t", "scaling_length_s", "scaling_diam_t", "scaling_diam_s", "g_scaling",
     "m_aero_scaling", "energy_scaling", "airspeed_ref", "alpha_max", "alpha_min", "beta_max", "beta_min",
     "aero_tightness", "norm_tracking", "norm_u_reg", "norm_theta_reg", "norm_xdot_reg", "norm_fictitious",
     "norm_beta", "n_elements", "anticollision_dist_min"]
    + [f"scaling{i}" for i in range(126)]
    + [f"sd_len{i}" for i in range(len(pb.SD_COEFFS) * len(pb.SD_INPUTS))]
)
NCONST = len(CONST_NAMES)
CONST_IDX = {n: i for i, n in enumerate(CONST_NAMES)}


# ---------------------------------------------------------------------------------------
# NLP layout (var_struct.py:39-115 with the single_reelout theta; constraints.py:48-170)
# ---------------------------------------------------------------------------------------
class MultiLayout:
    def __init__(self, model: Model, n_k: int, d: int, phase_fix: str = "single_reelout",
                 phase_fix_reelout: float = 0.7):
        self.model = model
        self.n_k, self.d = n_k, d
        self.single_reelout = phase_fix == "single_reelout"
        self.nk_reelout = int(round(n_k * phase_fix_reelout)) if self.single_reelout else n_k
        m = model
        # V.theta: node theta with t_f repeated (var_struct.get_phase_fix_theta)
        self.theta_names = []
        for n, s in m.TH:
            if n == "t_f" and self.single_reelout:
                self.theta_names += ["t_f0", "t_f1"]
            else:
                self.theta_names.append(n)
        self.n_theta = len(self.theta_names)
        self.v_phi = self.n_theta
        self.v_xi = self.n_theta + pb.NPHI
        self.v_intervals = self.n_theta + pb.NPHI + pb.NXI
        self.n_coll_var = m.nx + m.nz
        self.interval_stride = 2 * m.nx + m.nu + m.nz + d * self.n_coll_var
        self.n_v = self.v_intervals + n_k * self.interval_stride + m.nx
        self.rows_per_interval = m.n_eq + m.n_ineq + d * m.n_eq + m.nx
        self.g_periodic = n_k * self.rows_per_interval
        self.n_tf_rows = 2 if self.single_reelout else 0
        self.g_tf = self.g_periodic + m.nx
        self.n_g = self.g_tf + self.n_tf_rows
        self.n_p = self.n_v + m.nw + pb.NCOST + pb.NTHETA0
        self.p_ref, self.p_weights = 0, self.n_v
        self.p_cost, self.p_theta0 = self.n_v + m.nw, self.n_v + m.nw + pb.NCOST

    @property
    def nx(self):
        return self.model.nx

    def theta_index(self, name):
        return self.theta_names.index(name)

    def tf_index(self, k):
        """V index of the t_f governing interval k (struct_op.calculate_tf)."""
        if not self.single_reelout:
            return self.theta_index("t_f")
        return self.theta_index("t_f0") if k < self.nk_reelout else self.theta_index("t_f1")

    def node_theta_index(self, k):
        """V indices of the node theta vector of interval k (struct_op.get_V_theta)."""
        out = []
        for n, _ in self.model.TH:
            out.append(self.tf_index(k) if n == "t_f" else self.theta_index(n))
        return np.array(out)

    def base(self, k):
        return self.v_intervals + k * self.interval_stride

    def x(self, k):
        return np.arange(self.base(k), self.base(k) + self.model.nx)

    def u(self, k):
        b = self.base(k) + self.model.nx
        return np.arange(b, b + self.model.nu)

    def xdot(self, k):
        b = self.base(k) + self.model.nx + self.model.nu
        return np.arange(b, b + self.model.nx)

    def z(self, k):
        b = self.base(k) + 2 * self.model.nx + self.model.nu
        return np.arange(b, b + self.model.nz)

    def coll_x(self, k, j):
        b = self.base(k) + 2 * self.model.nx + self.model.nu + self.model.nz + j * self.n_coll_var
        return np.arange(b, b + self.model.nx)

    def coll_z(self, k, j):
        b = self.base(k) + 2 * self.model.nx + self.model.nu + self.model.nz + j * self.n_coll_var + self.model.nx
        return np.arange(b, b + self.model.nz)

    def phi(self):
        return np.arange(self.v_phi, self.v_phi + pb.NPHI)

    def g_shooting(self, k):
        b = k * self.rows_per_interval
        return np.arange(b, b + self.model.n_eq)

    def g_path(self, k):
        b = k * self.rows_per_interval + self.model.n_eq
        return np.arange(b, b + self.model.n_ineq)

    def g_bounds(self):
        lb, ub = np.zeros(self.n_g), np.zeros(self.n_g)
        for k in range(self.n_k):
            lb[self.g_path(k)] = -np.inf
        lb[self.g_tf:self.g_tf + self.n_tf_rows] = -np.inf
        return lb, ub

    def local_index(self, k):
        """V indices of interval k's local slice: [theta, phi, x[k], u, xdot, z, coll.., x[k+1]]."""
        glob = np.arange(0, self.n_theta + pb.NPHI)
        b = self.base(k)
        return np.concatenate([glob, np.arange(b, b + self.interval_stride + self.model.nx)])


def layout_for(consts: MultiConstants) -> MultiLayout:
    c = consts.cfg
    return MultiLayout(consts.model, c.n_k, c.d, c.phase_fix, c.phase_fix_reelout)


# ---------------------------------------------------------------------------------------
# standard multi-kite initial guess (standard_scenario.py:72-149, tools.py:39-330)
# ---------------------------------------------------------------------------------------
def _normalize(v):
    return v / np.linalg.norm(v)


def _ncross(a, b):
    return _normalize(np.cross(a, b))


def guess_values_at_time(t: float, consts: MultiConstants) -> dict:
    cfg, arch = consts.cfg, consts.model.arch
    hyp = cfg.l_t_init if arch.number_of_kites == 1 else cfg.l_s_init      # set_fixed_hypotenuse
    radius = hyp * math.sin(cfg.cone_deg * math.pi / 180.0)
    gs = cfg.groundspeed
    for _ in range(3):                        # clipping loop (no clip triggers at these options)
        period = 2. * math.pi * radius / gs
        gs = 2. * math.pi * radius / period
    height = (hyp ** 2. - radius ** 2.) ** 0.5
    omega_norm = gs / radius
    incl = cfg.inclination_deg * math.pi / 180.
    n_hat = np.array([math.cos(incl), 0.0, math.sin(incl)])
    xhat = np.array([1.0, 0.0, 0.0])
    y_rot = _ncross(n_hat, xhat)
    z_rot = _ncross(n_hat, y_rot)
    zz = cfg.l_t_init * n_hat[2]
    u_inf = _u_at(cfg, zz) * xhat
    ret = {"l_t": np.array([cfg.l_t_init]), "dl_t": np.array([0.0])}
    for n in range(1, arch.number_of_nodes):
        lab = arch.label(n)
        parent = arch.parent_map[n]
        p_pos = np.zeros(3) if parent == 0 else ret[f"q{arch.label(parent)}"]
        if n not in arch.kite_nodes:
            ret[f"q{lab}"] = p_pos + cfg.l_t_init * n_hat if n == 1 else p_pos + 100.0 * n_hat
            ret[f"dq{lab}"] = np.zeros(3)
            ret[f"ddq{lab}"] = np.zeros(3)
            continue
        sib = arch.level_siblings[parent]
        psi0 = 0.0 if len(sib) == 1 else float(sib.index(n)) / float(len(sib)) * 2. * math.pi
        psi = (psi0 + omega_norm * t) % (2. * math.pi)
        outward = z_rot * math.cos(psi) - y_rot * math.sin(psi)        # clockwise, sign = +1
        e_tan = _ncross(n_hat, outward)
        q = p_pos + outward * radius + n_hat * height
        dq = gs * e_tan
        ret[f"q{lab}"] = q
        ret[f"dq{lab}"] = dq
        ret[f"ddq{lab}"] = gs ** 2 / radius * (-outward)
        e_normal = _normalize(ret["q10"])                             # 'tether_parallel'
        e1 = _normalize(u_inf - dq)
        e2 = _ncross(e_normal, e1)
        e3 = _ncross(e1, e2)
        dcm = np.stack([e1, e2, e3], axis=1)
        om = omega_norm * np.array([0., 0., 1.])
        ddcm = dcm @ np.array([[0., -om[2], om[1]], [om[2], 0., -om[0]], [-om[1], om[0], 0.]])
        ret[f"omega{lab}"] = om
        ret[f"domega{lab}"] = np.zeros(3)
        ret[f"r{lab}"] = dcm.reshape(-1, order="F")
        ret[f"dr{lab}"] = ddcm.reshape(-1, order="F")
        ret[f"delta{lab}"] = np.zeros(3)
    ret["_tf"] = period * cfg.windings
    return ret


def initial_guess(consts: MultiConstants, lay: MultiLayout) -> np.ndarray:
    """Scaled V0 (initialization.get_initial_guess with the standard scenario)."""
    from .collocation import coefficients
    m = consts.model
    tf = guess_values_at_time(0.0, consts)["_tf"]
    tau, C, D, w = coefficients(lay.d, "radau")
    s = consts.scaling
    sx = s[m.w_x0:m.w_x0 + m.nx]

    def x_vec(ret):
        out = np.zeros(m.nx)
        pos = 0
        for n, sz in m.X:
            out[pos:pos + sz] = ret[n]
            pos += sz
        return out

    V = np.zeros(lay.n_v)
    th = {"diam_t": consts.cfg.diam_t_fixed, "t_f": tf, "t_f0": tf, "t_f1": tf,
          "l_s": consts.cfg.l_s_init, "diam_s": consts.cfg.diam_s_init}
    th_scale = {n: s[m.w_th0 + i] for i, (n, _) in enumerate(m.TH)}
    for i, n in enumerate(lay.theta_names):
        V[i] = th[n] / th_scale["t_f" if n.startswith("t_f") else n]
    V[lay.phi()] = 1.0
    n_k, d = lay.n_k, lay.d
    for k in range(n_k + 1):
        V[lay.x(k)] = x_vec(guess_values_at_time(k * tf / n_k, consts)) / sx
        if k < n_k:
            V[lay.z(k)] = 1.0
            for j in range(d):
                t = (k + tau[j + 1]) * tf / n_k
                V[lay.coll_x(k, j)] = x_vec(guess_values_at_time(t, consts)) / sx
                V[lay.coll_z(k, j)] = 1.0
    h = 1.0 / n_k
    for k in range(n_k):
        X = np.stack([V[lay.x(k)]] + [V[lay.coll_x(k, j)] for j in range(d)])
        V[lay.xdot(k)] = (C[:, 0] @ X) / h / V[lay.tf_index(k)]
    return V


def batch_member(v0: np.ndarray, lay: MultiLayout, b: int, sigma: float = 0.01,
                 seed_base: int = 20261015) -> np.ndarray:
    """V_b = V0 + 0.01 N(0,1) on all non-fixed entries, rng(20261015 + b)."""
    rng = np.random.default_rng(seed_base + b)
    v = v0.copy()
    noise = sigma * rng.standard_normal(v.shape)
    fixed = np.zeros(v.shape, dtype=bool)
    fixed[lay.theta_index("diam_t")] = True
    fixed[lay.v_xi:lay.v_xi + pb.NXI] = True
    v[~fixed] += noise[~fixed]
    return v


def pack_p(lay: MultiLayout, consts: MultiConstants, v_ref: np.ndarray, step: str = "power1",
           u_ref: float | None = None) -> np.ndarray:
    m = consts.model
    p = np.zeros(lay.n_p)
    p[lay.p_ref:lay.p_ref + lay.n_v] = v_ref
    p[lay.p_weights:lay.p_weights + m.nw] = consts.weights
    p[lay.p_cost:lay.p_cost + pb.NCOST] = consts.cost_steps[step]
    th = consts.theta0.copy()
    if u_ref is not None:
        th[pb.THETA0_OFF["wind.u_ref"][0]] = u_ref
    p[lay.p_theta0:lay.p_theta0 + pb.NTHETA0] = th
    return p
