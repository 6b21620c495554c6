"""CPU ORACLE for the 3-DOF tracking-MPC evaluator -- TEST INFRASTRUCTURE ONLY.

Independent CPU restatement (PyTorch float64, automatic differentiation) of the NLP that
``awebox/pmpc.py`` hands to IPOPT for ``examples/mpc_closed_loop.py`` (SURVEY.md section 8 row
a37, config 5).  Only ``tests/`` and ``bench.py``'s CPU leg may import it; the product
(``awebox_amd``) never does.

Parity status: CasADi 3.6.4 cannot run here, so this restatement is pinned
by the reference's analytic tests that cover its pieces -- the Lagrangian / holonomic / momentum
path it shares with the AP2 oracle (pendulum and pseudo-Atwood residuals,
``test/units/test_model.py:438-832``, restated in ``tests/test_oracle_known_answers.py``) -- and by
restated geometric properties of the 3-DOF force model (``tests/test_mpc.py``); "parity partially
pinned".

What is restated (file:line of the reference):
  * node variables: x = [q10, dq10, coeff10, l_t, dl_t, ddl_t], xdot = d<x>, u = [f_fict10,
    dcoeff10, dddl_t], z = [lambda10], theta = [diam_t, t_f] (system.py:42-230);
  * Lagrangian translational dynamics of the kite node with the tether kinetic/potential energy,
    holonomic constraint with Baumgarte stabilisation and open-system momentum correction
    (lagr_dyn.py:39-204, energy.py:43-144, holonomics.py:17-123, 267-312, mass.py:62-93), taken by
    automatic differentiation of L w.r.t. the *scaled* coordinates and a JVP ``time_derivative``
    over the (variable, derivative) pairs of tools.py:13-73;
  * 3-DOF aerodynamics: planar DCM from the tether and apparent wind, roll about the apparent wind,
    CL = coeff[0], CD = |CX0| + CL^2 / (pi AR) (three_dof_kite.py:98-199);
  * 'multi' tether drag, 5 elements, constant cd (element.py:60-104, segment.py:38-65);
  * log wind with smooth_abs(z, 1) (wind.py:184-208), ISA density (atmosphere.py:42-78);
  * trivial kinematics (lagr_dyn.py:141-169), tether stress and acceleration inequalities
    (dynamics.py:627-652, 706-790);
  * the MPC NLP: initial conditions x[0] - p.x0 (operation.py:303-326), shooting / path /
    collocation / continuity rows (constraints.py:210-373, collocation.py:202-336), and the
    tracking objective (pmpc.py:304-358).
"""
from __future__ import annotations

import math

import numpy as np
import torch
from torch.func import grad, hessian, jacfwd, jvp, vmap

from oracle.ap2_oracle import Ap2Oracle, cross, norm, smooth_abs, smooth_norm, smooth_sqrt

torch.set_default_dtype(torch.float64)

_X = [("q10", 3), ("dq10", 3), ("coeff10", 2), ("l_t", 1), ("dl_t", 1), ("ddl_t", 1)]
_XD = [("d" + n, s) for n, s in _X]
_U = [("f_fict10", 3), ("dcoeff10", 2), ("dddl_t", 1)]
_Z = [("lambda10", 1)]
_TH = [("diam_t", 1), ("t_f", 1)]
NX, NU, NZ = 11, 6, 1


def _build_index():
    idx, pos = {}, 0
    for vt, ents in (("x", _X), ("xdot", _XD), ("u", _U), ("z", _Z), ("theta", _TH)):
        for n, s in ents:
            idx[(vt, n)] = slice(pos, pos + s)
            pos += s
    return idx, pos


IDX, NW = _build_index()

# time_derivative pairs: for each xdot name 'd<v>', v and the first non-xdot container holding
# 'd<v>' (struct_op.get_variable_type prefers x/u/z/theta, struct_operations.py:737-761)
_PAIRS = [(("x", "q10"), ("x", "dq10")), (("x", "dq10"), ("xdot", "ddq10")),
          (("x", "coeff10"), ("u", "dcoeff10")), (("x", "l_t"), ("x", "dl_t")),
          (("x", "dl_t"), ("x", "ddl_t")), (("x", "ddl_t"), ("u", "dddl_t"))]

# trivial kinematics: sorted xdot names that also live in x (else u) (lagr_dyn.py:141-169)
_TRIVIAL = [("dcoeff10", ("u", "dcoeff10")), ("dddl_t", ("u", "dddl_t")), ("ddl_t", ("x", "ddl_t")),
            ("dl_t", ("x", "dl_t")), ("dq10", ("x", "dq10"))]


def get(w, vt, name):
    return w[IDX[(vt, name)]]


class Kite3Oracle:
    """consts: dict name -> value (awebox_amd.kite3.CONST_NAMES); scaling [31]."""

    def __init__(self, scaling, consts: dict, n_k=20, d=4, ts=0.1):
        self.s = torch.as_tensor(np.asarray(scaling, dtype=np.float64))
        self.c = dict(consts)
        self.n_k, self.d, self.ts = n_k, d, ts
        self.tau, self.C, self.D, self.w = Ap2Oracle._radau(d)

    # ---------------------------------------------------------------- environment --------
    def density(self, zz):
        c = self.c
        t = c["t_ref"] - c["gamma_air"] * zz
        return c["rho_ref"] * (t / c["t_ref"]) ** (c["g"] / c["gamma_air"] / c["r_air"] - 1.0)

    def wind_speed(self, zz, u_ref):
        c = self.c
        z_cropped = smooth_abs(zz, 1.0)
        return u_ref * torch.log10(z_cropped / c["z0_air"]) / math.log10(c["z_ref"] / c["z0_air"])

    def wind_velocity(self, zz, u_ref):
        u = self.wind_speed(zz, u_ref)
        z = torch.zeros((), dtype=u.dtype)
        return torch.stack([u, z, z])

    # ---------------------------------------------------------------- time derivative ----
    def tangent(self, w_sc):
        s = self.s
        t = torch.zeros(NW, dtype=w_sc.dtype)
        for (vt, vn), (dt, dn) in _PAIRS:
            iv, idv = IDX[(vt, vn)], IDX[(dt, dn)]
            t = t.index_put((torch.arange(iv.start, iv.stop),), s[idv] / s[iv] * w_sc[idv])
        return t

    def time_derivative(self, f):
        def df(w_sc, *args):
            _, out = jvp(lambda ww: f(ww, *args), (w_sc,), (self.tangent(w_sc),))
            return out
        return df

    # ---------------------------------------------------------------- model pieces -------
    def si(self, w_sc):
        return w_sc * self.s

    def seg_mass(self, w_sc):
        w = self.si(w_sc)
        diam = get(w, "theta", "diam_t")[0]
        return math.pi * (diam / 2.) ** 2. * self.c["rho_tether"] * norm(get(w, "x", "q10"))

    def holonomic(self, w_sc):
        w = self.si(w_sc)
        q = get(w, "x", "q10")
        l_t = get(w, "x", "l_t")[0]
        return 0.5 * (torch.dot(q, q) - l_t ** 2.0)

    def lagrangian(self, w_sc):
        w = self.si(w_sc)
        q, dq = get(w, "x", "q10"), get(w, "x", "dq10")
        m_t = self.seg_mass(w_sc)
        ehat = q / norm(q)
        dq_parent = torch.dot(dq, ehat) * ehat
        e_kin = 0.5 * m_t / 3 * (torch.dot(dq, dq) + torch.dot(dq_parent, dq_parent) + torch.dot(dq, dq_parent))
        e_kin = e_kin + 0.5 * self.c["m_k"] * torch.dot(dq, dq)
        g = self.c["g"]
        e_pot = g * m_t * (q[2] / 2.) + g * self.c["m_k"] * q[2]
        lam = get(w, "z", "lambda10")[0]
        return e_kin - e_pot - lam * self.holonomic(w_sc)

    def element_drag(self, q_up, q_lo, dq_up, dq_lo, diam, u_ref):
        zz = ((q_up + q_lo) / 2.)[2]
        ua = self.wind_velocity(zz, u_ref) - (dq_up + dq_lo) / 2.
        eps = 1.e-6
        ua_norm = smooth_norm(ua, eps)
        ehat = ua / smooth_norm(ua, eps)
        tether = q_up - q_lo
        l_par = torch.dot(tether, ehat)
        l_perp = smooth_sqrt(torch.dot(tether, tether) - l_par ** 2., eps ** 2.)
        return self.c["cd_tether"] * 0.5 * self.density(zz) * ua_norm * diam * l_perp * ua

    def tether_drag(self, w, u_ref):
        q, dq = get(w, "x", "q10"), get(w, "x", "dq10")
        diam = get(w, "theta", "diam_t")[0]
        n = int(self.c["n_elements"])
        ds = 1.0 / n
        s_grid = np.linspace(0.5 * ds, 1 - 0.5 * ds, n)
        total = torch.zeros(3, dtype=q.dtype)
        for e in range(n):
            lo, up = e / n, (e + 1) / n
            total = total + s_grid[e] * self.element_drag(q * up, q * lo, dq * up, dq * lo, diam, u_ref)
        return total

    def aero(self, w, u_ref):
        """three_dof_kite.get_force_from_u_sym_in_earth_frame / get_kite_dcm (:98-199)."""
        q, dq = get(w, "x", "q10"), get(w, "x", "dq10")
        coeff = get(w, "x", "coeff10")
        u = self.wind_velocity(q[2], u_ref) - dq
        v = cross(q, u)
        ww = cross(u, v)
        vhat = v / smooth_norm(v)
        what = ww / smooth_norm(ww)
        psi = coeff[1]
        ehat3 = torch.cos(psi) * what - torch.sin(psi) * vhat
        rho = self.density(q[2])
        CL = coeff[0]
        CD = self.c["cd0"] + CL ** 2 / (math.pi * self.c["ar"])
        s_ref = self.c["s_ref"]
        f_lift = CL * 0.5 * rho * torch.dot(u, u) * s_ref * ehat3
        f_drag = CD * 0.5 * rho * norm(u) * s_ref * u
        return f_lift + f_drag

    # ---------------------------------------------------------------- node residuals -----
    def node(self, w_sc, gamma, u_ref):
        s, c = self.s, self.c
        w = self.si(w_sc)
        q, dq = get(w, "x", "q10"), get(w, "x", "dq10")
        iq, idq = IDX[("x", "q10")], IDX[("x", "dq10")]

        def dL(w_):
            return grad(self.lagrangian)(w_)

        dldqdot_dt = self.time_derivative(lambda ww: dL(ww)[idq])(w_sc)
        lhs = dldqdot_dt / s[idq] - dL(w_sc)[iq] / s[iq]
        mass_flow = self.time_derivative(self.seg_mass)(w_sc)
        F = self.tether_drag(w, u_ref) + (gamma * get(w, "u", "f_fict10") + self.aero(w, u_ref))
        rhs = F + mass_flow * dq
        scaling_mass = math.pi * (c["scaling_diam"] / 2.) ** 2. * c["rho_tether"] * c["scaling_length"]
        force_scaling = (scaling_mass / 2. + c["m_k"]) * c["g_scaling"] * 10.
        trans = (lhs - rhs) / force_scaling

        g0 = self.holonomic(w_sc)
        g1 = self.time_derivative(self.holonomic)(w_sc)
        g2 = self.time_derivative(self.time_derivative(self.holonomic))(w_sc)
        kap = c["kappa"]
        hol = ((g2 + 2. * kap * g1 + kap ** 2 * g0) / (kap ** 2 * c["scaling_length"] * c["q_scaling_mean"])).reshape(1)

        triv = []
        for xd, (ut, un) in _TRIVIAL:
            mean = (s[IDX[(ut, un)]] * s[IDX[("xdot", xd)]]) ** 0.5
            triv.append((get(w, "xdot", xd) - get(w, ut, un)) / mean)
        eq = torch.cat([trans, hol] + triv)

        lam = get(w, "z", "lambda10")[0]
        diam = get(w, "theta", "diam_t")[0]
        area = math.pi * (diam / 2.) ** 2.
        char_tension = math.sqrt((c["lambda_scaling"] * c["scaling_length"]) ** 2 + 1e-16)
        stress = (lam * norm(q) - area * c["stress_max"]) / char_tension
        acc = get(w, "xdot", "ddq10")
        accel = torch.dot(acc, acc) / c["acc_max"] ** 2 - 1.
        return eq, torch.stack([stress, accel])

    # ---------------------------------------------------------------- NLP -----------------
    def interval_rows(self, wloc, u_ref):
        """g rows of interval k from wloc = [theta, phi, x[k], u[k], xdot[k], z[k], coll[k,:], x[k+1]]."""
        d = self.d
        theta, phi = wloc[0:2], wloc[2:9]
        o = 9
        xk = wloc[o:o + NX]; o += NX
        uk = wloc[o:o + NU]; o += NU
        xdk = wloc[o:o + NX]; o += NX
        zk = wloc[o:o + NZ]; o += NZ
        cx, cz = [], []
        for _ in range(d):
            cx.append(wloc[o:o + NX]); o += NX
            cz.append(wloc[o:o + NZ]); o += NZ
        xk1 = wloc[o:o + NX]
        gamma, tf = phi[0], theta[1]
        h = 1.0 / self.n_k
        C = torch.as_tensor(self.C)
        X = [xk] + cx
        W = [torch.cat([xk, xdk, uk, zk, theta])]
        for j in range(d):
            xp = sum(C[r, j + 1] * X[r] for r in range(d + 1))
            W.append(torch.cat([cx[j], xp / h / tf, uk, cz[j], theta]))
        eq, ineq = vmap(self.node, in_dims=(0, None, None))(torch.stack(W), gamma, u_ref)
        Dc = torch.as_tensor(self.D)
        cont = xk1 - sum(Dc[r] * X[r] for r in range(d + 1))
        return torch.cat([eq[0], ineq[0]] + [eq[j + 1] for j in range(d)] + [cont])

    def local_index(self, lay, k):
        base = lay.v_intervals + k * lay.interval_stride
        return np.concatenate([np.arange(0, 9), np.arange(base, base + lay.interval_stride + NX)])

    def nlp_g(self, V, p, lay):
        V, p = torch.as_tensor(V), torch.as_tensor(p)
        u_ref = p[lay.p_u_ref]
        init = V[torch.as_tensor(lay.x(0))] - p[lay.p_x0:lay.p_x0 + NX]
        locs = torch.stack([V[torch.as_tensor(self.local_index(lay, k))] for k in range(self.n_k)])
        rows = vmap(self.interval_rows, in_dims=(0, None))(locs, u_ref)
        return torch.cat([init, rows.reshape(-1)])

    def nlp_jac_g(self, V, p, lay):
        """J_g as a scipy CSC matrix (exact zeros dropped)."""
        import scipy.sparse as sp
        V, p = torch.as_tensor(V), torch.as_tensor(p)
        u_ref = p[lay.p_u_ref]
        idx = np.stack([self.local_index(lay, k) for k in range(self.n_k)])
        J = vmap(jacfwd(self.interval_rows), in_dims=(0, None))(V[torch.as_tensor(idx)], u_ref).numpy()
        rows, cols, vals = [np.arange(NX)], [lay.x(0)], [np.ones(NX)]
        for k in range(self.n_k):
            r, cc = np.nonzero(J[k])
            rows.append(NX + k * lay.rows_per_interval + r)
            cols.append(idx[k][cc])
            vals.append(J[k][r, cc])
        return sp.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                             shape=(lay.n_g, lay.n_v))

    def nlp_f(self, V, p, lay):
        """Tracking cost (pmpc.py:304-358): sum_k sum_j w_j (w - w_ref)^T diag(Q, Z, R) (w - w_ref) / N
        over w = [coll x, coll z, u_k], plus (x_N - ref_N)^T diag(P) (x_N - ref_N)."""
        V, p = torch.as_tensor(V), torch.as_tensor(p)
        ref = p[lay.p_ref:lay.p_ref + lay.n_v]
        Wt = torch.cat([p[lay.p_Q:lay.p_Q + NX], torch.ones(NZ), p[lay.p_R:lay.p_R + NU]])
        f = torch.zeros(())
        for k in range(self.n_k):
            ui = torch.as_tensor(lay.u(k))
            for j in range(self.d):
                ci = torch.as_tensor(np.concatenate([lay.coll_x(k, j), lay.coll_z(k, j)]))
                e = torch.cat([V[ci] - ref[ci], V[ui] - ref[ui]])
                f = f + self.w[j] * torch.dot(e * Wt, e)
        f = f / self.n_k
        xi = torch.as_tensor(lay.x(self.n_k))
        dx = V[xi] - ref[xi]
        return f + torch.dot(dx * p[lay.p_P:lay.p_P + NX], dx)

    def nlp_grad_f(self, V, p, lay):
        V = torch.as_tensor(V)
        return grad(lambda vv: self.nlp_f(vv, p, lay))(V)

    def nlp_hess_l(self, V, p, sigma, lam, lay):
        """Dense Hessian of sigma f + lam^T g (nlp_hess_l): per interval the Hessian of
        lam_k^T rows_k(wloc) by torch.func (the initial-condition rows are linear), scattered into
        V space; plus sigma times the Hessian of the tracking cost."""
        V, p = torch.as_tensor(V), torch.as_tensor(p)
        lam = torch.as_tensor(np.asarray(lam, dtype=np.float64))
        u_ref = p[lay.p_u_ref]
        idx = np.stack([self.local_index(lay, k) for k in range(self.n_k)])
        lk = torch.stack([lam[NX + k * lay.rows_per_interval:NX + (k + 1) * lay.rows_per_interval]
                          for k in range(self.n_k)])

        def lag(wloc, mu):
            return torch.dot(mu, self.interval_rows(wloc, u_ref))
        Hk = vmap(hessian(lag), in_dims=(0, 0))(V[torch.as_tensor(idx)], lk).numpy()
        H = np.zeros((lay.n_v, lay.n_v))
        for k in range(self.n_k):
            H[np.ix_(idx[k], idx[k])] += Hk[k]
        Hf = hessian(lambda vv: self.nlp_f(vv, p, lay))(V).numpy()
        return H + float(sigma) * Hf


def from_constants(k3, lay):
    """Oracle instance from awebox_amd.kite3 constants (values only; the oracle owns its math)."""
    from awebox_amd import kite3 as k3m
    consts = {n: float(k3.consts[i]) for i, n in enumerate(k3m.CONST_NAMES) if not (n.startswith("scaling") and n[7:].isdigit())}
    return Kite3Oracle(k3.scaling, consts, n_k=lay.n_k, d=lay.d, ts=k3.cfg.ts)
