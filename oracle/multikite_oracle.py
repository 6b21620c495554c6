"""CPU ORACLE for the multi-kite collocation evaluator -- TEST INFRASTRUCTURE ONLY.

Independent CPU restatement of the reference's model + NLP assembly for tree architectures with
a main tether (node 1) and kites either on it ({1: 0}) or on secondary tethers below the layer
node 1 ({1: 0, 2: 1, 3: 1}: examples/dual_kites_power_curve.py).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it.

Parity status: like ``ap2_oracle.py`` the math is CasADi's in the reference, which cannot run
here.  This restatement is pinned by (i) reproducing ``ap2_oracle`` --
itself pinned by the reference's analytic known-answer tests -- bit for bit in structure and to
rounding in value at the architecture {1: 0} (tests/test_dual.py), and (ii) the reference's own
Lagrangian pendulum/Atwood construction, which is what the generic segment Lagrangian below
generalises.  For the dual-kite rows no reference output exists: "parity partially pinned".

Design: the whole Lagrangian ``L = sum_segments (T_seg + T_kite - V_seg - V_kite - lambda c)`` is
built per tether segment exactly as ``lagr_dyn_dir/energy.py:43-144`` and
``holonomics.py:204-264`` do, and differentiated with ``torch.func``: translational equations by
``grad`` w.r.t. the scaled generalised coordinates and ``time_derivative`` as a JVP over the
(variable, derivative) pairs (``lagr_dyn_dir/tools.py:13-73``).  The HIP kernel instead uses
hand-derived per-segment closed forms, so the two are independent.
"""
from __future__ import annotations

import itertools
import math

import numpy as np
import torch
from torch.func import grad, jacfwd, jvp, vmap

from .ap2_oracle import cross, norm, reshape33, skew, smooth_abs, smooth_norm, smooth_sqrt, vec_col

torch.set_default_dtype(torch.float64)


class Arch:
    """awebox/mdl/architecture.py:33-120."""

    def __init__(self, parent_map):
        self.parent_map = dict(parent_map)
        self.number_of_nodes = len(self.parent_map) + 1
        parents = set(self.parent_map.values())
        self.kite_nodes = [n for n in self.parent_map if n not in parents]
        self.children = {}
        for n, p in self.parent_map.items():
            self.children.setdefault(p, []).append(n)
        self.siblings = {}
        for k in self.kite_nodes:
            self.siblings.setdefault(self.parent_map[k], []).append(k)

    def lab(self, n):
        return f"{n}{self.parent_map[n]}"


def variables(arch: Arch):
    """system.py:42-230 (kite_dof 6, surface_control 1, lift_mode, ddl_t)."""
    X, U, Z = [], [], []
    for n in range(1, arch.number_of_nodes):
        lb = arch.lab(n)
        if n in arch.kite_nodes:
            X += [(f"q{lb}", 3), (f"dq{lb}", 3), (f"omega{lb}", 3), (f"r{lb}", 9), (f"delta{lb}", 3)]
            U += [(f"f_fict{lb}", 3), (f"m_fict{lb}", 3), (f"ddelta{lb}", 3)]
        else:
            X += [(f"q{lb}", 3), (f"dq{lb}", 3)]
        Z.append((f"lambda{lb}", 1))
    X += [("l_t", 1), ("dl_t", 1)]
    U += [("ddl_t", 1)]
    TH = [("diam_t", 1), ("t_f", 1)]
    if arch.number_of_nodes - len(arch.kite_nodes) > 1:
        TH += [("l_s", 1), ("diam_s", 1)]
    return X, [("d" + n, s) for n, s in X], U, Z, TH


class MultiKiteOracle:
    """Restated multi-kite model + collocation NLP (radau, zoh, phase fix simple/single_reelout).

    ``scaling`` [nw] and ``consts`` (name -> float, ``awebox_amd.dual.CONST_NAMES``) are produced
    by the host option pipeline (``awebox_amd/dual.py``, checked in tests/test_dual.py).
    """

    def __init__(self, parent_map, scaling, consts: dict, sd_len, n_k, d, single_reelout, nk_reelout):
        self.arch = Arch(parent_map)
        self.X, self.XD, self.U, self.Z, self.TH = variables(self.arch)
        self.idx = {}
        pos = 0
        for vt, ents in (("x", self.X), ("xdot", self.XD), ("u", self.U), ("z", self.Z), ("theta", self.TH)):
            for n, s in ents:
                self.idx[(vt, n)] = slice(pos, pos + s)
                pos += s
        self.nw = pos
        self.nx = sum(s for _, s in self.X)
        self.nu = sum(s for _, s in self.U)
        self.nz = sum(s for _, s in self.Z)
        self.nth = sum(s for _, s in self.TH)
        self.s = torch.as_tensor(np.asarray(scaling, dtype=np.float64))
        self.c = dict(consts)
        self.sd_len = np.asarray(sd_len, dtype=np.int64).reshape(6, 9)
        self.n_k, self.d = n_k, d
        self.single_reelout, self.nk_reelout = single_reelout, nk_reelout
        from .ap2_oracle import Ap2Oracle
        self.tau, self.C, self.D, self.w = Ap2Oracle._radau(d)
        # time_derivative pairs: every xdot name 'd<v>' with v and the first container holding
        # 'd<v>' among x, u, z, theta, else xdot (tools.py:13-73, struct_operations.py:737-761)
        names = {vt: {n for n, _ in ents} for vt, ents in
                 (("x", self.X), ("u", self.U), ("z", self.Z), ("theta", self.TH))}
        self.pairs = []
        for dn, _ in self.XD:
            v = dn[1:]
            vt = next(t for t in ("x", "u", "z", "theta") if v in names[t])
            dt = next((t for t in ("x", "u", "z", "theta") if dn in names[t]), "xdot")
            self.pairs.append(((vt, v), (dt, dn)))
        self.trivial = sorted(dn for dn, _ in self.XD if dn in names["x"] or dn in names["u"])

    # ------------------------------------------------------------------ helpers --------------
    def get(self, w, vt, name):
        return w[self.idx[(vt, name)]]

    def si(self, w_sc):
        return w_sc * self.s

    @staticmethod
    def density(th, zz):
        t = th["atmosphere.t_ref"] - th["atmosphere.gamma_air"] * zz
        return th["atmosphere.rho_ref"] * (t / th["atmosphere.t_ref"]) ** (
            th["atmosphere.g"] / th["atmosphere.gamma_air"] / th["atmosphere.r"] - 1.0)

    @staticmethod
    def wind_velocity(th, zz):
        z_cropped = smooth_abs(zz, 1.0)
        u = th["wind.u_ref"] * (z_cropped / th["wind.z_ref"]) ** th["wind.power_wind.exp_ref"]
        z = torch.zeros((), dtype=u.dtype)
        return torch.stack([u, z, z])

    def tangent(self, w_sc):
        """t(w) with time_derivative(f) = J_f(w) t(w) (tools.py:13-73), incl. the DCM term."""
        s = self.s
        seg = {}
        for (vt, vn), (dt, dn) in self.pairs:
            iv, idv = self.idx[(vt, vn)], self.idx[(dt, dn)]
            seg[(vt, vn)] = s[idv] / s[iv] * w_sc[idv]
        for k in self.arch.kite_nodes:
            lb = self.arch.lab(k)
            r = reshape33(self.get(w_sc, "x", f"r{lb}"))
            om = self.get(w_sc, "x", f"omega{lb}")
            seg[("x", f"r{lb}")] = seg[("x", f"r{lb}")] + vec_col(skew(om) @ torch.linalg.inv(r.T))
        parts = []
        for key, sl in sorted(self.idx.items(), key=lambda kv: kv[1].start):
            parts.append(seg[key] if key in seg else torch.zeros(sl.stop - sl.start, dtype=w_sc.dtype))
        return torch.cat(parts)

    def time_derivative(self, f):
        def df(w_sc):
            _, out = jvp(f, (w_sc,), (self.tangent(w_sc),))
            return out
        return df

    # ------------------------------------------------------------------ segments -------------
    def segment(self, w, n):
        """(q_upper, q_lower, dq_upper, dq_lower, diam, length symbol value, main?) of the tether
        segment below node n (element.py:105-130, tether_aero.py:178-267)."""
        a = self.arch
        q, dq = self.get(w, "x", f"q{a.lab(n)}"), self.get(w, "x", f"dq{a.lab(n)}")
        p = a.parent_map[n]
        if p == 0:
            z3 = torch.zeros(3, dtype=q.dtype)
            return q, z3, dq, z3, self.get(w, "theta", "diam_t")[0], self.get(w, "x", "l_t")[0], True
        qp, dqp = self.get(w, "x", f"q{a.lab(p)}"), self.get(w, "x", f"dq{a.lab(p)}")
        return q, qp, dq, dqp, self.get(w, "theta", "diam_s")[0], self.get(w, "theta", "l_s")[0], False

    def seg_mass(self, w_sc, th, n):
        w = self.si(w_sc)
        qu, ql, _, _, diam, _, _ = self.segment(w, n)
        return math.pi * (diam / 2.) ** 2. * th["tether.rho"] * norm(qu - ql)

    def holonomic(self, w_sc, n):
        w = self.si(w_sc)
        qu, ql, _, _, _, length, _ = self.segment(w, n)
        return 0.5 * (torch.dot(qu - ql, qu - ql) - length ** 2.0)

    def lagrangian(self, w_sc, th):
        """energy.py:43-144 (kinetic/potential per node), holonomics.py:17-123 (W = sum lambda c)."""
        a = self.arch
        w = self.si(w_sc)
        g = th["atmosphere.g"]
        m_k = th["geometry.m_k"]
        J = reshape33(th["geometry.j"])
        lag = torch.zeros((), dtype=w.dtype)
        for n in range(1, a.number_of_nodes):
            qu, ql, dqu, dql, _, _, main = self.segment(w, n)
            m_seg = self.seg_mass(w_sc, th, n)
            if main:
                ehat = qu / norm(qu)
                dq_parent = torch.dot(self.get(w, "x", "dq10"), ehat) * ehat   # get_reelout_speed
            else:
                dq_parent = dql
            e_kin = 0.5 * m_seg / 3 * (torch.dot(dqu, dqu) + torch.dot(dq_parent, dq_parent)
                                      + torch.dot(dqu, dq_parent))
            e_pot = g * m_seg * ((qu + ql) / 2.)[2]
            if n in a.kite_nodes:
                om = self.get(w, "x", f"omega{a.lab(n)}")
                e_kin = e_kin + 0.5 * m_k * torch.dot(dqu, dqu) + 0.5 * om @ J @ om
                e_pot = e_pot + g * m_k * qu[2]
            lam = self.get(w, "z", f"lambda{a.lab(n)}")[0]
            lag = lag + e_kin - e_pot - lam * self.holonomic(w_sc, n)
        return lag

    def element_drag(self, q_upper, q_lower, dq_upper, dq_lower, diam, th):
        # element.get_element_drag_fun (element.py:60-104); cd 'constant'
        q_average = (q_upper + q_lower) / 2.
        zz = q_average[2]
        ua = self.wind_velocity(th, zz) - (dq_upper + dq_lower) / 2.
        eps = 1.e-6
        ua_norm = smooth_norm(ua, eps)
        ehat_ua = ua / smooth_norm(ua, eps)
        tether = q_upper - q_lower
        length_par = torch.dot(tether, ehat_ua)
        length_perp = smooth_sqrt(torch.dot(tether, tether) - length_par ** 2., eps ** 2.)
        return th["tether.cd"] * 0.5 * self.density(th, zz) * ua_norm * diam * length_perp * ua

    def segment_forces(self, w, th, n):
        """(lower, upper) 'multi' drag shares of the segment below n (segment.py:38-65)."""
        qt, qb, dqt, dqb, diam, _, _ = self.segment(w, n)
        ne = int(self.c["n_elements"])
        ds = 1.0 / ne
        s_grid = np.linspace(0.5 * ds, 1 - 0.5 * ds, ne)
        up = torch.zeros(3, dtype=w.dtype)
        lo = torch.zeros(3, dtype=w.dtype)
        for e in range(ne):
            lphi, uphi = float(e) / float(ne), float(e + 1) / float(ne)
            drag = self.element_drag(qb + (qt - qb) * uphi, qb + (qt - qb) * lphi,
                                     dqb + (dqt - dqb) * uphi, dqb + (dqt - dqb) * lphi, diam, th)
            up = up + s_grid[e] * drag
            lo = lo + (1 - s_grid[e]) * drag
        return lo, up

    def aero(self, w, th, k):
        """6-DOF stability-derivative force/moment of kite k (six_dof_kite.py:165-201)."""
        lb = self.arch.lab(k)
        q, dq = self.get(w, "x", f"q{lb}"), self.get(w, "x", f"dq{lb}")
        omega = self.get(w, "x", f"omega{lb}")
        R = reshape33(self.get(w, "x", f"r{lb}"))
        delta = self.get(w, "x", f"delta{lb}")
        u = self.wind_velocity(th, q[2]) - dq
        rho = self.density(th, q[2])
        e1, e2, e3 = R[:, 0], R[:, 1], R[:, 2]
        alpha = torch.dot(u, e3) / smooth_abs(torch.dot(u, e1))
        beta = torch.dot(u, e2) / smooth_abs(torch.dot(u, e1))
        airspeed = norm(u)
        om_hat = omega * torch.tensor([-1., 1., -1.]) / (2. * airspeed)
        b, cr = th["geometry.b_ref"], th["geometry.c_ref"]
        inputs = [torch.ones((), dtype=u.dtype), alpha, -beta, om_hat[0] * b, om_hat[1] * cr, om_hat[2] * b,
                  delta[0], delta[1], delta[2]]
        sd = th["aero.stab_derivs"].reshape(6, 9, 3)
        coeffs = []
        for ci in range(6):
            acc = torch.zeros((), dtype=u.dtype)
            for ii in range(9):
                nl = int(self.sd_len[ci, ii])
                if nl == 0:
                    continue
                stack = torch.stack([inputs[ii] * alpha ** l for l in range(nl)])
                weight = th["aero.moment_factor"] if (ci >= 3 and ii >= 6) else 1.0
                acc = acc + weight * torch.dot(sd[ci, ii, :nl], stack)
            coeffs.append(acc)
        dyn = 0.5 * rho * torch.dot(u, u)
        s_ref = th["geometry.s_ref"]
        flip = torch.tensor([-1., 1., -1.])
        F_earth = R @ (flip * (torch.stack(coeffs[:3]) * dyn * s_ref))
        M_body = flip * (dyn * s_ref * (torch.stack([b, cr, b]) * torch.stack(coeffs[3:])))
        return dict(u=u, beta=beta, airspeed=airspeed, F_earth=F_earth, M_body=M_body, R=R, q=q)

    @staticmethod
    def unskew(A):
        return 0.5 * torch.stack([A[2, 1] - A[1, 2], A[0, 2] - A[2, 0], A[1, 0] - A[0, 1]])

    # ------------------------------------------------------------------ node residuals -------
    def node(self, w_sc, gamma, th):
        """Model eq [n_eq], ineq [n_ineq], power integrand, kite side slips at one node."""
        a, s, c = self.arch, self.s, self.c
        w = self.si(w_sc)
        nodes = list(range(1, a.number_of_nodes))
        rho_t = th["tether.rho"]

        def scaling_length(n):
            return c["scaling_length_t"] if a.parent_map[n] == 0 else c["scaling_length_s"]

        def scaling_mass(n):
            diam = c["scaling_diam_t"] if a.parent_map[n] == 0 else c["scaling_diam_s"]
            return math.pi * (diam / 2.) ** 2. * rho_t * scaling_length(n)

        aero = {k: self.aero(w, th, k) for k in a.kite_nodes}
        # node forces (forces.py:47-80, tether_aero.py:73-95): upper share to the node, lower
        # share to the parent (dropped at the ground)
        F = {n: torch.zeros(3, dtype=w.dtype) for n in nodes}
        for n in nodes:
            lo, up = self.segment_forces(w, th, n)
            if a.parent_map[n] != 0:
                F[a.parent_map[n]] = F[a.parent_map[n]] + lo
            F[n] = F[n] + up
        for k in a.kite_nodes:
            F[k] = F[k] + (gamma * self.get(w, "u", f"f_fict{a.lab(k)}") + aero[k]["F_earth"])

        dL = lambda ww: grad(lambda x: self.lagrangian(x, th))(ww)  # noqa: E731
        trans = []
        mass_flow = self.time_derivative(lambda ww: self.seg_mass(ww, th, 1))(w_sc)
        for n in nodes:
            iq, idq = self.idx[("x", f"q{a.lab(n)}")], self.idx[("x", f"dq{a.lab(n)}")]
            ddt = self.time_derivative(lambda ww, idq=idq: dL(ww)[idq])(w_sc)
            lhs = ddt / s[idq] - dL(w_sc)[iq] / s[iq]
            rhs = F[n]
            if n == 1:                                           # lagr_dyn.py:174-204
                rhs = rhs + mass_flow * self.get(w, "x", "dq10")
            node_mass = scaling_mass(n) / 2.                     # mass.py:62-93
            for ch in a.children.get(n, []):
                node_mass = node_mass + scaling_mass(ch) / 2.
            if n in a.kite_nodes:
                node_mass = node_mass + th["geometry.m_k"]
            trans.append((lhs - rhs) / (node_mass * c["g_scaling"] * 10.))

        kappa = th["tether.kappa"]
        hol = []
        for n in nodes:                                          # holonomics.py:17-123, 267-312
            cf = lambda ww, n=n: self.holonomic(ww, n)  # noqa: E731
            g0 = cf(w_sc)
            g1 = self.time_derivative(cf)(w_sc)
            g2 = self.time_derivative(self.time_derivative(cf))(w_sc)
            sq = s[self.idx[("x", f"q{a.lab(n)}")]]
            scale = kappa ** 2. * (scaling_length(n) * sq.mean())
            hol.append(((g2 + 2. * kappa * g1 + kappa ** 2. * g0) / scale).reshape(1))

        work = lambda ww: sum(self.si(ww)[self.idx[("z", f"lambda{a.lab(n)}")]][0] * self.holonomic(ww, n)  # noqa
                              for n in nodes)
        dW = grad(work)(w_sc)
        J = reshape33(th["geometry.j"])
        rot = []
        for k in a.kite_nodes:                                   # lagr_dyn.py:207-254
            lb = a.lab(k)
            om = self.get(w, "x", f"omega{lb}")
            R = aero[k]["R"]
            dW_dr = dW[self.idx[("x", f"r{lb}")]]
            n_tether = 2. * self.unskew(R.T @ reshape33(dW_dr))
            M = gamma * self.get(w, "u", f"m_fict{lb}") + aero[k]["M_body"]
            od = M - (J @ self.get(w, "xdot", f"domega{lb}") + cross(om, J @ om) + n_tether)
            rot.append(od / c["m_aero_scaling"])
            ortho = th["kappa_r"] / 2. * (torch.eye(3) - R.T @ R)
            rot.append(vec_col(reshape33(self.get(w, "xdot", f"dr{lb}")) - R @ (ortho + skew(om))))

        triv = []
        xs = {n for n, _ in self.X}
        for dn in self.trivial:
            ut = "x" if dn in xs else "u"
            diff = self.get(w, "xdot", dn) - self.get(w, ut, dn)
            mean = (s[self.idx[(ut, dn)]] * s[self.idx[("xdot", dn)]]) ** 0.5
            triv.append(diff / mean)
        eq = torch.cat(trans + hol + rot + triv)

        # inequalities (dynamics.py:457-486, 655-821, 1022-1117)
        ineq = []
        f_lim = th["model_bounds.tether_force_limits"]
        for k in a.kite_nodes:
            qu, ql, _, _, _, _, _ = self.segment(w, k)
            tension = self.get(w, "z", f"lambda{a.lab(k)}")[0] * norm(qu - ql)
            fs = s[self.idx[("z", f"lambda{a.lab(k)}")]][0] * scaling_length(k)
            ineq += [(tension - f_lim[1]) / fs, (f_lim[0] - tension) / fs]
        a_lim = th["model_bounds.airspeed_limits"]
        for k in a.kite_nodes:
            sp = aero[k]["airspeed"]
            ineq += [(sp - a_lim[1]) / th["wind.u_ref"], (a_lim[0] - sp) / th["wind.u_ref"]]
        tight, aref = c["aero_tightness"], c["airspeed_ref"]
        sabs = lambda v: math.sqrt(v ** 2 + 1e-16)  # noqa: E731
        for k in a.kite_nodes:
            u, R = aero[k]["u"], aero[k]["R"]
            e1, e2, e3 = R[:, 0], R[:, 1], R[:, 2]
            amax, amin, bmax, bmin = c["alpha_max"], c["alpha_min"], c["beta_max"], c["beta_min"]
            ineq += [(torch.dot(u, e3) - torch.dot(u, e1) * amax) * tight / aref / sabs(amax),
                     (-torch.dot(u, e3) + torch.dot(u, e1) * amin) * tight / aref / sabs(amin),
                     (torch.dot(u, e2) - torch.dot(u, e1) * bmax) * tight / aref / sabs(bmax),
                     (-torch.dot(u, e2) + torch.dot(u, e1) * bmin) * tight / aref / sabs(bmin)]
        for ka, kb in itertools.combinations(a.kite_nodes, 2):
            dist = self.get(w, "x", f"q{a.lab(ka)}") - self.get(w, "x", f"q{a.lab(kb)}")
            ineq.append(1 - torch.dot(dist, dist) / c["anticollision_dist_min"] ** 2)
        gmax = th["model_bounds.rot_angles"][2]
        for k in a.kite_nodes:
            qu, ql, _, _, _, _, _ = self.segment(w, k)
            qh = qu - ql
            R = aero[k]["R"]
            scale = c["scaling_length_t"] if k == 1 else c["scaling_length_s"]
            ineq.append(-1. * (torch.dot(qh, R[:, 2]) - torch.cos(gmax) * norm(qh)) / scale)
        power = (self.get(w, "z", "lambda10")[0] * self.get(w, "x", "l_t")[0] * self.get(w, "x", "dl_t")[0]
                 / c["energy_scaling"])
        betas = torch.stack([aero[k]["beta"] for k in a.kite_nodes])
        return eq, torch.stack(ineq), power, betas

    # ------------------------------------------------------------------ NLP assembly ---------
    def interval_split(self, wloc, n_theta):
        d, nx, nu, nz = self.d, self.nx, self.nu, self.nz
        o = n_theta + 7
        xk = wloc[o:o + nx]; o += nx
        uk = wloc[o:o + nu]; o += nu
        xdk = wloc[o:o + nx]; o += nx
        zk = wloc[o:o + nz]; o += nz
        cx, cz = [], []
        for _ in range(d):
            cx.append(wloc[o:o + nx]); o += nx
            cz.append(wloc[o:o + nz]); o += nz
        return xk, uk, xdk, zk, cx, cz, wloc[o:o + nx]

    def node_theta(self, theta_v, phase):
        """Node theta from V.theta (struct_op.get_V_theta): t_f of the interval's phase."""
        if not self.single_reelout:
            return theta_v
        tf = torch.where(phase == 0, theta_v[1], theta_v[2])
        return torch.cat([theta_v[0:1], tf.reshape(1), theta_v[3:]])

    def interval_rows(self, wloc, phase, th):
        """g rows of one interval (constraints.py:210-373) from its local V slice."""
        d = self.d
        nth_v = self.nth + (1 if self.single_reelout else 0)
        theta = self.node_theta(wloc[:nth_v], phase)
        gamma = wloc[nth_v]
        xk, uk, xdk, zk, cx, cz, xk1 = self.interval_split(wloc, nth_v)
        tf = theta[1]
        h = 1.0 / self.n_k
        C = torch.as_tensor(self.C)
        X = [xk] + cx
        W = [torch.cat([xk, xdk, uk, zk, theta])]
        for j in range(d):
            xp = sum(C[r, j + 1] * X[r] for r in range(d + 1))
            W.append(torch.cat([cx[j], xp / h / tf, uk, cz[j], theta]))
        eq, ineq, _, _ = vmap(self.node, in_dims=(0, None, None))(torch.stack(W), gamma, th)
        Dc = torch.as_tensor(self.D)
        cont = xk1 - sum(Dc[r] * X[r] for r in range(d + 1))
        return torch.cat([eq[0], ineq[0]] + [eq[j + 1] for j in range(d)] + [cont])

    def _phases(self):
        return torch.as_tensor([0 if k < self.nk_reelout else 1 for k in range(self.n_k)])

    def nlp_g(self, V, P, lay, th):
        V = torch.as_tensor(V)
        idx = torch.as_tensor(np.stack([lay.local_index(k) for k in range(self.n_k)]))
        rows = vmap(self.interval_rows, in_dims=(0, 0, None))(V[idx], self._phases(), th)
        order = torch.as_tensor(self.periodic_order())
        x0 = V[torch.as_tensor(lay.x(0))]
        xT = V[torch.as_tensor(lay.coll_x(self.n_k - 1, self.d - 1))]
        g = [rows.reshape(-1), x0[order] - xT[order]]
        if self.single_reelout:                                   # constraints.py:148-170
            T = self.time_period(V, lay)
            frac = self.c["phase_fix_reelout"]
            g.append(torch.stack([(T - self.c["tf_ub"]) / frac, (self.c["tf_lb"] - T) / frac]))
        return torch.cat(g)

    def time_period(self, V, lay):
        """ocp_outputs.find_time_period (ocp_outputs.py:118-140)."""
        if not self.single_reelout:
            return V[lay.theta_index("t_f")]
        n = self.n_k
        return V[lay.theta_index("t_f0")] * self.nk_reelout / n + V[lay.theta_index("t_f1")] * (n - self.nk_reelout) / n

    def periodic_order(self):
        off, pos = {}, 0
        for n, s in self.X:
            off[n] = (pos, s)
            pos += s
        out = []
        for name in sorted(off):
            o, s = off[name]
            out.extend(range(o, o + s))
        return np.array(out)

    def nlp_jac_g(self, V, P, lay, th):
        """J_g as a dense numpy array (test sizes only): interval blocks by jacfwd, the periodic
        and t_f rows by jacfwd of the whole g."""
        V = torch.as_tensor(V)
        return jacfwd(lambda v: self.nlp_g(v, P, lay, th))(V).numpy()

    def nlp_jac_g_sparse(self, V, P, lay, th):
        """J_g as scipy CSC (exact zeros dropped): per-interval forward-mode blocks (vmap of
        jacfwd over the interval slices) plus the periodic and t_f rows -- full sizes."""
        import scipy.sparse as sp
        V = torch.as_tensor(V)
        idx = np.stack([lay.local_index(k) for k in range(self.n_k)])
        J = vmap(jacfwd(self.interval_rows), in_dims=(0, 0, None))(V[torch.as_tensor(idx)], self._phases(), th).numpy()
        R = lay.rows_per_interval
        rows, cols, vals = [], [], []
        for k in range(self.n_k):
            r, c = np.nonzero(J[k])
            rows.append(k * R + r)
            cols.append(idx[k][c])
            vals.append(J[k][r, c])
        order = self.periodic_order()
        pr = lay.g_periodic + np.arange(self.nx)
        rows += [pr, pr]
        cols += [lay.x(0)[order], lay.coll_x(self.n_k - 1, self.d - 1)[order]]
        vals += [np.ones(self.nx), -np.ones(self.nx)]
        if self.single_reelout:
            n, frac = self.n_k, self.c["phase_fix_reelout"]
            a0, a1 = self.nk_reelout / n / frac, (n - self.nk_reelout) / n / frac
            t0, t1 = lay.theta_index("t_f0"), lay.theta_index("t_f1")
            rows.append(np.array([lay.g_tf, lay.g_tf, lay.g_tf + 1, lay.g_tf + 1]))
            cols.append(np.array([t0, t1, t0, t1]))
            vals.append(np.array([a0, a1, -a0, -a1]))
        return sp.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))),
                             shape=(lay.n_g, lay.n_v))

    def nlp_f(self, V, P, lay, th, cost_names, phi_names):
        """Objective (ocp/objective.py:45-544) with per-interval t_f and the phase-fixed period."""
        V = torch.as_tensor(V)
        P = torch.as_tensor(P)
        cost = {n: P[lay.p_cost + i] for i, n in enumerate(cost_names)}
        weights = P[lay.p_weights:lay.p_weights + self.nw]
        vref = P[lay.p_ref:lay.p_ref + lay.n_v]
        c, d, n_k = self.c, self.d, self.n_k
        h = 1.0 / n_k
        C = torch.as_tensor(self.C)
        phi = V[torch.as_tensor(lay.phi())]
        psi, gamma = phi[phi_names.index("psi")], phi[phi_names.index("gamma")]
        cats = {"tracking": [], "xdot_regularisation": [], "u_regularisation": [], "fictitious": [],
                "theta_regularisation": []}
        for (vt, n), sl in self.idx.items():
            if vt in ("x", "z"):
                cat = "tracking"
            elif vt == "xdot":
                cat = "xdot_regularisation"
            elif vt == "u":
                cat = "fictitious" if n.startswith("f_fict") or n.startswith("m_fict") else "u_regularisation"
            else:
                cat = None if n == "t_f" else "theta_regularisation"
            if cat is not None:
                cats[cat].extend(range(sl.start, sl.stop))
        norm_of = {"tracking": c["norm_tracking"], "xdot_regularisation": c["norm_xdot_reg"],
                   "u_regularisation": c["norm_u_reg"], "fictitious": c["norm_fictitious"],
                   "theta_regularisation": c["norm_theta_reg"]}
        w_eff = weights.clone()
        for cat, ids in cats.items():
            it = torch.as_tensor(ids)
            w_eff = w_eff.index_put((it,), weights[it] * cost[cat] / norm_of[cat])
        Wn, Rn, wj, tfs = [], [], [], []
        for k in range(n_k):
            th_idx = torch.as_tensor(lay.node_theta_index(k))
            theta, theta_ref = V[th_idx], vref[th_idx]
            tf = theta[1]
            X = [V[torch.as_tensor(lay.x(k))]] + [V[torch.as_tensor(lay.coll_x(k, j))] for j in range(d)]
            for j in range(d):
                xp = sum(C[r, j + 1] * X[r] for r in range(d + 1))
                Wn.append(torch.cat([X[j + 1], xp / h / tf, V[torch.as_tensor(lay.u(k))],
                                     V[torch.as_tensor(lay.coll_z(k, j))], theta]))
                Rn.append(torch.cat([vref[torch.as_tensor(lay.coll_x(k, j))], torch.zeros(self.nx),
                                     vref[torch.as_tensor(lay.u(k))], vref[torch.as_tensor(lay.coll_z(k, j))],
                                     theta_ref]))
                wj.append(self.w[j])
            tfs.append(tf)
        Wn, Rn = torch.stack(Wn), torch.stack(Rn)
        wj = torch.as_tensor(np.array(wj))
        reg = wj[:, None] * w_eff[None, :] * (Wn - Rn) ** 2
        comp = {cat: reg[:, torch.as_tensor(ids)].sum() for cat, ids in cats.items()}
        _, _, power, betas = vmap(self.node, in_dims=(0, None, None))(Wn, gamma, th)
        # integral outputs (collocation.py:272-316): cumulative, interval t_f
        Lam = torch.as_tensor(np.linalg.solve(self.C[1:, 1:], np.eye(d)))
        Dc = torch.as_tensor(self.D)
        e_end = torch.zeros(())
        pw = power.reshape(n_k, d)
        for k in range(n_k):
            io = tfs[k] / n_k * (Lam.T @ pw[k])
            e_end = e_end + sum(Dc[j + 1] * io[j] for j in range(d))
        T = self.time_period(V, lay)
        power_cost = cost["power"] * (-1.) * e_end / T
        beta_cost = cost["beta"] * (wj[:, None] * betas ** 2).sum() / c["norm_beta"]
        T_ref = self.time_period(vref, lay)
        time_cost = cost["t_f"] * (T - T_ref) * (T - T_ref)
        homotopy = sum(cost[n] * phi[i] for i, n in enumerate(phi_names))
        general = (comp["fictitious"] + comp["u_regularisation"] + comp["xdot_regularisation"]
                   + comp["theta_regularisation"] + beta_cost + time_cost)
        return psi * comp["tracking"] + (1. - psi) * power_cost + general + homotopy

    def nlp_grad_f(self, V, P, lay, th, cost_names, phi_names):
        V = torch.as_tensor(V)
        return grad(lambda v: self.nlp_f(v, P, lay, th, cost_names, phi_names))(V)

    def nlp_hess_l(self, V, P, sigma, lam_g, lay, th, cost_names, phi_names):
        """Hessian of sigma f + lam_g^T g (nlp_hess_l) as a full symmetric scipy CSC matrix (test
        sizes only).  The continuity, periodicity and t_f rows are linear; every other g row lives
        in one interval, so lam^T g contributes per-interval blocks (torch.func hessian of
        lam_k^T interval_rows); the objective couples the intervals through the phase-fixed
        period, so its Hessian is taken densely (forward over reverse of nlp_f)."""
        import scipy.sparse as sp
        from torch.func import hessian
        V = torch.as_tensor(V)
        lam_g = torch.as_tensor(lam_g)
        idx = np.stack([lay.local_index(k) for k in range(self.n_k)])
        R = lay.rows_per_interval
        lam_k = lam_g[:self.n_k * R].reshape(self.n_k, R)
        Hk = vmap(hessian(lambda wl, ph, lk: lk @ self.interval_rows(wl, ph, th)), in_dims=(0, 0, 0))(
            V[torch.as_tensor(idx)], self._phases(), lam_k).numpy()
        n = lay.n_v
        rows = np.repeat(idx[:, :, None], idx.shape[1], axis=2)
        cols = np.repeat(idx[:, None, :], idx.shape[1], axis=1)
        H = sp.csc_matrix((Hk.ravel(), (rows.ravel(), cols.ravel())), shape=(n, n))
        Hf = jacfwd(grad(lambda v: self.nlp_f(v, P, lay, th, cost_names, phi_names)))(V).numpy()
        H = (H + sp.csc_matrix(float(sigma) * Hf)).tocsc()
        H.eliminate_zeros()
        return H


def from_constants(mc, lay):
    """Build the oracle from an ``awebox_amd.dual.MultiConstants`` (inputs only)."""
    from awebox_amd import dual as du
    import re
    cd = {n: float(mc.consts[i]) for i, n in enumerate(du.CONST_NAMES) if not re.match(r"(scaling|sd_len)\d+$", n)}
    return MultiKiteOracle(mc.cfg.parent_map, mc.scaling, cd, mc.sd_len, lay.n_k, lay.d,
                           lay.single_reelout, lay.nk_reelout)


def theta0_dict(theta0_vec):
    from awebox_amd import problem as pb
    th = {}
    for name, (o, sz) in pb.THETA0_OFF.items():
        v = torch.as_tensor(np.asarray(theta0_vec[o:o + sz], dtype=np.float64))
        th[name] = v[0] if sz == 1 else v
    return th
