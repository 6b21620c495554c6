"""Batched real-time iterations of the tracking MPC (config 5: B closed loops on one MI355X).

The reference closes the loop around ``Pmpc.step`` (awebox/pmpc.py:252-270, driven by
``sim.Simulation`` in examples/mpc_closed_loop.py): at every sampling time the MPC NLP is
re-solved from the shifted previous solution and the first control is applied to the plant.
Here B such loops run side by side as *real-time iterations* (Diehl's RTI): one Gauss-Newton SQP
step per sampling time for every loop, all loops batched:

* linearisation: one batched launch of the HIP MPC evaluator (f, g, grad f, J_g; awempc.hip);
* Hessian: the tracking cost (pmpc.py:304-358) is quadratic with a constant diagonal Hessian
  (computed once); constraint curvature is dropped (Gauss-Newton);
* step: the equality-constrained KKT system [H + dw I, J^T; J, -dc I] of every loop, solved by
  structured elimination -- the interior of each horizon interval (u, xdot, z, collocation
  variables and the multipliers of its node and collocation rows, 126 unknowns) by the batched LU
  kernel (batched_lu.hip, B x N blocks), then the Schur complement on the shooting states, the
  continuity and initial-condition multipliers (462 unknowns, B blocks, same kernel);
* plant: the first sampling interval is integrated with the applied control by the model's own
  radau collocation (Newton on the shooting and collocation rows of interval 0, the interval's
  60 x 60 block of J_g) -- the collocation integrator of ``sim``;
* shift: the horizon moves one interval (the new last interval copies the old one).

The path inequalities (tether stress, acceleration) and variable bounds are not part of the
step: along the tracked orbit they are inactive and the driver reports their maximum residual
(``rti_step`` output ``path_max``) instead of enforcing them; ``mpc_solve.BatchedPmpc`` solves the
same loops with bounds and inequalities to convergence (Pmpc.step).  Fixed globals (theta, phi,
xi) and the fictitious forces f_fict (fixed to 0 by pmpc.py:181-190) are not unknowns.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from . import kite3 as k3
from .collocation import coefficients
from .ipm import scatter_sum


def orbit_states(orbit: k3.CircularOrbit, t: np.ndarray) -> np.ndarray:
    """Vectorised CircularOrbit.state -> scaled-free x vectors [len(t), NX] (SI)."""
    cfg = orbit.cfg
    incl = cfg.inclination_deg * math.pi / 180.
    n_hat = np.array([math.cos(incl), 0.0, math.sin(incl)])
    y_rot = np.cross(n_hat, [1.0, 0.0, 0.0])
    y_rot /= np.linalg.norm(y_rot)
    z_rot = np.cross(n_hat, y_rot)
    z_rot /= np.linalg.norm(z_rot)
    psi = (orbit.angular_speed * (t % orbit.period)) % (2. * math.pi)
    outward = z_rot[None, :] * np.cos(psi)[:, None] - y_rot[None, :] * np.sin(psi)[:, None]
    e_tan = np.cross(n_hat[None, :], outward)
    e_tan /= np.linalg.norm(e_tan, axis=1, keepdims=True)
    X = np.zeros((len(t), k3.NX))
    X[:, 0:3] = outward * orbit.radius + n_hat[None, :] * orbit.height
    X[:, 3:6] = orbit.groundspeed * e_tan
    X[:, 6:8] = np.asarray(cfg.coeff_ref)
    X[:, 8] = cfg.l_t_init
    return X


class BatchedRti:
    """B tracking-MPC closed loops advanced by one real-time iteration per call of ``step``."""

    def __init__(self, consts: k3.Kite3Constants, batch: int, device="cuda", delta_w=1e-8, delta_c=0.0,
                 evaluator=None, plant="collocation", n_fe=20, fix_fict=True):
        """``evaluator``: anything with MpcEvaluator's device interface (sparsity_jac, n_p, nnz,
        eval_nlp_device); default = the HIP evaluator (awempc) for ``batch`` instances.
        ``plant``: "collocation" (interval 0's Radau collocation) or "rk4root" (the reference's
        sim integrator: ``n_fe`` RK4 steps per sampling time, the algebraic and derivative
        variables by a Newton rootfinder at every stage; tools/integrator_routines.py:32-96).
        ``fix_fict``: the fictitious forces stay at 0 (pmpc.py:181-190); False frees them."""
        self.consts, self.B, self.dev = consts, batch, torch.device(device)
        cfg = consts.cfg
        self.lay = lay = k3.MpcLayout(cfg.n_k, cfg.d)
        self.orbit = k3.CircularOrbit(cfg)
        if evaluator is None:
            from .mpc import MpcEvaluator
            evaluator = MpcEvaluator(consts, batch=batch)
        self.ev = evaluator
        self.tau, self.C, self.D, self.w = coefficients(cfg.d, "radau")
        f64 = dict(dtype=torch.float64, device=self.dev)
        B, n_v, n_g = batch, lay.n_v, lay.n_g
        nx, nk, st, v0 = k3.NX, lay.n_k, lay.interval_stride, lay.v_intervals
        # ---- unknowns: free V entries (interval variables + x[n_k]) and equality multipliers
        self.free = np.arange(v0, n_v)
        self.fict = k3.fict_columns(lay) if fix_fict else np.zeros(0, dtype=np.int64)
        self.free = np.setdiff1d(self.free, self.fict)
        path = np.concatenate([lay.g_path(k) for k in range(nk)])
        self.eq = np.setdiff1d(np.arange(n_g), path)
        self.path = path
        nw, ne = len(self.free), len(self.eq)
        self.nw, self.ne, self.N = nw, ne, nw + ne
        colmap = -np.ones(n_v, dtype=np.int64)
        colmap[self.free] = np.arange(nw)
        rowmap = -np.ones(n_g, dtype=np.int64)
        rowmap[self.eq] = np.arange(ne)
        # owner interval of every unknown (-1 = separator)
        owner = np.full(self.N, -1, dtype=np.int64)
        for p, v in enumerate(self.free):
            k, o = divmod(v - v0, st)
            if k < nk and o >= nx:
                owner[p] = k
        rows_pi = lay.rows_per_interval
        for i, r in enumerate(self.eq):
            if r >= nx:
                k, o = divmod(r - nx, rows_pi)
                if o < rows_pi - nx:                 # node / collocation rows; continuity -> separator
                    owner[nw + i] = k
        sep = np.where(owner < 0)[0]
        nS = len(sep)
        sep_id = np.full(self.N, -1, dtype=np.int64)
        sep_id[sep] = np.arange(nS)
        loc = np.full(self.N, -1, dtype=np.int64)
        counts = np.zeros(nk, dtype=np.int64)
        for p in np.where(owner >= 0)[0]:
            loc[p] = counts[owner[p]]
            counts[owner[p]] += 1
        nI = int(counts.max())
        if counts.min() != nI:
            raise ValueError("unequal interval interiors")
        self.nI, self.nS, self.nk = nI, nS, nk
        # ---- KKT pattern (both orientations): H diagonal, J (eq rows, free cols), -dc I
        colind, row = self.ev.sparsity_jac()
        jcol = np.repeat(np.arange(n_v), np.diff(colind))
        keep = (colmap[jcol] >= 0) & (rowmap[row] >= 0)
        self.j_keep = torch.tensor(np.where(keep)[0], device=self.dev)
        jr = nw + rowmap[row[keep]]
        jc = colmap[jcol[keep]]
        P_ = np.concatenate([np.arange(nw), jr, jc, nw + np.arange(ne)])
        Q_ = np.concatenate([np.arange(nw), jc, jr, nw + np.arange(ne)])
        self.nh = nw
        self.nj = len(jr)
        oP, oQ = owner[P_], owner[Q_]
        if ((oP >= 0) & (oQ >= 0) & (oP != oQ)).any():
            raise ValueError("KKT couples two interval interiors")
        ii, is_, ss = (oP >= 0) & (oP == oQ), (oP >= 0) & (oQ < 0), (oP < 0) & (oQ < 0)
        lsep = [sorted(set(sep_id[Q_[is_ & (oP == k)]].tolist())) for k in range(nk)]
        L = max(len(x) for x in lsep)
        lsep_arr = np.full((nk, L), nS, dtype=np.int64)
        lpos = np.full((nk, nS + 1), -1, dtype=np.int64)
        for k, l_ in enumerate(lsep):
            lsep_arr[k, :len(l_)] = l_
            lpos[k, l_] = np.arange(len(l_))
        self.L = L
        t = lambda a: torch.tensor(a, device=self.dev)  # noqa: E731
        bI, bIS = nk * nI * nI, nk * nI * L
        bo = np.arange(B)[:, None]
        self.sel_ii, self.sel_is, self.sel_ss = t(np.where(ii)[0]), t(np.where(is_)[0]), t(np.where(ss)[0])
        self.dst_ii = t((oP[ii] * nI * nI + loc[P_[ii]] * nI + loc[Q_[ii]])[None, :] + bo * bI).reshape(-1)
        isi = np.where(is_)[0]
        self.dst_is = t((oP[isi] * nI * L + loc[P_[isi]] * L + lpos[oP[isi], sep_id[Q_[isi]]])[None, :]
                        + bo * bIS).reshape(-1)
        r_idx = lsep_arr[:, :, None].repeat(L, axis=2)
        c_idx = lsep_arr[:, None, :].repeat(L, axis=1)
        self.lsep = t(lsep_arr)
        # ---- separators in stage order: stage 0 = [initial-condition multipliers, x[0]], stage
        # k + 1 = [continuity multipliers of interval k, x[k + 1]]; the separator system is then
        # block tridiagonal (awelu_btd_solve_batched).
        stage = np.full(nS, -1, dtype=np.int64)
        for q, p in enumerate(sep):
            if p < nw:
                stage[q] = (self.free[p] - v0) // st
            else:
                r = self.eq[p - nw]
                stage[q] = 0 if r < nx else (r - nx) // rows_pi + 1
        nb = int(stage.max()) + 1
        spos = np.zeros(nS, dtype=np.int64)
        sizes = np.zeros(nb, dtype=np.int64)
        for q in range(nS):
            spos[q] = sizes[stage[q]]
            sizes[stage[q]] += 1
        m = int(sizes.max())
        self.nb, self.m = nb, m

        def btd_index(qr, qc):
            a, b_ = stage[qr], stage[qc]
            if np.any(np.abs(a - b_) > 1):
                raise ValueError("separator system is not block tridiagonal in stage order")
            return ((a * 3 + 1 + b_ - a) * m + spos[qr]) * m + spos[qc]
        bT = nb * 3 * m * m
        self.bT = bT
        self.btd_ss = t(btd_index(sep_id[P_[ss]], sep_id[Q_[ss]])[None, :] + bo * bT).reshape(-1)
        valid = (r_idx < nS) & (c_idx < nS)                      # [nk, L, L]
        self.schur_src = t(np.where(valid.reshape(-1))[0])
        self.btd_schur = t(btd_index(r_idx[valid], c_idx[valid])[None, :] + bo * bT).reshape(-1)
        # fixed-order sums over the duplicate destinations (the separators shared by neighbouring
        # intervals): index_add_ would add them with run-dependent atomics on the GPU
        self._schur_sum = scatter_sum(self.btd_schur.cpu().numpy(), self.dev)
        self._rs_sum = scatter_sum(self.lsep.reshape(-1).cpu().numpy(), self.dev)
        T0 = np.zeros((nb, 3, m, m))
        for a in range(nb):
            for i in range(sizes[a], m):
                T0[a, 1, i, i] = 1.0                              # padding of short stages
        self.T0 = t(T0.reshape(-1))
        self.sep_btd = t(stage * m + spos)                        # separator q -> stage-order slot
        int_p = np.where(owner >= 0)[0]
        self.int_p, self.int_flat = t(int_p), t(owner[int_p] * nI + loc[int_p])
        self.sep_p = t(sep)
        self.bI, self.bIS = bI, bIS
        self.delta_w, self.delta_c = delta_w, delta_c
        # ---- constant Gauss-Newton Hessian: the diagonal of the quadratic tracking cost
        self.V = torch.zeros(B, n_v, **f64)
        self.P = torch.zeros(B, self.ev.n_p, **f64)
        self.f = torch.zeros(B, **f64)
        self.g = torch.zeros(B, n_g, **f64)
        # the evaluator's preferred layout (instance-minor for the HIP MPC evaluator's generated path)
        self.grad = self.ev.alloc_grad(self.dev) if hasattr(self.ev, "alloc_grad") else torch.zeros(B, n_v, **f64)
        self.jac = self.ev.alloc_jac(self.dev) if hasattr(self.ev, "alloc_jac") else torch.zeros(B, self.ev.nnz, **f64)
        self.free_t, self.eq_t = t(self.free), t(self.eq)
        self.path_t = t(path)
        self.u0_idx = t(lay.u(0))
        self.hdiag = None
        # plant: interval 0's shooting + collocation rows against its interior unknowns
        self.pl_rows = t(np.concatenate([lay.g_shooting(0), np.concatenate([lay.g_coll(0, j) for j in range(cfg.d)])]))
        self.pl_cols = t(np.concatenate([lay.xdot(0), lay.z(0)] + [np.concatenate([lay.coll_x(0, j), lay.coll_z(0, j)])
                                                                  for j in range(cfg.d)]))
        jr_all, jc_all = row, jcol
        rsel = {int(r): i for i, r in enumerate(self.pl_rows.cpu().numpy())}
        csel = {int(c): i for i, c in enumerate(self.pl_cols.cpu().numpy())}
        pk = [e for e in range(len(row)) if int(jr_all[e]) in rsel and int(jc_all[e]) in csel]
        self.n_pl = n_pl = len(rsel)
        if len(csel) != n_pl:
            raise ValueError("interval 0 is not square in its interior unknowns")
        self.pl_keep = t(np.array(pk))
        self.pl_dst = t(np.array([rsel[int(jr_all[e])] * n_pl + csel[int(jc_all[e])] for e in pk]))
        self.x_idx = [t(lay.x(0))] + [t(lay.coll_x(0, j)) for j in range(cfg.d)]
        if plant not in ("collocation", "rk4root"):
            raise ValueError(f"unknown plant {plant!r}")
        self.plant, self.n_fe = plant, n_fe
        self.plant_tol = 1e-9                   # step(): plant_converged = residual <= plant_tol
        self.sim_blocks = self.sim_xs = None
        # rk4root: the shooting-node rows of interval 0 against (xdot[0], z[0])
        self.rk_rows = t(lay.g_shooting(0))
        self.rk_cols = t(np.concatenate([lay.xdot(0), lay.z(0)]))
        rsel = {int(r): i for i, r in enumerate(lay.g_shooting(0))}
        csel = {int(c): i for i, c in enumerate(np.concatenate([lay.xdot(0), lay.z(0)]))}
        if len(rsel) != len(csel):
            raise ValueError("shooting rows and (xdot, z) do not form a square system")
        pk = [e for e in range(len(row)) if int(jr_all[e]) in rsel and int(jc_all[e]) in csel]
        self.n_rk = len(rsel)
        self.rk_keep = t(np.array(pk))
        self.rk_dst = t(np.array([rsel[int(jr_all[e])] * self.n_rk + csel[int(jc_all[e])] for e in pk]))
        self.xdot_idx = t(lay.xdot(0))
        s_ = consts.scaling
        self.rk_ratio = torch.tensor(s_[k3.NX:2 * k3.NX] / s_[:k3.NX], dtype=torch.float64, device=self.dev)

    # ------------------------------------------------------------------ set-up ----------
    def reference(self, t0: np.ndarray) -> np.ndarray:
        """Scaled reference windows [B, n_v] starting at times t0[B] (kite3.reference_window)."""
        cfg, lay, s = self.consts.cfg, self.lay, self.consts.scaling
        nk, d, nx = lay.n_k, lay.d, k3.NX
        times = [t0[:, None] + np.arange(nk + 1)[None, :] * cfg.ts]
        tc = t0[:, None, None] + (np.arange(nk)[None, :, None] + self.tau[None, None, 1:]) * cfg.ts
        R = np.zeros((len(t0), lay.n_v))
        R[:, lay.theta()] = np.array([cfg.diam_t, nk * cfg.ts]) / s[2 * nx + k3.NU + k3.NZ:]
        Xs = orbit_states(self.orbit, times[0].reshape(-1)).reshape(len(t0), nk + 1, nx) / s[:nx]
        Xc = orbit_states(self.orbit, tc.reshape(-1)).reshape(len(t0), nk, d, nx) / s[:nx]
        for k in range(nk + 1):
            R[:, lay.x(k)] = Xs[:, k]
            if k < nk:
                for j in range(d):
                    R[:, lay.coll_x(k, j)] = Xc[:, k, j]
                    R[:, lay.coll_z(k, j)] = 1.0
        return R

    def _reference_setup(self):
        """Index maps and constants of the device-side reference window (``_reference_device``)."""
        cfg, lay, s = self.consts.cfg, self.lay, self.consts.scaling
        nk, d, nx = lay.n_k, lay.d, k3.NX
        t = lambda a: torch.tensor(a, device=self.dev)  # noqa: E731
        incl = cfg.inclination_deg * math.pi / 180.
        n_hat = np.array([math.cos(incl), 0.0, math.sin(incl)])
        y_rot = np.cross(n_hat, [1.0, 0.0, 0.0])
        y_rot /= np.linalg.norm(y_rot)
        z_rot = np.cross(n_hat, y_rot)
        z_rot /= np.linalg.norm(z_rot)
        o = self.orbit
        self._ref = {
            "n_hat": t(n_hat), "y_rot": t(y_rot), "z_rot": t(z_rot),
            "sx": t(s[:nx]), "coeff": t(np.asarray(cfg.coeff_ref, dtype=np.float64)),
            "offs": t(np.concatenate([np.arange(nk + 1, dtype=np.float64),
                                      (np.arange(nk)[:, None] + self.tau[None, 1:]).reshape(-1)]) * cfg.ts),
            "idx": t(np.concatenate([np.stack([lay.x(k) for k in range(nk + 1)]),
                                     np.stack([lay.coll_x(k, j) for k in range(nk) for j in range(d)])])),
            "base": t(self.reference(np.zeros(1))[0] * 0.0),
        }
        base = self._ref["base"]
        base[t(lay.theta())] = t(np.array([cfg.diam_t, nk * cfg.ts]) / s[2 * nx + k3.NU + k3.NZ:])
        for k in range(nk):
            for j in range(d):
                base[t(lay.coll_z(k, j))] = 1.0
        self._ref.update(radius=o.radius, height=o.height, omega=o.angular_speed, period=o.period,
                         speed=o.groundspeed, l_t=cfg.l_t_init)

    def _reference_device(self, t0):
        """``reference`` on the device: t0 [B] float64 tensor -> scaled windows [B, n_v]."""
        r = self._ref
        tt = t0[:, None] + r["offs"][None, :]                                  # [B, n_times]
        psi = torch.remainder(r["omega"] * torch.remainder(tt, r["period"]), 2.0 * math.pi)
        outward = r["z_rot"] * torch.cos(psi)[..., None] - r["y_rot"] * torch.sin(psi)[..., None]
        e_tan = torch.linalg.cross(r["n_hat"].expand_as(outward), outward, dim=-1)
        e_tan = e_tan / e_tan.norm(dim=-1, keepdim=True)
        X = torch.cat([outward * r["radius"] + r["n_hat"] * r["height"], r["speed"] * e_tan,
                       r["coeff"].expand(*tt.shape, 2), torch.full_like(tt, r["l_t"])[..., None],
                       torch.zeros(*tt.shape, 2, dtype=tt.dtype, device=tt.device)], dim=-1) / r["sx"]
        R = r["base"].repeat(t0.shape[0], 1)
        R[:, r["idx"].reshape(-1)] = X.reshape(t0.shape[0], -1)
        return R

    def start(self, seed: int = 99, sigma: float = 0.01, x0_entries=None):
        """Loop i starts at phase i T / B with x0 and the initial guess perturbed by sigma N(0,1)
        (SURVEY 8(d) config 5); ``x0_entries`` restricts the x0 perturbation to those state
        indices (default: all)."""
        B, lay = self.B, self.lay
        self.t0 = np.arange(B) * self.orbit.period / B
        ref = self.reference(self.t0)
        rng = [np.random.default_rng(seed + i) for i in range(B)]
        noise = sigma * np.stack([r.standard_normal(k3.NX) for r in rng])
        if x0_entries is not None:
            keep = np.zeros(k3.NX, dtype=bool)
            keep[np.asarray(x0_entries)] = True
            noise[:, ~keep] = 0.0
        x0 = ref[:, lay.x(0)] + noise
        V = ref + sigma * np.stack([r.standard_normal(lay.n_v) for r in rng])
        V[:, :lay.v_intervals] = ref[:, :lay.v_intervals]
        V[:, self.fict] = 0.0
        P = np.stack([k3.pack_p(lay, self.consts, x0[i], ref[i]) for i in range(B)])
        self.V.copy_(torch.tensor(V))
        self.P.copy_(torch.tensor(P))
        self.lam = torch.zeros(B, self.ne, dtype=torch.float64, device=self.dev)
        self.step_count = 0
        self.sim_blocks = self.sim_xs = None
        self.t0_dev = torch.tensor(self.t0, dtype=torch.float64, device=self.dev)
        self._reference_setup()
        if self.hdiag is None:
            self._hessian_diagonal()

    def simulate_reference(self, n_nodes: int, u_c: torch.Tensor | None = None):
        """Track a trajectory of the 3-DOF model instead of the synthetic circle.

        The reference's MPC tracks an optimised power cycle, a solution of the model by
        construction (pmpc.py:__create_reference_interpolator); the circle of
        kite3.reference_window is not one without the fictitious forces, so a loop tracking it
        keeps a tracking error of order 1 and never converges.  Here every loop's reference is the
        plant (interval 0's radau collocation) integrated on the sampling grid for ``n_nodes``
        sampling times from the circle's state at the loop's phase with the constant control
        ``u_c`` (default zero rates: CL, roll and reel acceleration hold), so each window
        (shooting states, collocation states and z, controls) is an exact solution of the MPC's
        own discretisation.  The current perturbations of x0 and of the initial guess are kept
        relative to the new windows; ``_shift`` then reads windows of this trajectory."""
        lay, B = self.lay, self.B
        nx, st, v0, nk = k3.NX, lay.interval_stride, lay.v_intervals, lay.n_k
        if n_nodes < nk:
            raise ValueError("the simulated reference must cover at least one horizon")
        if u_c is None:
            u_c = torch.zeros(B, k3.NU, dtype=torch.float64, device=self.dev)
        ref_old = self.P[:, lay.p_ref:lay.p_ref + lay.n_v].clone()
        dx0 = self.P[:, lay.p_x0:lay.p_x0 + nx] - ref_old[:, lay.x(0)[0]:lay.x(0)[0] + nx]
        dV = self.V - ref_old
        V_save = self.V.clone()
        blocks = torch.zeros(B, n_nodes, st, dtype=torch.float64, device=self.dev)
        xs = torch.zeros(B, n_nodes + 1, nx, dtype=torch.float64, device=self.dev)
        x = ref_old[:, lay.x(0)[0]:lay.x(0)[0] + nx].clone()
        u0 = self.u0_idx
        for j in range(n_nodes):
            self.P[:, lay.p_x0:lay.p_x0 + nx] = x
            self.V[:, u0] = u_c
            x1, res = self._plant()
            if float(res.max()) > 1e-9:
                raise RuntimeError(f"reference simulation: plant residual {float(res.max()):.2e} at node {j}")
            blocks[:, j] = self.plant_V[:, v0:v0 + st]
            xs[:, j] = x
            self.V[:, v0:v0 + st] = self.plant_V[:, v0:v0 + st]
            x = x1
        xs[:, n_nodes] = x
        self.sim_blocks, self.sim_xs = blocks, xs
        R = self._reference_sim(0)
        self.P[:, lay.p_ref:lay.p_ref + lay.n_v] = R
        self.P[:, lay.p_x0:lay.p_x0 + nx] = R[:, lay.x(0)[0]:lay.x(0)[0] + nx] + dx0
        self.V.copy_(R + dV)
        self.V[:, :v0] = V_save[:, :v0]
        self.V[:, self.fict] = V_save[:, self.fict]

    def _reference_sim(self, s: int) -> torch.Tensor:
        """Window s (sampling times s .. s + N) of the simulated reference trajectory."""
        lay = self.lay
        nx, st, v0, nk = k3.NX, lay.interval_stride, lay.v_intervals, lay.n_k
        if s + nk > self.sim_blocks.shape[1]:
            raise ValueError(f"the simulated reference ends before window {s}; simulate more nodes")
        R = self._ref["base"].repeat(self.B, 1)
        R[:, v0:v0 + nk * st] = self.sim_blocks[:, s:s + nk].reshape(self.B, nk * st)
        xN = lay.x(nk)[0]
        R[:, xN:xN + nx] = self.sim_xs[:, s + nk]
        return R

    def _hessian_diagonal(self):
        """The tracking cost is quadratic and separable: grad(V + h) - grad(V) = h diag(H)."""
        self.ev.eval_nlp_device(self.V, self.P, self.f, self.g, self.grad, self.jac)
        g0 = self.grad.clone()
        Vh = self.V.clone()
        Vh[:, self.free_t] += 1.0
        self.ev.eval_nlp_device(Vh, self.P, self.f, self.g, self.grad, self.jac)
        self.hdiag = (self.grad - g0)[:, self.free_t].contiguous()          # [B, nw]

    # ------------------------------------------------------------------ one RTI ---------
    @staticmethod
    def _lu(A):
        """Batched LU: the awelu kernel for device blocks, torch's for host tensors (CPU tests)."""
        if A.is_cuda:
            from .batched_lu import lu_factor
            return lu_factor(A)
        return torch.linalg.lu_factor(A)

    @staticmethod
    def _solve(LU, piv, B):
        if LU.is_cuda:
            from .batched_lu import lu_solve
            return lu_solve(LU, piv, B)
        return torch.linalg.lu_solve(LU, piv, B)

    @staticmethod
    def _btd(T, X):
        from .batched_lu import btd_dense, btd_factor, btd_solve
        if T.is_cuda:
            F, Dinv = btd_factor(T)
            return btd_solve(F, Dinv, X)
        b, nb, m, nrhs = X.shape
        return torch.linalg.solve(btd_dense(T), X.reshape(b, nb * m, nrhs)).view(b, nb, m, nrhs)

    def _factor_solve(self, rhs):
        B, nk, nI, L, nS = self.B, self.nk, self.nI, self.L, self.nS
        f64 = dict(dtype=torch.float64, device=self.dev)
        jv = self.jac[:, self.j_keep]
        vals = torch.cat([self.hdiag + self.delta_w, jv, jv, torch.full((B, self.ne), -self.delta_c, **f64)], dim=1)
        KII = torch.zeros(B * self.bI, **f64)
        KII[self.dst_ii] = vals[:, self.sel_ii].reshape(-1)
        KIS = torch.zeros(B * self.bIS, **f64)
        KIS[self.dst_is] = vals[:, self.sel_is].reshape(-1)
        Tb = self.T0.repeat(B)
        Tb[self.btd_ss] = vals[:, self.sel_ss].reshape(-1)
        KII = KII.view(B * nk, nI, nI)
        KIS = KIS.view(B * nk, nI, L)
        LU, piv = self._lu(KII)
        rI = torch.zeros(B, nk * nI, **f64)
        rI[:, self.int_flat] = rhs[:, self.int_p]
        # K_II^-1 [K_IS | r_I] in one batched solve (the solve is latency-bound, not width-bound)
        Xz = self._solve(LU, piv, torch.cat([KIS, rI.view(B * nk, nI, 1)], dim=2))
        X, z = Xz[:, :, :L], Xz[:, :, L:]
        Tsch = (KIS.transpose(1, 2) @ X).view(B, nk * L * L)
        self._schur_sum.add_into(Tb, -Tsch[:, self.schur_src].reshape(-1))
        upd = (KIS.transpose(1, 2) @ z).view(B, nk * L)
        rS = torch.zeros(B, nS + 1, **f64)
        rS[:, :nS] = rhs[:, self.sep_p]
        self._rs_sum.add_into(rS, -upd)
        rb = torch.zeros(B, self.nb * self.m, **f64)
        rb[:, self.sep_btd] = rS[:, :nS]
        xb = self._btd(Tb.view(B, self.nb, 3, self.m, self.m), rb.view(B, self.nb, self.m, 1)).view(B, -1)
        xS = torch.zeros(B, nS + 1, **f64)
        xS[:, :nS] = xb[:, self.sep_btd]
        xI = z.reshape(B * nk, nI) - (X @ xS[:, self.lsep].reshape(B * nk, L, 1)).view(B * nk, nI)
        sol = torch.empty(B, self.N, **f64)
        sol[:, self.int_p] = xI.view(B, nk * nI)[:, self.int_flat]
        sol[:, self.sep_p] = xS[:, :nS]
        return sol

    def iterate(self):
        """One Gauss-Newton SQP iteration at the current P for every loop (linearise, solve, full
        step); returns the equality residual and the largest path-constraint value at the
        linearisation point."""
        self.ev.eval_nlp_device(self.V, self.P, self.f, self.g, self.grad, self.jac)
        g_eq = self.g[:, self.eq_t]
        rhs = torch.cat([-self.grad[:, self.free_t], -g_eq], dim=1)
        sol = self._factor_solve(rhs)
        self.V[:, self.free_t] += sol[:, :self.nw]
        self.lam = sol[:, self.nw:]
        return g_eq.abs().amax(dim=1), self.g[:, self.path_t].amax(dim=1)

    def step(self):
        """One RTI for every loop: an SQP iteration, the first control applied to the plant, the
        horizon shifted.  Returns per-loop diagnostics."""
        kkt_res, path_max = self.iterate()
        self.u0 = self.V[:, self.u0_idx].clone()
        x1, plant_res = self._plant() if self.plant == "collocation" else self._rk4root()
        self._shift(x1)
        self.step_count += 1
        x_ref = self.P[:, self.lay.p_ref + self.lay.x(0)[0]:self.lay.p_ref + self.lay.x(0)[0] + k3.NX]
        return {"eq_residual": kkt_res, "path_max": path_max, "plant_residual": plant_res,
                "plant_converged": plant_res <= self.plant_tol,
                "tracking_error": (x1 - x_ref).norm(dim=1), "x0": x1, "u0": self.u0}

    def _plant(self, max_newton=8, tol=1e-11):
        """x(t + ts) from x0 and the applied u[0]: radau collocation of interval 0, Newton on its
        shooting + collocation rows (60 for d = 4) in its interior unknowns (sim's collocation
        integrator), until every loop's residual is below ``tol``.  Returns (x1, final residual)."""
        n = self.n_pl
        Vp = self.V.clone()
        Vp[:, self.x_idx[0]] = self.P[:, self.lay.p_x0:self.lay.p_x0 + k3.NX]
        for it in range(max_newton + 1):
            self.ev.eval_nlp_device(Vp, self.P, self.f, self.g, self.grad, self.jac)
            r = self.g[:, self.pl_rows]
            res = r.abs().amax(dim=1)
            if it == max_newton or (it >= 2 and float(res.max()) < tol):
                break
            A = torch.zeros(self.B, n * n, dtype=torch.float64, device=self.dev)
            A[:, self.pl_dst] = self.jac[:, self.pl_keep]
            LU, piv = self._lu(A.view(self.B, n, n))
            Vp[:, self.pl_cols] -= self._solve(LU, piv, r.unsqueeze(-1).contiguous()).squeeze(-1)
        x1 = sum(float(self.D[r_]) * Vp[:, self.x_idx[r_]] for r_ in range(self.lay.d + 1))
        self.plant_V = Vp                       # interval 0's solved variables (simulated references)
        return x1, res

    def _rk4root(self, max_newton=6, tol=1e-11):
        """The reference's plant (sim.py:72-78 -> rk4root, integrator_routines.py:32-96): n_fe RK4
        steps over one sampling time with the applied u[0]; at every stage the rootfinder solves
        the shooting-node rows (dynamics, holonomic and trivial rows: 12 for the 3-DOF kite) for
        (xdot, z) at the stage state -- here Newton on the HIP evaluator's rows and Jacobian
        block, warm-started from the previous stage.  Returns (x1, the largest rootfinder
        residual)."""
        n, B = self.n_rk, self.B
        h = self.consts.cfg.ts / self.n_fe
        Vp = self.V.clone()
        x = self.P[:, self.lay.p_x0:self.lay.p_x0 + k3.NX].clone()
        worst = torch.zeros(B, dtype=torch.float64, device=self.dev)

        def ode(xs):
            nonlocal worst
            Vp[:, self.x_idx[0]] = xs
            for it in range(max_newton + 1):
                self.ev.eval_nlp_device(Vp, self.P, self.f, self.g, self.grad, self.jac)
                r = self.g[:, self.rk_rows]
                res = r.abs().amax(dim=1)
                if it == max_newton or float(res.max()) < tol:
                    break
                A = torch.zeros(B, n * n, dtype=torch.float64, device=self.dev)
                A[:, self.rk_dst] = self.jac[:, self.rk_keep]
                LU, piv = self._lu(A.view(B, n, n))
                Vp[:, self.rk_cols] -= self._solve(LU, piv, r.unsqueeze(-1).contiguous()).squeeze(-1)
            worst = torch.maximum(worst, res)
            return Vp[:, self.xdot_idx] * self.rk_ratio

        for _ in range(self.n_fe):
            k1 = ode(x)
            k2 = ode(x + 0.5 * h * k1)
            k3_ = ode(x + 0.5 * h * k2)
            k4 = ode(x + h * k3_)
            x = x + h * (k1 + 2.0 * k2 + 2.0 * k3_ + k4) / 6.0
        return x, worst

    def _shift(self, x1):
        """Move the horizon one interval: V[k] <- V[k+1], keep the last interval; new x0 and the
        reference window of the next sampling time."""
        lay, st, v0 = self.lay, self.lay.interval_stride, self.lay.v_intervals
        nk = lay.n_k
        body = self.V[:, v0:v0 + nk * st].view(self.B, nk, st)
        shifted = torch.cat([body[:, 1:], body[:, -1:]], dim=1).reshape(self.B, nk * st)
        self.V[:, v0:v0 + nk * st] = shifted
        self.P[:, lay.p_x0:lay.p_x0 + k3.NX] = x1
        if self.sim_blocks is not None:
            R = self._reference_sim(self.step_count + 1)
            self.P[:, lay.p_ref:lay.p_ref + lay.n_v] = R
            # the new last interval and x[N]: the reference's (a solution of the dynamics) instead of
            # a copy of the old last interval
            tail = slice(v0 + (nk - 1) * st, lay.n_v)
            self.V[:, tail] = R[:, tail]
            self.V[:, self.fict] = 0.0
        else:
            self.P[:, lay.p_ref:lay.p_ref + lay.n_v] = self._reference_device(
                self.t0_dev + (self.step_count + 1) * self.consts.cfg.ts)
