"""DAE integrators over one shooting interval, on the HIP evaluator.

The reference re-integrates a solved trajectory with the DAE integrators of its multiple-shooting
discretisation to check the direct-collocation solution (test/reg/test_discretization.py:20-193):

* ``collocation``: CasADi's collocation integrator with the NLP's own scheme (radau, d = 4) and one
  step per interval (``nlp.integrator.num_steps_overwrite = 1``).  Its equations over one interval
  are the direct-collocation rows of that interval, so it reproduces ``V.x[k+1]`` to the NLP
  tolerance (the reference asserts 1e-7 relative);
* ``rk4root``: awebox's own RK4 with a rootfinder for the algebraic variables at every stage
  (``tools/integrator_routines.py:32-96``), 30 steps per interval in the test (2e-2 relative).

The awebox DAE treats the state derivatives as algebraic variables (``dae.fill_in_dae_variables``:
x = states, z = [xdot, z], p = [u, theta, params]): ode x' = xdot, alg 0 = F(x, xdot, u, z).  Both
integrators here solve exactly those rows with the HIP evaluator's values and Jacobian blocks:

* collocation: Newton on interval k's shooting-node rows and collocation rows in its interior
  unknowns (xdot[k], z[k], and the collocation states and algebraics), from V's values;
* rk4root: RK4 on x' = xdot(x) where xdot(x), z(x) solve the shooting-node rows at the stage state
  (Newton, warm-started from the previous stage); the quadrature (the power integral output,
  ``dynamics.py:318-330``) is integrated by the same RK4 stages.

All arithmetic is float64 on the evaluator's device; the small Newton systems (24 and 120 unknowns
for the AP2 kite) are dense solves.  ``integrand(x, z)`` returns the quadrature integrand per
instance from scaled states x [B, n_x] and algebraic variables z [B, n_z].
"""
from __future__ import annotations

import numpy as np
import torch


class IntervalIntegrator:
    """Integrators of interval ``k`` of a collocation NLP on the evaluator ``ev`` (batch B)."""

    def __init__(self, ev, lay, scaling, k: int = 0, device="cuda"):
        self.ev, self.lay, self.k = ev, lay, k
        self.dev = torch.device(device)
        t = lambda a: torch.tensor(np.asarray(a, dtype=np.int64), device=self.dev)  # noqa: E731
        colind, row = ev.sparsity_jac()
        jcol = np.repeat(np.arange(ev.n_v), np.diff(colind))
        d = lay.d
        nx = len(lay.x(k))

        def block(rows, cols):
            rsel = {int(r): i for i, r in enumerate(rows)}
            csel = {int(c): i for i, c in enumerate(cols)}
            if len(rsel) != len(csel):
                raise ValueError("rows and unknowns do not form a square system")
            keep = np.where(np.isin(row, rows) & np.isin(jcol, cols))[0]
            dst = np.array([rsel[int(row[e])] * len(rsel) + csel[int(jcol[e])] for e in keep], dtype=np.int64)
            return t(rows), t(cols), t(keep), t(dst), len(rsel)

        shoot_rows = lay.g_shooting(k)
        shoot_cols = np.concatenate([lay.xdot(k), lay.z(k)])
        self.rk = block(shoot_rows, shoot_cols)
        coll_rows = np.concatenate([shoot_rows] + [lay.g_coll(k, j) for j in range(d)])
        coll_cols = np.concatenate([shoot_cols] + [np.concatenate([lay.coll_x(k, j), lay.coll_z(k, j)])
                                                   for j in range(d)])
        self.co = block(coll_rows, coll_cols)
        self.x_idx = t(lay.x(k))
        self.xdot_idx = t(lay.xdot(k))
        self.xcol_idx = [t(lay.coll_x(k, j)) for j in range(d)]
        self.z_idx = t(lay.z(k))
        self.zcol_idx = [t(lay.coll_z(k, j)) for j in range(d)]
        s = np.asarray(scaling, dtype=np.float64)
        self.ratio = torch.tensor(s[nx:2 * nx] / s[:nx], device=self.dev)   # xdot_scaled -> d(x_scaled)/dt
        from .collocation import coefficients
        tau, C, D, w = coefficients(d, "radau")
        self.D = [float(v) for v in np.asarray(D, dtype=float)]
        self.w = [float(v) for v in np.asarray(w, dtype=float)]
        self._B = None

    def _buffers(self, B):
        if self._B != B:
            f64 = dict(dtype=torch.float64, device=self.dev)
            ev = self.ev
            self.f, self.g = torch.zeros(B, **f64), torch.zeros(B, ev.n_g, **f64)
            self.grad, self.jac = torch.zeros(B, ev.n_v, **f64), torch.zeros(B, ev.nnz, **f64)
            self._B = B

    def _newton(self, V, P, blk, max_newton, tol, damped=False):
        """Newton on the rows of ``blk`` in its unknowns, in place in V; with ``damped`` the step is
        halved until the max-norm residual decreases (per instance).  Returns the final residual."""
        rows, cols, keep, dst, n = blk
        B = V.shape[0]
        self._buffers(B)
        self.ev.eval_nlp_device(V, P, self.f, self.g, self.grad, self.jac)
        r = self.g[:, rows].clone()
        res = r.abs().amax(dim=1)
        for it in range(max_newton):
            if float(res.max()) < tol:
                break
            A = torch.zeros(B, n * n, dtype=torch.float64, device=self.dev)
            A[:, dst] = self.jac[:, keep]
            step = torch.linalg.solve(A.view(B, n, n), r.unsqueeze(-1)).squeeze(-1)
            base = V[:, cols].clone()
            a = torch.ones(B, 1, dtype=torch.float64, device=self.dev)
            for _ in range(30 if damped else 1):
                V[:, cols] = base - a * step
                self.ev.eval_nlp_device(V, P, self.f, self.g, self.grad, self.jac)
                r_t = self.g[:, rows]
                res_t = r_t.abs().amax(dim=1)
                bad = ~(res_t < res) & (res >= tol)
                if not damped or not bool(bad.any()):
                    break
                a = torch.where(bad.unsqueeze(1), 0.5 * a, a)
            r, res = r_t.clone(), res_t
        return res

    def collocation(self, V, P, integrand, h, x0=None, max_newton=30, tol=1e-12, warm=False):
        """One radau collocation step over the interval (length h [s] per instance, tensor [B]) from
        x0 (default: V.x[k]).  The Newton iteration starts from CasADi's collocation-integrator
        guess -- x0 and the shooting node's z at every collocation point -- unless ``warm`` (V's
        own collocation values).  Returns dict(x_end, z_end, q, residual, V) with the collocation
        unknowns solved in a copy of V."""
        Vp = V.clone()
        if x0 is not None:
            Vp[:, self.x_idx] = x0
        if not warm:
            for j in range(len(self.xcol_idx)):
                Vp[:, self.xcol_idx[j]] = Vp[:, self.x_idx]
                Vp[:, self.zcol_idx[j]] = Vp[:, self.z_idx]
        res = self._newton(Vp, P, self.co, max_newton, tol, damped=True)
        x_end = sum(self.D[r] * (Vp[:, self.x_idx] if r == 0 else Vp[:, self.xcol_idx[r - 1]])
                    for r in range(len(self.D)))
        q = sum(h * self.w[j] * integrand(Vp[:, self.xcol_idx[j]], Vp[:, self.zcol_idx[j]])
                for j in range(len(self.w)))
        z_end = Vp[:, self.zcol_idx[-1]]
        return {"x_end": x_end, "z_end": z_end, "q": q, "residual": res, "V": Vp}

    def rk4root(self, V, P, integrand, h, n_steps=30, x0=None, max_newton=20, tol=1e-12):
        """n_steps RK4 steps over the interval (length h [s], tensor [B]) with the stage rootfinder.
        Returns dict(x_end, z_end, q, residual) (z_end from the rootfinder at x_end)."""
        Vp = V.clone()
        x = (Vp[:, self.x_idx] if x0 is None else x0).clone()
        dt = (h / n_steps).unsqueeze(-1)
        worst = torch.zeros(V.shape[0], dtype=torch.float64, device=self.dev)

        def ode(xs):
            nonlocal worst
            Vp[:, self.x_idx] = xs
            res = self._newton(Vp, P, self.rk, max_newton, tol)
            worst = torch.maximum(worst, res)
            return Vp[:, self.xdot_idx] * self.ratio, integrand(xs, Vp[:, self.z_idx])

        q = torch.zeros(V.shape[0], dtype=torch.float64, device=self.dev)
        for _ in range(n_steps):
            k1, p1 = ode(x)
            k2, p2 = ode(x + 0.5 * dt * k1)
            k3, p3 = ode(x + 0.5 * dt * k2)
            k4, p4 = ode(x + dt * k3)
            x = x + dt * (k1 + 2.0 * k2 + 2.0 * k3 + k4) / 6.0
            q = q + dt[:, 0] * (p1 + 2.0 * p2 + 2.0 * p3 + p4) / 6.0
        ode(x)
        z_end = Vp[:, self.z_idx]
        return {"x_end": x, "z_end": z_end, "q": q, "residual": worst}
