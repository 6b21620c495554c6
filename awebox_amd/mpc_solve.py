"""Converged tracking MPC for B closed loops: ``Pmpc.step`` (awebox/pmpc.py:221-302) restated on
the batched GPU interior-point method.

Where ``rti.BatchedRti`` takes one Gauss-Newton step per sampling time on the equality rows only,
``BatchedPmpc`` solves every loop's MPC NLP to IPOPT's tolerance with everything the reference's
solver sees:

* variable bounds (kite3.variable_bounds: system bounds on x[1..N], u, z; x[0] released; f_fict,
  theta, phi, xi fixed) and the path inequalities (tether stress, acceleration; released at k = 0,
  pmpc.py:125-131) as inequality rows with slacks;
* the exact Hessian of the Lagrangian (IPOPT's default, pmpc.py:193-217, default.py:323) from the
  HIP MPC evaluator's hyper-dual Hessian kernel (awempc_eval_hess: one thread per structurally
  nonzero direction pair of a node, tracking cost added in closed form), one batched launch per
  Hessian; coloured central differences of the exact gradient (fd_hessian.FdHessian) remain as
  ``hessian="fd"`` for evaluators without a Hessian;
* ``homotopy_warmstart`` (mpc_closed_loop.py:69): a 2-iteration pre-solve at mu = 1e-3
  (``mu_init = mu_target = 1e-3``, ``tol = 1e-4``, ``max_iter = 2``, pmpc.py:206-212) whose
  primal point starts the main solve (``mu_init = 1e-3``, ``tol = 1e-6``, pmpc.py:199-207);
  multipliers are not carried over (nlpsol is called with x0 only, :257-270);
* the shift of the previous solution (``__shift_solution``) and the plant, shared with the RTI.

All B loops are one ``ipm.solve_batch`` call: B instances of the structured KKT factorisation
(interval interiors by the awelu LU, the 21-stage separator chain by the fused BTD kernels).
"""
from __future__ import annotations

from dataclasses import replace

import numpy as np
import torch

from . import kite3 as k3
from .fd_hessian import FdHessian
from .ipm import IpmOptions, solve_batch
from .rti import BatchedRti


def simulated_reference(loop: BatchedRti, x0: torch.Tensor, u_c: torch.Tensor | None = None) -> torch.Tensor:
    """A dynamically feasible reference window [B, n_v] (scaled): the plant (interval 0's radau
    collocation, ``BatchedRti._plant``) integrated over the horizon from ``x0`` [B, nx] with the
    constant control ``u_c`` [B, nu] (default: zero rates dcoeff = dddl_t = 0 and f_fict = 0, so
    CL, roll and reel acceleration hold their initial values).  The reference's tracking
    references are optimised trajectories, feasible by construction
    (pmpc.py:__create_reference_interpolator); the synthetic circle of kite3.reference_window is
    not a solution of the 3-DOF dynamics without the fictitious forces, so tests that need
    inactive bounds track a simulated window instead."""
    lay, B = loop.lay, loop.B
    nx, st, v0 = k3.NX, lay.interval_stride, lay.v_intervals
    if u_c is None:
        u_c = torch.zeros(B, k3.NU, dtype=torch.float64, device=loop.dev)
    V_save, P_save = loop.V.clone(), loop.P.clone()
    R = torch.zeros(B, lay.n_v, dtype=torch.float64, device=loop.dev)
    R[:, :v0] = loop.V[:, :v0]
    u0 = torch.as_tensor(lay.u(0), device=loop.dev)
    x = x0.clone()
    try:
        for k in range(lay.n_k):
            loop.P[:, lay.p_x0:lay.p_x0 + nx] = x
            loop.V[:, u0] = u_c
            x1, res = loop._plant()
            if float(res.max()) > 1e-9:
                raise RuntimeError(f"plant did not converge on interval {k}: {float(res.max()):.2e}")
            R[:, v0 + k * st:v0 + (k + 1) * st] = loop.plant_V[:, v0:v0 + st]
            R[:, lay.x(k)[0]:lay.x(k)[0] + nx] = x
            loop.V[:, v0:v0 + st] = loop.plant_V[:, v0:v0 + st]          # warm start of the next interval
            x = x1
        R[:, lay.x(lay.n_k)[0]:lay.x(lay.n_k)[0] + nx] = x
    finally:
        loop.V.copy_(V_save)
        loop.P.copy_(P_save)
    return R


# states that enter neither the tether constraint c = (|q|^2 - l_t^2) / 2 nor its derivative
# q.dq - l_t dl_t: CL, roll, reel acceleration
CONSISTENT_X0 = (6, 7, 10)


class BatchedPmpc(BatchedRti):
    """B tracking-MPC closed loops, each sampling time solved to convergence.

    The algebraic variable of the first shooting node is fixed by x0 (the node's dynamics rows
    are square in (xdot[0], z[0])), and the index-reduced tether dynamics turn an x0 that violates
    the tether invariants into a large tether force of either sign; with lambda >= 0 such an
    x0 makes the NLP locally infeasible.  In closed loop x0 comes from the plant and is
    consistent; ``start`` therefore perturbs only the invariant-free states (CONSISTENT_X0)
    unless told otherwise."""

    def start(self, seed: int = 99, sigma: float = 0.01, x0_entries=CONSISTENT_X0):
        super().start(seed=seed, sigma=sigma, x0_entries=x0_entries)

    def __init__(self, consts: k3.Kite3Constants, batch: int, device="cuda", evaluator=None,
                 make_batched=None, plant="collocation", n_fe=20, homotopy_warmstart=True,
                 opts: IpmOptions | None = None, hessian="exact"):
        """``hessian``: "exact" -- the evaluator's own nlp_hess_l (the HIP hyper-dual Hessian kernel,
        IPOPT's default exact Hessian); "fd" -- coloured central differences of the exact gradient
        (fd_hessian.FdHessian, ``make_batched(b)``: an evaluator of the same NLP for b instances, by
        default the HIP MPC evaluator), for evaluators without a Hessian."""
        super().__init__(consts, batch, device=device, evaluator=evaluator, plant=plant, n_fe=n_fe,
                         fix_fict=True)
        if hessian == "exact" and hasattr(self.ev, "eval_hess_device"):
            self.nlp_ev = self.ev
        else:
            if make_batched is None:
                from .mpc import MpcEvaluator

                def make_batched(b):
                    return MpcEvaluator(consts, batch=b)
            self.nlp_ev = FdHessian(self.ev, make_batched, self.lay, device=self.dev, tail=True)
        self.hessian = "exact" if self.nlp_ev is self.ev else "fd"
        self.lbx, self.ubx = k3.variable_bounds(consts, self.lay)
        self.lbg, self.ubg = self.lay.g_bounds()
        self.homotopy_warmstart = homotopy_warmstart
        base = opts or IpmOptions()
        self.pre_opts = replace(base, mu_init=1e-3, mu_target=1e-3, tol=1e-4, max_iter=2)
        self.opts = replace(base, mu_init=1e-3, tol=1e-6)
        self.results = None

    def solve(self):
        """Solve every loop's MPC NLP at the current (V, P); V <- the solutions."""
        P = self.P.cpu().numpy()
        V0 = self.V.cpu().numpy()
        args = (self.lbx, self.ubx, self.lbg, self.ubg)
        if self.homotopy_warmstart:
            pre = solve_batch(self.nlp_ev, P, V0, *args, opts=self.pre_opts, device=self.dev)
            V0 = np.stack([r.x for r in pre])
        res = solve_batch(self.nlp_ev, P, V0, *args, opts=self.opts, device=self.dev)
        self.V.copy_(torch.as_tensor(np.stack([r.x for r in res]), device=self.dev))
        self.results = res
        return res

    def iterate(self):
        """The converged solve in place of one real-time iteration; returns the equality residual
        and the largest path-constraint value at the solution (as BatchedRti.iterate)."""
        self.solve()
        self.ev.eval_nlp_device(self.V, self.P, self.f, self.g, self.grad, self.jac)
        return self.g[:, self.eq_t].abs().amax(dim=1), self.g[:, self.path_t].amax(dim=1)

    def step(self):
        out = super().step()
        out["status"] = [r.status for r in self.results]
        out["iterations"] = np.array([r.iterations for r in self.results])
        return out
