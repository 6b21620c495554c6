"""The interior-point solver's per-iteration measures (ipm.solve_batch): IPOPT's optimality error and
its parts, and the merit pair (theta, phi) of the filter line search.

IPOPT evaluates these in IpIpoptCalculatedQuantities (curr_nlp_error, curr_barrier_obj,
curr_constraint_violation) for the reference's solver (opti/preparation.py:285-323).  Written as
torch operations they are ~130 launches per iteration -- each a few microseconds of host time, and
the converged MPC and the sweeps are host-bound.  On the device one libawelu
launch (``awelu_ipm_measures``: a workgroup per instance) computes the same values in one pass; the
torch composition below stays as the CPU harness's path and as the restatement the kernel is checked
against bitwise (tests/test_ipm_measures_gpu.py): the same operations per entry, every sum in
det.row_sum's order, torch's host-scalar divisions as products with the host reciprocal.

``AWE_IPM_FUSED=0`` selects the torch composition on the device too (A/B measurements)."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import det


class AweluIpmMeasures(ctypes.Structure):
    """include/awelu.h AweluIpmMeasures."""
    _fields_ = [("B", ctypes.c_longlong)] + [(k, ctypes.c_int) for k in ("ny", "n", "m", "mI", "mode")] + \
        [(k, ctypes.c_void_p) for k in ("grad", "jt_lam", "lam", "ineq", "zl", "zu", "y", "yl", "yu", "hl", "hu",
                                        "lo_only", "hi_only", "c", "c_scale", "cs_slack", "eq_row", "gl0", "gu0",
                                        "obj_scale", "f", "mu")] + \
        [(k, ctypes.c_double) for k in ("mu_target", "kappa_d", "s_max", "inv_mnb", "inv_nb", "inv_smax")] + \
        [("out", ctypes.c_void_p)]


class AweluIpmNewton(ctypes.Structure):
    """include/awelu.h AweluIpmNewton."""
    _fields_ = [(k, ctypes.c_int) for k in ("B", "ny", "n", "m", "mI")] + \
        [(k, ctypes.c_void_p) for k in ("y", "yl", "yu", "hl", "hu", "zl", "zu", "grad", "jt_lam", "lam", "c", "ineq",
                                        "lo_only", "hi_only", "mu")] + \
        [("kappa_d", ctypes.c_double)] + [(k, ctypes.c_void_p) for k in ("dl", "du", "sigma", "grad_phi", "rhs")]


class AweluIpmStep(ctypes.Structure):
    """include/awelu.h AweluIpmStep."""
    _fields_ = [(k, ctypes.c_int) for k in ("B", "ny", "m", "any_acc")] + \
        [(k, ctypes.c_void_p) for k in ("y", "y_new", "dy", "lam", "dlam", "zl", "zu", "yl", "yu", "dl_old", "du_old",
                                        "hl", "hu", "acc", "mu", "tau", "alpha")] + \
        [("kappa_sigma", ctypes.c_double)] + \
        [(k, ctypes.c_void_p) for k in ("y_out", "lam_out", "zl_out", "zu_out", "alpha_z")]


HEAD_ROWS = 10      # kkt error, e_dual, e_pr, e_c, unscaled dual / primal / compl, barrier error, theta, phi


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class Measures:
    """The measures of one solve_batch call: B instances, y = [x_free; slacks] of length ny = n + mI,
    m constraint rows (mI of them inequalities with slacks).  ``jt_op``: the solver's fixed-order
    J^T product (ipm._GatherMv)."""

    def __init__(self, nlp, opts, jt_op, dev, n, mI, m, B):
        f64 = dict(dtype=torch.float64, device=dev)
        self.nlp, self.opts, self.jt_op, self.dev = nlp, opts, jt_op, dev
        self.n, self.mI, self.m, self.B = n, mI, m, B
        self.ny = n + mI
        self.hl, self.hu = nlp.has_l, nlp.has_u
        self.lo_only = (self.hl & ~self.hu).to(torch.float64)
        self.hi_only = (self.hu & ~self.hl).to(torch.float64)
        self.damp_dir = self.lo_only - self.hi_only
        self.nb = int(self.hl[0].sum().item() + self.hu[0].sum().item())
        self.cs_slack = nlp.c_scale[:, nlp.ineq_t]
        self.gl0 = torch.tensor(nlp.yl0[n:], **f64)
        self.gu0 = torch.tensor(nlp.yu0[n:], **f64)
        self.eq_mask = torch.ones(m, dtype=torch.bool, device=dev)
        self.eq_mask[nlp.ineq_t] = False
        self.fused = torch.device(dev).type == "cuda" and os.environ.get("AWE_IPM_FUSED", "1") != "0"
        if self.fused:
            # the masks per instance are equal (one structure); the kernel reads row 0's
            self._lo = self.lo_only[0].contiguous()
            self._hi = self.hi_only[0].contiguous()
            if not (torch.equal(self.lo_only, self._lo.expand_as(self.lo_only))
                    and torch.equal(self.hi_only, self._hi.expand_as(self.hi_only))):
                raise ValueError("bound masks differ between instances")
            self._hl = self.hl.contiguous()
            self._hu = self.hu.contiguous()
            self._ineq = nlp.ineq_t.to(torch.int64).contiguous()
            self._eq = self.eq_mask.to(torch.uint8).contiguous()
            self._cs = self.cs_slack.contiguous()
            self._cscale = nlp.c_scale.contiguous()
            from .batched_lu import load_library
            self._lib = load_library()
            self._lib.awelu_ipm_measures.argtypes = [ctypes.POINTER(AweluIpmMeasures), ctypes.c_void_p]
            self._lib.awelu_ipm_newton.argtypes = [ctypes.POINTER(AweluIpmNewton), ctypes.c_void_p]
            self._lib.awelu_ipm_step.argtypes = [ctypes.POINTER(AweluIpmStep), ctypes.c_void_p]

    # ---- device kernel ---------------------------------------------------------------------------
    def _launch(self, mode, y, c, f, mu, grad=None, jt_lam=None, lam=None, zl=None, zu=None):
        nlp, o = self.nlp, self.opts
        rows = HEAD_ROWS if mode == 0 else 2
        out = torch.empty(rows, self.B, dtype=torch.float64, device=self.dev)
        keep = [t.contiguous() if t is not None else None for t in (y, c, f, mu, grad, jt_lam, lam, zl, zu)]
        y, c, f, mu, grad, jt_lam, lam, zl, zu = keep
        for t, shape in ((y, (self.B, self.ny)), (c, (self.B, self.m)), (f, (self.B,)), (mu, (self.B,)),
                         (grad, (self.B, self.n)), (jt_lam, (self.B, self.ny)), (lam, (self.B, self.m)),
                         (zl, (self.B, self.ny)), (zu, (self.B, self.ny))):
            if t is not None and (tuple(t.shape) != shape or t.dtype != torch.float64 or not t.is_cuda):
                raise ValueError(f"ipm measures: operand {tuple(t.shape)} {t.dtype}, expected {shape} float64 on the device")
        a = AweluIpmMeasures(
            B=self.B, ny=self.ny, n=self.n, m=self.m, mI=self.mI, mode=mode,
            grad=_ptr(grad), jt_lam=_ptr(jt_lam), lam=_ptr(lam), ineq=_ptr(self._ineq),
            zl=_ptr(zl), zu=_ptr(zu), y=_ptr(y), yl=_ptr(nlp.yl), yu=_ptr(nlp.yu), hl=_ptr(self._hl), hu=_ptr(self._hu),
            lo_only=_ptr(self._lo), hi_only=_ptr(self._hi), c=_ptr(c), c_scale=_ptr(self._cscale),
            cs_slack=_ptr(self._cs), eq_row=_ptr(self._eq), gl0=_ptr(self.gl0), gu0=_ptr(self.gu0),
            obj_scale=_ptr(nlp.obj_scale), f=_ptr(f), mu=_ptr(mu),
            mu_target=o.mu_target, kappa_d=o.kappa_d, s_max=o.s_max,
            inv_mnb=1.0 / max(1, self.m + self.nb), inv_nb=1.0 / max(1, self.nb), inv_smax=1.0 / o.s_max,
            out=_ptr(out))
        s = torch.cuda.current_stream(self.dev).cuda_stream
        if self._lib.awelu_ipm_measures(ctypes.byref(a), ctypes.c_void_p(s)) != 0:
            raise RuntimeError(f"awelu_ipm_measures: {self._lib.awelu_last_error().decode()}")
        return out

    def _check(self, rc, name):
        if rc != 0:
            raise RuntimeError(f"{name}: {self._lib.awelu_last_error().decode()}")

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def _dev_mask(self, a):
        """A host [B] bool array as a device uint8 tensor (pinned, asynchronous)."""
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8))
        return t.pin_memory().to(self.dev, non_blocking=True)

    def _dev_vec(self, a):
        t = torch.from_numpy(np.array(a, dtype=np.float64))
        return t.pin_memory().to(self.dev, non_blocking=True)

    # ---- the solver's calls ----------------------------------------------------------------------
    def head(self, grad, jv, c, y, lam, zl, zu, f, mu_head):
        """[10, B] device tensor: the scaled error at mu_target with its parts (rows 0-3), the
        unscaled dual / primal / complementarity tests (4-6), the barrier problem's error at
        ``mu_head`` (7), theta (8) and phi at ``mu_head`` (9)."""
        if self.fused:
            return self._launch(0, y, c, f, mu_head, grad=grad, jt_lam=self.jt_op.mv(jv, lam), lam=lam, zl=zl, zu=zu)
        mu_t = torch.full((self.B,), self.opts.mu_target, dtype=torch.float64, device=self.dev)
        return torch.stack(self.errors_torch(grad, jv, c, y, lam, zl, zu, mu_t, unscaled=True) +
                           [self.errors_torch(grad, jv, c, y, lam, zl, zu, mu_head, damped=True)[0],
                            det.row_sum(c.abs()), self.barrier_phi_torch(f, y, mu_head)])

    def barrier_error(self, grad, jv, c, y, lam, zl, zu, f, mu):
        """The barrier problem's error at ``mu`` per instance (host [B])."""
        if self.fused:
            return self.head(grad, jv, c, y, lam, zl, zu, f, mu)[7].cpu().numpy()
        return self.errors_torch(grad, jv, c, y, lam, zl, zu, mu, damped=True)[0].cpu().numpy()

    def merit(self, c, f, y, mu):
        """[2, B] device tensor: theta = ||c||_1 and the barrier function phi at ``mu``."""
        if self.fused:
            return self._launch(1, y, c, f, mu)
        return torch.stack([det.row_sum(c.abs()), self.barrier_phi_torch(f, y, mu)])

    def newton(self, grad, jv, c, y, lam, zl, zu, mu):
        """(dl, du, sigma, grad_phi, rhs) of the Newton system at the iterate, ``mu`` a [B] device
        tensor: the bound gaps, the barrier diagonal, the barrier gradient and the right-hand side
        [-(grad phi + A^T lam); -c] ([B, ny + m])."""
        if not self.fused:
            return self.newton_torch(grad, jv, c, y, lam, zl, zu, mu)
        B, ny, m = self.B, self.ny, self.m
        f64 = dict(dtype=torch.float64, device=self.dev)
        jt = self.jt_op.mv(jv, lam)
        y, zl, zu, grad, lam, c, mu = (t.contiguous() for t in (y, zl, zu, grad, lam, c, mu))
        dl, du, sigma, gp = (torch.empty(B, ny, **f64) for _ in range(4))
        rhs = torch.empty(B, ny + m, **f64)
        a = AweluIpmNewton(B=B, ny=ny, n=self.n, m=m, mI=self.mI, y=_ptr(y), yl=_ptr(self.nlp.yl), yu=_ptr(self.nlp.yu),
                           hl=_ptr(self._hl), hu=_ptr(self._hu), zl=_ptr(zl), zu=_ptr(zu), grad=_ptr(grad),
                           jt_lam=_ptr(jt), lam=_ptr(lam), c=_ptr(c), ineq=_ptr(self._ineq), lo_only=_ptr(self._lo),
                           hi_only=_ptr(self._hi), mu=_ptr(mu), kappa_d=self.opts.kappa_d, dl=_ptr(dl), du=_ptr(du),
                           sigma=_ptr(sigma), grad_phi=_ptr(gp), rhs=_ptr(rhs))
        self._check(self._lib.awelu_ipm_newton(ctypes.byref(a), self._stream()), "awelu_ipm_newton")
        return dl, du, sigma, gp, rhs

    def step(self, acc, y, y_new, dy, lam, dlam, zl, zu, dl, du, mu, tau, alpha, restore=None):
        """The accepted step and the kappa_sigma safeguard: (y, lam, zl, zu, alpha_z) after the
        iteration.  ``acc`` host [B] bool (stepped instances), ``alpha`` host [B] primal step lengths,
        ``dl``, ``du`` the Newton system's gaps, ``mu``, ``tau`` [B] device tensors; ``restore`` =
        (host mask, (y, lam, zl, zu) of the watchdog's start) returns those instances there before
        the safeguard (the torch composition then)."""
        if not self.fused or restore is not None:
            return self.step_torch(acc, y, y_new, dy, lam, dlam, zl, zu, dl, du, mu, tau, alpha, restore)
        B, ny, m = self.B, self.ny, self.m
        f64 = dict(dtype=torch.float64, device=self.dev)
        any_acc = bool(np.any(acc))
        y, y_new, dy, lam, dlam, zl, zu, mu, tau = (t.contiguous() for t in (y, y_new, dy, lam, dlam, zl, zu, mu, tau))
        acc_d = self._dev_mask(acc)
        al = self._dev_vec(alpha)
        y_o, zl_o, zu_o = (torch.empty(B, ny, **f64) for _ in range(3))
        lam_o = torch.empty(B, m, **f64) if any_acc else lam
        az = torch.empty(B, **f64)
        a = AweluIpmStep(B=B, ny=ny, m=m, any_acc=int(any_acc), y=_ptr(y), y_new=_ptr(y_new), dy=_ptr(dy), lam=_ptr(lam),
                         dlam=_ptr(dlam), zl=_ptr(zl), zu=_ptr(zu), yl=_ptr(self.nlp.yl), yu=_ptr(self.nlp.yu),
                         dl_old=_ptr(dl.contiguous()), du_old=_ptr(du.contiguous()), hl=_ptr(self._hl), hu=_ptr(self._hu),
                         acc=_ptr(acc_d), mu=_ptr(mu), tau=_ptr(tau), alpha=_ptr(al), kappa_sigma=self.opts.kappa_sigma,
                         y_out=_ptr(y_o), lam_out=_ptr(lam_o), zl_out=_ptr(zl_o), zu_out=_ptr(zu_o), alpha_z=_ptr(az))
        self._check(self._lib.awelu_ipm_step(ctypes.byref(a), self._stream()), "awelu_ipm_step")
        return y_o, lam_o, zl_o, zu_o, az

    # ---- the torch composition (the CPU harness; the kernel's restatement) --------------------------
    def newton_torch(self, grad, jv, c, y, lam, zl, zu, mu_d):
        hl, hu, B, mI = self.hl, self.hu, self.B, self.mI
        dl, du = self.gaps(y)
        sigma = torch.where(hl, zl / dl, torch.zeros_like(y)) + torch.where(hu, zu / du, torch.zeros_like(y))
        grad_y = torch.cat([grad, torch.zeros(B, mI, dtype=torch.float64, device=grad.device)], 1)
        grad_phi = grad_y - torch.where(hl, mu_d[:, None] / dl, torch.zeros_like(y)) + \
            torch.where(hu, mu_d[:, None] / du, torch.zeros_like(y)) + self.opts.kappa_d * mu_d[:, None] * self.damp_dir
        rhs_top = -(grad_phi + self.A_T_lam(jv, lam))
        return dl, du, sigma, grad_phi, torch.cat([rhs_top, -c], 1)

    def ftb(self, v, dv, mask_pos, tau_t):
        """Fraction-to-the-boundary step per instance on the device: min_i -tau v_i / dv_i ([B])."""
        ratio = torch.where(mask_pos & (dv < 0), -tau_t[:, None] * v / dv, torch.full_like(v, float("inf")))
        return ratio.amin(1) if ratio.shape[1] else torch.full((self.B,), float("inf"), dtype=torch.float64,
                                                               device=v.device)

    def step_torch(self, acc, y, y_new, dy, lam, dlam, zl, zu, dl, du, mu_d, tau_d, alpha, restore=None):
        hl, hu, B, opts = self.hl, self.hu, self.B, self.opts
        f64 = dict(dtype=torch.float64, device=y.device)
        dev_m = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=bool)).to(y.device)  # noqa: E731
        if np.any(acc):
            sel = dev_m(acc)[:, None]
            dzl = torch.where(hl, mu_d[:, None] / dl - zl - zl / dl * dy, torch.zeros_like(y))
            dzu = torch.where(hu, mu_d[:, None] / du - zu + zu / du * dy, torch.zeros_like(y))
            az_dev = torch.minimum(torch.minimum(self.ftb(zl, dzl, hl, tau_d), self.ftb(zu, dzu, hu, tau_d)),
                                   torch.ones(B, **f64))
            az = torch.where(dev_m(acc), az_dev, torch.zeros_like(az_dev))[:, None]
            y = torch.where(sel, y_new, y)
            lam = lam + torch.tensor(np.where(acc, alpha, 0.0), **f64)[:, None] * dlam
            zl = zl + az * dzl
            zu = zu + az * dzu
        else:
            az_dev = torch.zeros(B, **f64)
        if restore is not None:
            # the watchdog failed: the iterate returns to its starting point
            selr = dev_m(restore[0])[:, None]
            y, lam, zl, zu = (torch.where(selr, r, t) for t, r in zip((y, lam, zl, zu), restore[1]))
        dl, du = self.gaps(y)
        zl = torch.where(hl, torch.clamp(zl, min=mu_d[:, None] / (opts.kappa_sigma * dl),
                                         max=opts.kappa_sigma * mu_d[:, None] / dl), zl)
        zu = torch.where(hu, torch.clamp(zu, min=mu_d[:, None] / (opts.kappa_sigma * du),
                                         max=opts.kappa_sigma * mu_d[:, None] / du), zu)
        return y, lam, zl, zu, az_dev

    def gaps(self, yv):
        dl = torch.where(self.hl, yv - self.nlp.yl, torch.ones_like(yv))
        du = torch.where(self.hu, self.nlp.yu - yv, torch.ones_like(yv))
        return dl, du

    def barrier_phi_torch(self, fv, yv, mu_t):
        """phi = f - mu sum log(gaps) + kappa_d mu (damping of one-sided bounds) per instance: IPOPT's
        barrier objective with its kappa_d damping."""
        hl, hu = self.hl, self.hu
        dl, du = self.gaps(yv)
        lg = det.row_sum(torch.where(hl, torch.log(dl), torch.zeros_like(dl))) + \
            det.row_sum(torch.where(hu, torch.log(du), torch.zeros_like(du)))
        dmp = det.row_sum(self.lo_only * dl) + det.row_sum(self.hi_only * du)
        return fv - mu_t * lg + self.opts.kappa_d * mu_t * dmp

    def A_T_lam(self, jvv, lamv):
        r = self.jt_op.mv(jvv, lamv)
        r[:, self.n:] -= lamv[:, self.nlp.ineq_t]
        return r

    def errors_torch(self, gradv, jvv, cv, yv, lamv, zlv, zuv, mu_t, damped=False, unscaled=False):
        """IPOPT's scaled optimality error per instance ([B] device tensors): total, dual, primal,
        complementarity at barrier parameter mu_t ([B] tensor); ``damped`` adds the kappa_d term
        (the barrier problem's error).  With ``unscaled`` also the unscaled dual infeasibility,
        constraint violation (original bounds of the inequality rows) and complementarity that
        IPOPT's termination tests compare with dual_inf_tol / constr_viol_tol / compl_inf_tol."""
        nlp, opts, n, mI, m, B, nb = self.nlp, self.opts, self.n, self.mI, self.m, self.B, self.nb
        hl, hu = self.hl, self.hu
        f64 = dict(dtype=torch.float64, device=self.dev)
        dl, du = self.gaps(yv)
        dual = torch.cat([gradv, torch.zeros(B, mI, **f64)], 1) + self.A_T_lam(jvv, lamv) - zlv + zuv
        if damped:
            dual = dual + opts.kappa_d * mu_t[:, None] * self.damp_dir
        compl_l = torch.where(hl, dl * zlv - mu_t[:, None], torch.zeros_like(yv))
        compl_u = torch.where(hu, du * zuv - mu_t[:, None], torch.zeros_like(yv))
        zsum = det.row_sum(zlv.abs()) + det.row_sum(zuv.abs())
        s_d = torch.clamp((det.row_sum(lamv.abs()) + zsum) / max(1, m + nb), min=opts.s_max) / opts.s_max
        s_c = torch.clamp(zsum / max(1, nb), min=opts.s_max) / opts.s_max
        e_dual = dual.abs().amax(1) / s_d
        e_pr = cv.abs().amax(1) if m else torch.zeros(B, **f64)
        compl = torch.maximum(compl_l.abs().amax(1), compl_u.abs().amax(1))
        e_c = compl / s_c
        parts = [torch.maximum(torch.maximum(e_dual, e_pr), e_c), e_dual, e_pr, e_c]
        if unscaled:
            osc = nlp.obj_scale
            cs_slack = self.cs_slack
            u_dual = torch.maximum(dual[:, :n].abs().amax(1) if n else torch.zeros(B, **f64),
                                   (dual[:, n:] * cs_slack).abs().amax(1) if mI else torch.zeros(B, **f64)) / osc
            c_u = cv / nlp.c_scale
            u_pr = torch.where(self.eq_mask, c_u.abs(), torch.zeros_like(c_u)).amax(1) if m else torch.zeros(B, **f64)
            if mI:
                gI = (cv[:, nlp.ineq_t] + yv[:, n:]) / cs_slack         # g of the inequality rows, unscaled
                vI = torch.maximum(torch.where(torch.isfinite(self.gu0), gI - self.gu0, torch.zeros_like(gI)),
                                   torch.where(torch.isfinite(self.gl0), self.gl0 - gI, torch.zeros_like(gI)))
                u_pr = torch.maximum(u_pr, torch.clamp(vI, min=0.0).amax(1))
            parts += [u_dual, u_pr, compl / osc]
        return parts
