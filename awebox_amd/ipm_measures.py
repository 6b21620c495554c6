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

    # ---- the torch composition (the CPU harness; the kernel's restatement) --------------------------
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
