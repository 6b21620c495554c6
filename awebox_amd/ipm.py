"""Primal-dual interior-point NLP solver on the GPU.

The reference hands the collocation NLP to IPOPT through ``casadi.nlpsol`` (opti/preparation.py:
366-400) and drives it through the homotopy (opti/optimization.py:273-382).  IPOPT is not
available here, so this module restates the IPOPT algorithm (Waechter & Biegler, Math. Prog.
106, 2006) at the level the AP2 problem needs, with every piece of data on the device:

* NLP functions, gradient, Jacobian and the exact Hessian of the Lagrangian come from the HIP
  evaluator (awebox_amd.evaluator) on device tensors;
* B instances of one NLP structure (sweep points, homotopy runs) are solved side by side
  (solve_batch): each keeps its own IPOPT iteration, while evaluations, Hessians and KKT
  factorisations are batched;
* the primal-dual KKT system [W + Sigma + dw I, A^T; A, -dc I] is solved by structured
  elimination (StructuredKKT: batched LU of the interval interiors on the awelu kernel, a dense
  or block-tridiagonal Schur complement on the separators), assembled in a fixed summation order
  (deterministic gather-sum tables); IPOPT's inertia correction gets the exact inertia of K from
  Bunch-Kaufman counts of the interval blocks and the separator pivot blocks (Haynsworth
  additivity); the curvature test of Chiang & Zavala (2016) remains as an option;
* fixed variables (lbx == ubx) are removed (IPOPT's fixed_variable_treatment=make_parameter);
  inequality rows get slacks; gradient-based NLP scaling, bound push, monotone Fiacco-McCormick
  barrier update, fraction-to-the-boundary rule and the filter line search follow IPOPT's
  defaults (tol 1e-8, mu_init 0.1, kappa_mu 0.2, theta_mu 1.5, tau_min 0.99);
* second-order corrections in the line search (max_soc 4, kappa_soc 0.99);
* after a failed line search: a retry with stronger regularisation, then a reduced feasibility
  restoration (Gauss-Newton steps on ||c|| inside the bounds until the filter accepts) followed
  by least-squares constraint multipliers.

* IPOPT's watchdog: after 10 consecutive shortened steps, up to 3 full steps judged against the
  watchdog's starting point, then back to that point with a backtracking line search;

What is left out: IPOPT's full restoration-phase NLP and quasi-Newton options.
"""
from __future__ import annotations

import math
import os
import time
import weakref
from dataclasses import dataclass, field

import numpy as np
import torch

from . import det
from .ipm_measures import Measures
from . import problem as pb


@dataclass
class IpmOptions:
    tol: float = 1e-8
    acceptable_tol: float = 1e-6
    max_iter: int = 1000
    mu_init: float = 0.1
    mu_target: float = 0.0           # barrier parameter floor; convergence is measured at it
    warm_start_bound_push: float = 1e-3
    warm_start_mult_bound_push: float = 1e-3
    kappa_eps: float = 10.0
    kappa_mu: float = 0.2
    theta_mu: float = 1.5
    tau_min: float = 0.99
    kappa_sigma: float = 1e10
    bound_push: float = 1e-2
    bound_frac: float = 1e-2
    s_max: float = 100.0
    nlp_scaling_max_gradient: float = 100.0
    delta_w0: float = 1e-4
    delta_w_min: float = 1e-20
    delta_w_max: float = 1e40
    delta_c: float = 1e-8
    curvature_kappa: float = 1e-8
    gamma_theta: float = 1e-5
    gamma_phi: float = 1e-8
    delta_switch: float = 1.0
    s_theta: float = 1.1
    s_phi: float = 2.3
    eta_phi: float = 1e-8
    alpha_min_frac: float = 0.05
    max_backtracks: int = 40
    max_soc: int = 4                 # second-order corrections per line search (IPOPT max_soc)
    kappa_soc: float = 0.99
    # IPOPT's watchdog (Chamberlain et al.'s technique as IPOPT's BacktrackingLineSearch applies it):
    # after this many consecutive iterations whose accepted step was shortened by the line search, the
    # next full steps are taken without backtracking, each judged against the point where the
    # watchdog started; accepted -> the watchdog ends, after watchdog_trial_iter_max failures the
    # iterate returns to that point and its line search backtracks (0: off)
    watchdog_shortened_iter_trigger: int = 10
    watchdog_trial_iter_max: int = 3
    # IPOPT's bound relaxation: every finite bound of a free variable or an inequality row moves
    # outward by min(constr_viol_tol, bound_relax_factor max(1, |b|)) before the solve
    bound_relax_factor: float = 1e-8
    kappa_d: float = 1e-5            # linear damping of variables bounded on one side only
    constr_mult_init_max: float = 1e3  # cold start: least-square multipliers unless larger than this
    # IPOPT's termination tests beyond the scaled error (unscaled quantities) and its
    # "acceptable" termination after acceptable_iter consecutive acceptable iterations
    constr_viol_tol: float = 1e-4
    dual_inf_tol: float = 1.0
    compl_inf_tol: float = 1e-4
    acceptable_iter: int = 15
    acceptable_constr_viol_tol: float = 1e-2
    acceptable_dual_inf_tol: float = 1e10
    acceptable_compl_inf_tol: float = 1e-2
    lu_backend: str = "awelu"        # interval-block LU: "awelu" (batched_lu.hip) or "torch" (rocSOLVER)
    separators: str = "btd"          # separator system: "dense" LU or "btd" (awebox_amd/btd.py block sweep)
    inertia: str = "exact"           # inertia correction: "curvature" test (Chiang & Zavala) or "exact" (IPOPT:
                                     # In(K) = In(K_II) + In(S) from symmetric eigenvalues of the blocks)
    profile: bool = False            # synchronise and time the solver's phases (IpmResult.timing)
    verbose: bool = False
    callback: object = None          # callback(iteration, V [B, n_v] device tensor, stepped [B] bool)


@dataclass
class IpmResult:
    x: np.ndarray            # full V
    lam_g: np.ndarray
    f: float
    status: str
    iterations: int
    kkt_error: float
    constr_viol: float
    seconds: float
    zl: np.ndarray = None    # bound multipliers on V (lower / upper), for warm starts
    zu: np.ndarray = None
    log: list = field(default_factory=list)
    kkt_solves: int = 0      # linear solves, and how many fell back to a dense LU (structured KKT)
    kkt_dense: int = 0
    timing: dict = field(default_factory=dict)   # seconds per phase when IpmOptions.profile


class DeviceNlp:
    """Evaluator-backed NLP restricted to the free variables, with slacks for inequality rows, for
    B instances at once (the evaluator's batch): same structure (free set, inequality rows,
    bounds), per-instance P and scaling."""

    def __init__(self, ev, P, lbx, ubx, lbg, ubg, device, relax=0.0, relax_cap=1e-4):
        self.ev, self.dev = ev, device
        n_v, n_g = ev.n_v, ev.n_g
        P = np.atleast_2d(np.asarray(P, dtype=np.float64))
        self.B = B = P.shape[0]
        self.P = torch.tensor(P, device=device)
        lbx, ubx = np.asarray(lbx, dtype=np.float64), np.asarray(ubx, dtype=np.float64)
        self.fixed = lbx >= ubx
        self.free = np.where(~self.fixed)[0]
        self.n = len(self.free)
        self.x_fix = np.where(self.fixed, lbx, 0.0)
        lbg, ubg = np.asarray(lbg, dtype=np.float64), np.asarray(ubg, dtype=np.float64)
        self.ineq = np.where(lbg < ubg)[0]
        self.eq = np.where(lbg >= ubg)[0]
        self.m, self.mI = n_g, len(self.ineq)
        self.g_target = torch.tensor(np.where(lbg >= ubg, lbg, 0.0), device=device)
        # bounds of y = [x_free; s] (slack bounds are scaled per instance once c_scale is known)
        yl = np.concatenate([lbx[self.free], lbg[self.ineq]])
        yu = np.concatenate([ubx[self.free], ubg[self.ineq]])
        # the original bounds (reported violations), then IPOPT's bound relaxation
        # (TNLPAdapter: fixed variables and equality rows are not relaxed)
        self.yl0, self.yu0 = yl.copy(), yu.copy()
        if relax > 0.0:
            with np.errstate(invalid="ignore"):
                yl = np.where(np.isfinite(yl), yl - np.minimum(relax_cap, relax * np.maximum(1.0, np.abs(yl))), yl)
                yu = np.where(np.isfinite(yu), yu + np.minimum(relax_cap, relax * np.maximum(1.0, np.abs(yu))), yu)
        self.yl = torch.tensor(np.tile(yl, (B, 1)), device=device)
        self.yu = torch.tensor(np.tile(yu, (B, 1)), device=device)
        self.has_l = torch.isfinite(self.yl)
        self.has_u = torch.isfinite(self.yu)
        self.ny = self.n + self.mI
        # reduced patterns
        col_map = -np.ones(n_v, dtype=np.int64)
        col_map[self.free] = np.arange(self.n)
        colind, row = ev.sparsity_jac()
        jcol = np.repeat(np.arange(n_v), np.diff(colind))
        keep = col_map[jcol] >= 0
        self.j_keep = torch.tensor(np.where(keep)[0], device=device)
        self.j_row = torch.tensor(row[keep].astype(np.int64), device=device)
        self.j_col = torch.tensor(col_map[jcol[keep]], device=device)
        hcolind, hrow = ev.sparsity_hess()
        hcol = np.repeat(np.arange(n_v), np.diff(hcolind))
        hk = (col_map[hcol] >= 0) & (col_map[hrow] >= 0)
        self.h_keep = torch.tensor(np.where(hk)[0], device=device)
        self.h_r = torch.tensor(col_map[hrow[hk]], device=device)
        self.h_c = torch.tensor(col_map[hcol[hk]], device=device)
        self.h_offdiag = self.h_r != self.h_c
        self.s_row = torch.tensor(self.ineq.astype(np.int64), device=device)
        # device buffers of the evaluator
        f64 = dict(dtype=torch.float64, device=device)
        self.V = torch.tensor(np.tile(self.x_fix, (B, 1)), device=device)
        self.f = torch.zeros(B, **f64)
        self.g = torch.zeros(B, n_g, **f64)
        self.grad = ev.alloc_grad(device) if hasattr(ev, "alloc_grad") else torch.zeros(B, n_v, **f64)
        # J_g in the evaluator's instance-minor layout where it has one (the AP2 evaluator writes it
        # with coalesced stores, awe_eval_nlp_im); a [B, nnz] view either way
        self.jac = ev.alloc_jac(device) if hasattr(ev, "alloc_jac") else torch.zeros(B, ev.nnz, **f64)
        # H instance-minor where the evaluator's Hessian kernel writes it that way (the generated
        # Hessian, awe_eval_hess_im); per instance for the hyper-dual kernels
        self.h_im = getattr(ev, "hess_path", None) == "generated" and hasattr(ev, "alloc_hess")
        self.H = ev.alloc_hess(device) if self.h_im else torch.zeros(B, ev.nnz_h, **f64)
        self.sig = torch.ones(B, **f64)
        self.free_t = torch.tensor(self.free, device=device)
        self.ineq_t = torch.tensor(self.ineq, device=device)
        self.obj_scale = torch.ones(B, **f64)
        self.c_scale = torch.ones(B, n_g, **f64)

    def full_x(self, x):
        self.V[:, self.free_t] = x
        return self.V

    def eval_all(self, x):
        """f [B], grad_f (reduced) [B, n], g [B, m] and the Jacobian values (reduced, scaled)."""
        self.ev.eval_nlp_device(self.full_x(x), self.P, self.f, self.g, self.grad, self.jac)
        f = self.f * self.obj_scale
        grad = self.grad[:, self.free_t] * self.obj_scale[:, None]
        g = self.g * self.c_scale
        jv = self.jac[:, self.j_keep] * self.c_scale[:, self.j_row]
        return f, grad, g, jv

    def eval_fg(self, x):
        self.ev.eval_nlp_device(self.full_x(x), self.P, self.f, self.g, self.grad, self.jac)
        return self.f * self.obj_scale, self.g * self.c_scale

    def hess(self, x, lam):
        """Hessian of obj_scale f + (c_scale lam)^T g, reduced upper values [B, nH]."""
        lam_unscaled = (lam * self.c_scale).contiguous()
        self.sig.copy_(self.obj_scale)
        if self.h_im:
            self.ev.eval_hess_device_im(self.full_x(x), self.P, self.sig, lam_unscaled, self.H)
        else:
            self.ev.eval_hess_device(self.full_x(x), self.P, self.sig, lam_unscaled, self.H)
        return self.H[:, self.h_keep]

    def constraints(self, g, s):
        """c(y) = [g_E - target; g_I - s] (scaled rows), [B, m]."""
        c = g - self.g_target * self.c_scale
        c[:, self.ineq_t] = c[:, self.ineq_t] - s
        return c


class _ScatterSum:
    """out[..., dst[i]] += vals[..., i] for a fixed index pattern, deterministically and without
    atomics: the duplicates of every destination are pre-grouped on the host into gather tables
    (one per power-of-two bucket of the multiplicity, padding -> a zero slot), and each table row is
    summed as one fixed-order reduction instead of index_put_(accumulate=True) / index_add_, whose
    atomics add duplicates in a run-dependent order (the homotopy path is
    sensitive to that roundoff).  Leading (batch) dimensions of ``out`` and ``vals`` are kept.

    On the GPU every bucket up to width 64 goes through one launch of libawelu's gather-sum
    kernel (awelu_gather_sum: lists in lanes, adjacent-pair shuffle trees -- bitwise the gather,
    row sum and indexed add that torch performs per bucket, ~5 launches each); the wider buckets (the
    few long rows, e.g. t_f's column of J) go through a second launch (awelu_gather_sum_wide) that sums
    each list in det.row_sum's order -- bitwise torch's gather, row sum and indexed add for them."""

    NATIVE_MAX_W = 64

    def __init__(self, dst, dev):
        dst = np.asarray(dst, dtype=np.int64).reshape(-1)
        self.n_src = len(dst)
        self.dev = torch.device(dev)
        order = np.argsort(dst, kind="stable")
        uniq, start, count = np.unique(dst[order], return_index=True, return_counts=True)
        self.buckets = []                                       # (dst, table) on the device, all widths
        narrow = []                                             # host tables of width <= 64
        wide_h = []                                             # host tables wider than 64
        lo, width = 0, 1
        while lo < (count.max() if len(count) else 0):
            sel = np.where((count > lo) & (count <= width))[0]
            if len(sel):
                # row u of the table: the sources of destination uniq[sel[u]] in order, padded
                cnt, st = count[sel], start[sel]
                wi = np.arange(width)
                has = wi[None, :] < cnt[:, None]
                table = np.full((len(sel), width), len(dst), dtype=np.int64)
                table[has] = order[(st[:, None] + wi[None, :])[has]]
                self.buckets.append((torch.tensor(uniq[sel], device=dev), torch.tensor(table, device=dev)))
                if width <= self.NATIVE_MAX_W:
                    narrow.append((uniq[sel], table))
                else:
                    wide_h.append((uniq[sel], table))
            lo, width = width, 2 * width
        self.wide = [(d, t) for d, t in self.buckets if t.shape[1] > self.NATIVE_MAX_W]
        # AWE_NATIVE_GATHER_SUM=0: the torch reduction everywhere (A/B measurements)
        self.native = self.dev.type == "cuda" and os.environ.get("AWE_NATIVE_GATHER_SUM", "1") != "0"
        self._sel_lanes = {}
        self.lanes_host = self.build_lanes(narrow, len(dst))
        if self.native:
            lsrc, lw, ldst = self.lanes_host
            self.lsrc = torch.tensor(lsrc.astype(np.int32), device=dev)
            self.lw = torch.tensor(lw, device=dev)
            self.ldst = torch.tensor(ldst.astype(np.int32), device=dev)
        # the wide lists in one launch too (awelu_gather_sum_wide, det.row_sum's order);
        # AWE_NATIVE_WIDE=0: torch's gather + row sum for them (A/B measurements)
        self.native_wide = self.native and bool(wide_h) and os.environ.get("AWE_NATIVE_WIDE", "1") != "0"
        if self.native_wide:
            wsrc = np.concatenate([np.where(t == len(dst), -1, t).reshape(-1) for _, t in wide_h])
            ww = np.concatenate([np.full(t.shape[0], t.shape[1]) for _, t in wide_h])
            self.wsrc_host = wsrc
            self.wsrc = torch.tensor(wsrc.astype(np.int32), device=dev)
            self.ww = torch.tensor(ww.astype(np.int32), device=dev)
            self.woff = torch.tensor(np.concatenate([[0], np.cumsum(ww)[:-1]]).astype(np.int32), device=dev)
            self.wdst = torch.tensor(np.concatenate([d for d, _ in wide_h]).astype(np.int32), device=dev)

    @staticmethod
    def build_lanes(narrow, n_src):
        """(lsrc, lw, ldst) host arrays of awelu_gather_sum for the buckets [(dst, table)] of width
        <= 64: widest bucket first, so every list starts at a multiple of its width; padding
        (table entry n_src) -> source -1; the destination on a list's first lane."""
        lsrc, lw, ldst = [np.zeros(0, np.int64)], [np.zeros(0, np.uint8)], [np.zeros(0, np.int64)]
        for d, table in sorted(narrow, key=lambda b: -b[1].shape[1]):
            n_u, w = table.shape
            lsrc.append(np.where(table == n_src, -1, table).reshape(-1))
            lw.append(np.full(n_u * w, w, dtype=np.uint8))
            dd = np.full((n_u, w), -1, dtype=np.int64)
            dd[:, 0] = d
            ldst.append(dd.reshape(-1))
        return np.concatenate(lsrc), np.concatenate(lw), np.concatenate(ldst)

    # --- the torch reduction (host tensors, and the buckets wider than 64) ------------------------
    def _torch_buckets(self, out, vals, buckets):
        """The gather-sums by torch indexing, in the kernels' orders: a list of width <= 64 as the
        adjacent-pair tree of awelu_gather_sum, a wider one in det.row_sum's order (awelu_row_sum on
        the device).  Neither depends on the leading (batch) shape."""
        ext = torch.cat([vals, vals.new_zeros(vals.shape[:-1] + (1,))], dim=-1)
        for d, table in buckets:
            g = ext[..., table]
            out[..., d] += det.tree_sum(g) if table.shape[1] <= self.NATIVE_MAX_W else det.row_sum(g)
        return out

    def _native_ok(self, out, vals, x=None):
        """The kernel's contract: float64 device tensors, ``out`` contiguous (written in place),
        the same leading shape everywhere, at most 65,535 rows (vals and x are made contiguous by
        an exact copy where needed)."""
        return (self.native and out.is_cuda and out.dtype == torch.float64 and vals.dtype == torch.float64
                and out.is_contiguous() and out.shape[:-1] == vals.shape[:-1] and out.numel() // max(1, out.shape[-1]) <= 65535
                and (x is None or (x.dtype == torch.float64 and x.shape[:-1] == out.shape[:-1])))

    def _launch(self, out, vals, lsrc, x=None, cols=None):
        from .batched_lu import gather_sum
        rows = out.numel() // max(1, out.shape[-1]) if out.dim() > 1 else 1
        gather_sum(lsrc, self.lw, self.ldst, vals.contiguous(), out, rows,
                   x=x.contiguous() if x is not None else None, cols=cols)

    def _launch_wide(self, out, vals, wsrc, x=None, cols=None):
        from .batched_lu import gather_sum_wide
        rows = out.numel() // max(1, out.shape[-1]) if out.dim() > 1 else 1
        gather_sum_wide(wsrc, self.woff, self.ww, self.wdst, vals.contiguous(), out, rows,
                        x=x.contiguous() if x is not None else None, cols=cols)

    def add_into(self, out, vals):
        if not self._native_ok(out, vals):
            return self._torch_buckets(out, vals, self.buckets)
        self._launch(out, vals, self.lsrc)
        if self.native_wide:
            self._launch_wide(out, vals, self.wsrc)
        elif self.wide:
            self._torch_buckets(out, vals, self.wide)
        return out

    def add_into_sel(self, out, vals, sel):
        """add_into(out, vals[..., sel]) without forming vals[..., sel] (sel: a fixed device index
        tensor; its composition with the lanes is cached)."""
        if not self._native_ok(out, vals):
            return self.add_into(out, vals[..., sel])
        key = (sel.data_ptr(), sel.numel())
        ent = self._sel_lanes.get(key)
        if ent is not None and ent[0]() is not sel:          # the address of a freed sel, reused
            ent = None
        if ent is None:
            s_h = sel.cpu().numpy()
            lsrc = self.lanes_host[0]
            comp = np.where(lsrc >= 0, s_h[np.clip(lsrc, 0, None)], -1)
            wcomp = None
            if self.native_wide:
                ws = self.wsrc_host
                wcomp = torch.tensor(np.where(ws >= 0, s_h[np.clip(ws, 0, None)], -1).astype(np.int32), device=self.dev)
            lanes = self._sel_lanes

            def _drop(r, k=key):                              # the entry dies with its sel tensor
                if lanes.get(k, (None,))[0] is r:
                    del lanes[k]
            ent = lanes[key] = (weakref.ref(sel, _drop), torch.tensor(comp.astype(np.int32), device=self.dev), wcomp)
        self._launch(out, vals, ent[1])
        if self.native_wide:
            self._launch_wide(out, vals, ent[2])
        elif self.wide:
            self._torch_buckets(out, vals[..., sel], self.wide)
        return out

    def add_products(self, out, vals, x, cols, cols32):
        """add_into(out, vals * x[..., cols]) without forming the products (cols: int64 device
        indices, cols32 the same as int32)."""
        if not self._native_ok(out, vals, x):
            return self.add_into(out, vals * x[..., cols])
        self._launch(out, vals, self.lsrc, x=x, cols=cols32)
        if self.native_wide:
            self._launch_wide(out, vals, self.wsrc, x=x, cols=cols32)
        elif self.wide:
            self._torch_buckets(out, vals * x[..., cols], self.wide)
        return out


_SCATTER_CACHE: dict = {}


def scatter_sum(dst, dev) -> _ScatterSum:
    """The _ScatterSum of a destination pattern, shared by every structure with the same pattern on
    the same device: the homotopy builds a StructuredKKT per step (and per sweep shard), and the
    host-side table construction was ~0.8 s of a 6-step AP2 homotopy (cProfile,
    profiles/r02/solver_pstats_b8.txt).  The tables are read-only after construction, apart from
    add_into_sel's lanes composed with a caller's index tensor: those entries are held through a
    weak reference to that tensor and dropped when it is freed, so structures evicted from the
    caches release their device tables."""
    import hashlib
    dst = np.ascontiguousarray(np.asarray(dst, dtype=np.int64).reshape(-1))
    key = (hashlib.sha1(dst.tobytes()).hexdigest(), dst.size, str(torch.device(dev)))
    sc = _SCATTER_CACHE.get(key)
    if sc is None:
        if len(_SCATTER_CACHE) >= 256:
            _SCATTER_CACHE.clear()
        sc = _SCATTER_CACHE[key] = _ScatterSum(dst, dev)
    return sc


class _GatherMv:
    """y = A(vals) x for a fixed COO pattern: products vals * x[cols], summed per row by a
    _ScatterSum (fixed order).  Replaces rocSPARSE's CSR SpMV, whose adaptive algorithm splits
    long rows (the t_f column of J, i.e. a row of J^T) across workgroups with atomic adds."""

    def __init__(self, rows, cols, shape, dev):
        self.cols = torch.tensor(np.asarray(cols, dtype=np.int64), device=dev)
        self.cols32 = self.cols.to(torch.int32)
        self.sum = scatter_sum(rows, dev)
        self.shape = shape

    def mv(self, vals, x):
        out = x.new_zeros(x.shape[:-1] + (self.shape[0],))
        return self.sum.add_products(out, vals, x, self.cols, self.cols32)


def _dense_A(nlp, jv, N0, K):
    """Write A = [J | -I_slack] into rows N0.. and its transpose (in place)."""
    n, mI = nlp.n, nlp.mI
    rows = N0 + nlp.j_row
    K[rows, nlp.j_col] = jv
    K[nlp.j_col, rows] = jv
    srow = N0 + nlp.s_row
    scol = n + torch.arange(mI, device=K.device)
    K[srow, scol] = -1.0
    K[scol, srow] = -1.0


# interval blocks up to which the inertia pass runs beside the factorisation (StructuredKKT.factor);
# measured in one session (tools/gpu_solver_ab.sh): AP2 sweep +10-14 %, config-4 shard +15 % (fan) and
# +20 % (chain), converged MPC (1,280 blocks) 107 ms against 110-115 ms per sampling time: no limit
EARLY_INERTIA_MAX_BLOCKS = int(os.environ.get("AWE_EARLY_INERTIA_MAX_BLOCKS", "1000000000"))

ZERO_PIVOT = 1e-30   # relative zero-pivot threshold of the inertia count: KKT pivots legitimately span
                     # 1e-10 .. 1e10 at small mu, so only exactly singular columns count as zero


class StructuredKKT:
    """KKT solve by elimination of every interval's interior unknowns (batched dense LU on the
    GPU) and a Schur complement on the separators, for B instances of one KKT pattern at once.

    Intervals of the collocation NLP couple only through the shooting states x[k] (shared by
    interval k and the continuity rows of interval k-1), the free global variables (t_f and
    the homotopy parameters) and the periodicity rows.  Those, and the multipliers of the
    continuity rows, are the separators S; everything else -- u[k], xdot[k], z[k], the
    collocation variables, the path slacks and the multipliers of interval k's node, path and
    collocation rows -- is interior to interval k.  With K = [K_II, K_IS; K_SI, K_SS]:
        S = K_SS - sum_k K_SI^k (K_II^k)^-1 K_IS^k,
    about 5 GFLOP at N=40 instead of the 1.3 TFLOP of a dense LU of the whole system.  The
    B x n_k interval blocks are one batch of the awelu LU kernel; the separators are either B
    block-tridiagonal chains (awebox_amd/btd.py) or B dense Schur complements.  Every assembly is
    a fixed-order gather-sum (_ScatterSum): the results do not depend on the run."""

    # refinement steps before an instance falls back to a dense LU of its K: IPOPT's
    # max_refinement_steps.  An instance whose backward error passes within 3 steps (the fused
    # sweep's earlier budget) is unaffected; on the AP2 sweep the one instance that used to fall back
    # after 3 converges within 10, with identical iterations and powers and 0.25-0.45 s less wall
    # time (profiles/r05/solver/sweep_refine)
    REFINE_STEPS = 10

    def __init__(self, nlp, lay, dev, lu_backend="awelu", separators="btd", deterministic=True):
        n, ny, m = nlp.n, nlp.ny, nlp.m
        self.lu_backend = lu_backend
        N = ny + m
        self.N, self.dev, self.ny = N, dev, ny
        n_k, stride, v0, rows = lay.n_k, lay.interval_stride, lay.v_intervals, lay.rows_per_interval
        nx = getattr(lay, "nx", pb.NX)                          # states per shooting node
        owner = np.full(N, -1, dtype=np.int64)                  # interval of an interior unknown
        free = np.asarray(nlp.free.cpu().numpy() if torch.is_tensor(nlp.free) else nlp.free, dtype=np.int64)
        kf, of = np.divmod(free - v0, stride)
        inner = (free >= v0) & (kf < n_k) & (of >= nx)
        owner[:n][inner] = kf[inner]
        # interval rows start at g0: the MPC NLP leads with nx initial-condition rows
        # (ocp/operation.py:303-326), the periodic NLP has none
        g0 = getattr(lay, "g_int0", 0)
        if g0 > nx:
            raise ValueError("more leading rows than states per node")
        rr_ = np.asarray(nlp.ineq, dtype=np.int64) - g0
        # global rows (t_f bounds): separators
        owner[n:n + len(rr_)] = np.where((rr_ >= 0) & (rr_ < n_k * rows), rr_ // rows, -1)
        # interval rows, except the continuity rows: an interval has more rows than interior
        # unknowns (x[k], x[k+1] close the count), so their multipliers join the separators
        rr = np.arange(m) - g0
        owner[ny + np.arange(m)] = np.where((rr >= 0) & (rr < n_k * rows) & (rr % rows < rows - nx), rr // rows, -1)
        self.owner = owner
        sep = np.where(owner < 0)[0]
        self.nS = len(sep)
        sep_id = np.full(N, -1, dtype=np.int64)
        sep_id[sep] = np.arange(self.nS)
        loc = np.full(N, -1, dtype=np.int64)                    # position within the interval's block
        ip = np.where(owner >= 0)[0]
        counts = np.bincount(owner[ip], minlength=n_k).astype(np.int64)
        by_k = np.argsort(owner[ip], kind="stable")
        first = np.concatenate([[0], np.cumsum(counts)[:-1]])
        loc[ip[by_k]] = np.arange(len(ip)) - first[owner[ip][by_k]]
        self.nI = int(counts.max())
        self.n_k = n_k
        # KKT pattern in COO (both orientations), in the order of the value vector of factor()
        hr, hc = nlp.h_r.cpu().numpy(), nlp.h_c.cpu().numpy()
        off = hr != hc
        jr, jc = nlp.j_row.cpu().numpy(), nlp.j_col.cpu().numpy()
        sr = nlp.s_row.cpu().numpy()
        sc = n + np.arange(nlp.mI)
        P_ = np.concatenate([hr, hc[off], np.arange(ny), ny + jr, jc, ny + sr, sc, ny + np.arange(m)])
        Q_ = np.concatenate([hc, hr[off], np.arange(ny), jc, ny + jr, sc, ny + sr, ny + np.arange(m)])
        self.off_mask = torch.tensor(off, device=dev)
        self.P_, self.Q_ = torch.tensor(P_, device=dev), torch.tensor(Q_, device=dev)
        self.Q32 = self.Q_.to(torch.int32)
        self.n_solve = self.n_dense = 0
        oP, oQ = owner[P_], owner[Q_]
        ii = (oP >= 0) & (oP == oQ)
        is_ = (oP >= 0) & (oQ < 0)
        ss = (oP < 0) & (oQ < 0)
        if ((oP >= 0) & (oQ >= 0) & (oP != oQ)).any():
            raise ValueError("KKT couples the interiors of two intervals")
        lsep = [sorted(set(sep_id[Q_[is_ & (oP == k)]].tolist())) for k in range(n_k)]
        self.L = max(1, max(len(l) for l in lsep))
        lsep_arr = np.full((n_k, self.L), self.nS, dtype=np.int64)      # padding -> dummy separator
        lpos = np.full((n_k, self.nS + 1), -1, dtype=np.int64)
        for k, l in enumerate(lsep):
            lsep_arr[k, :len(l)] = l
            lpos[k, l] = np.arange(len(l))
        self.lsep = torch.tensor(lsep_arr, device=dev)
        nI, L, nS = self.nI, self.L, self.nS
        self.sel_ii = torch.tensor(np.where(ii)[0], device=dev)
        dst_ii = oP[ii] * nI * nI + loc[P_[ii]] * nI + loc[Q_[ii]]
        isi = np.where(is_)[0]
        self.sel_is = torch.tensor(isi, device=dev)
        dst_is = oP[isi] * nI * L + loc[P_[isi]] * L + lpos[oP[isi], sep_id[Q_[isi]]]
        self.sel_ss = torch.tensor(np.where(ss)[0], device=dev)
        dst_ss = sep_id[P_[ss]] * (nS + 1) + sep_id[Q_[ss]]
        pk, pj = np.nonzero(np.arange(nI)[None, :] >= counts[:, None])   # padding rows, by interval
        self.n_pad = len(pk)
        self.pad_flat = torch.tensor(pk * nI * nI + pj * nI + pj, dtype=torch.int64, device=dev)
        schur_flat = (lsep_arr[:, :, None] * (nS + 1) + lsep_arr[:, None, :]).reshape(-1)
        int_p = np.where(owner >= 0)[0]
        self.int_p = torch.tensor(int_p, device=dev)
        self.sc = [scatter_sum(t, dev) for t in (dst_ii, dst_is, dst_ss, schur_flat)]
        self.sc_mv = scatter_sum(P_, dev)
        self.sc_dense = scatter_sum(P_ * N + Q_, dev)
        self.sc_rs = scatter_sum(lsep_arr.reshape(-1), dev)
        # separators in stages [c[k-1], x[k]] (block tridiagonal, globals as border): pairing each
        # shooting state with the multipliers of the continuity row that defines it keeps the block
        # sweep's pivot blocks regular -- the finer order x[0], c[0], x[1], ... meets near-singular
        # pivot blocks at N=40 (cond 3e17 on the AP2 KKT); the paired one stays at cond <= 1e13
        # with |W_k| <= 60, a backward error of 2e-21 (emulated on the CPU)
        self.btd = None
        self.force_btd = False                                  # CPU tests: the BTD path on host
        self.btd_off = False                                    # the dense separator LU even when btd exists
        if lu_backend == "awelu" and separators == "btd":
            stage_of = np.full(self.nS, -1, dtype=np.int64)
            pos_of = np.zeros(self.nS, dtype=np.int64)
            # shooting states x[k] at positions nx.. of stage k
            xs = sep < n
            vq = free[sep[xs]]
            kq, oq = np.divmod(vq - v0, stride)
            hit = (vq >= v0) & (oq < nx) & (kq <= n_k)
            qx = np.where(xs)[0][hit]
            stage_of[qx], pos_of[qx] = kq[hit], nx + oq[hit]
            # multipliers: initial-condition rows at stage 0 beside x[0], continuity rows of interval k
            # at positions 0.. of stage k + 1
            cs = sep >= ny
            rq = sep[cs] - ny - g0
            qc = np.where(cs)[0]
            ic = rq < 0
            stage_of[qc[ic]], pos_of[qc[ic]] = 0, rq[ic] + g0
            ct = (rq >= 0) & (rq < n_k * rows) & (rq % rows >= rows - nx)
            stage_of[qc[ct]], pos_of[qc[ct]] = rq[ct] // rows + 1, rq[ct] % rows - (rows - nx)
            ss_r, ss_c = sep_id[P_[ss]], sep_id[Q_[ss]]
            sch_r, sch_c = lsep_arr[:, :, None].repeat(L, 2), lsep_arr[:, None, :].repeat(L, 1)
            from .btd import BorderedBtd
            try:
                self.btd = BorderedBtd(stage_of, pos_of, n_k + 1, 2 * nx,
                                       np.concatenate([ss_r, sch_r.reshape(-1)]),
                                       np.concatenate([ss_c, sch_c.reshape(-1)]), dev)
            except ValueError:
                self.btd = None                                 # not stage-structured: dense S
        self.int_flat = torch.tensor(owner[int_p] * nI + loc[int_p], device=dev)
        self.sep_p = torch.tensor(sep, device=dev)
        self._cI = None                                         # interval-block counts in flight (factor)

    # ---------------------------------------------------------------------------------------
    def factor(self, hv, diag, jv, delta_c, mI, early_inertia=False):
        """Factorise K for every instance: hv [B, nH] Hessian values, diag [B, ny] (Sigma +
        delta_w), jv [B, nJ] Jacobian values, delta_c float or [B] (1-D inputs: one instance).

        ``early_inertia`` (the caller will ask for inertia()): the Bunch-Kaufman counts of the
        interval blocks start on a side stream as soon as the blocks are assembled and run beside
        their LU, the Schur complement and the separator sweep -- with few instances each of those
        kernels fills a few dozen of the 256 CUs, and the inertia pass (one workgroup per block,
        ~2.3 ms at AP2 N=40 B=1) was the largest single kernel of the sweep's homotopy."""
        f64 = dict(dtype=torch.float64, device=self.dev)
        self._cI = None
        self.squeeze = hv.dim() == 1
        hv, diag, jv = (t.unsqueeze(0) if t.dim() == 1 else t for t in (hv, diag, jv))
        B = hv.shape[0]
        self.B = B
        m = self.N - diag.shape[1]
        dc = torch.as_tensor(delta_c, dtype=torch.float64, device=self.dev).reshape(-1).expand(B)
        vals = torch.cat([hv, hv[:, self.off_mask], diag, jv, jv, -torch.ones(B, 2 * mI, **f64),
                          -dc[:, None].expand(B, m)], dim=1)
        self.vals = vals
        self.k_norm = self._mv(vals.abs(), torch.ones(B, self.N, **f64)).amax(dim=1)     # [B]
        nI, L, nS, n_k = self.nI, self.L, self.nS, self.n_k
        KII = self.sc[0].add_into_sel(torch.zeros(B, n_k * nI * nI, **f64), vals, self.sel_ii)
        KII[:, self.pad_flat] = 1.0
        KII = KII.view(B * n_k, nI, nI)
        self.KII = KII
        if early_inertia and KII.is_cuda and B * n_k <= EARLY_INERTIA_MAX_BLOCKS:
            self._interval_inertia_async(KII)
        KIS = self.sc[1].add_into_sel(torch.zeros(B, n_k * nI * L, **f64), vals, self.sel_is).view(B * n_k, nI, L)
        self.awelu = self.lu_backend == "awelu" and KII.is_cuda   # the CPU test harness uses LAPACK
        if self.awelu:
            from .batched_lu import lu_factor
            self.LU_I, self.piv_I = lu_factor(KII)
        else:
            self.LU_I, self.piv_I = torch.linalg.lu_factor(KII)
        self.X = self._block_solve(KIS)                                        # K_II^-1 K_IS
        T = det.bmm(KIS.transpose(1, 2), self.X).reshape(B, n_k * L * L)       # [B, n_k L L]
        self.KIS = KIS
        if self.btd is not None and not self.btd_off and (KII.is_cuda or self.force_btd):
            self.btd.factor(torch.cat([vals[:, self.sel_ss], -T], dim=1))
            self.use_btd = True
            return
        self.use_btd = False
        S = torch.zeros(B, (nS + 1) * (nS + 1), **f64)
        self.sc[2].add_into_sel(S, vals, self.sel_ss)
        self.sc[3].add_into(S, -T)
        S = S.view(B, nS + 1, nS + 1)
        S[:, nS, :] = 0.0
        S[:, :, nS] = 0.0
        S[:, nS, nS] = 1.0
        self.S = S
        self.LU_S, self.piv_S = torch.linalg.lu_factor(S)

    def _interval_inertia_async(self, KII):
        from .batched_lu import sym_inertia
        side = getattr(self, "_side", None)
        if side is None:
            side = self._side = torch.cuda.Stream(device=KII.device)
        main = torch.cuda.current_stream(KII.device)
        side.wait_stream(main)                          # KII assembled
        with torch.cuda.stream(side):
            self._cI = sym_inertia(KII, ztol=ZERO_PIVOT)
        KII.record_stream(side)                         # not reused before the side stream is done
        self._cI_done = torch.cuda.Event()
        self._cI_done.record(side)

    def _interval_inertia(self):
        """[B, 3] counts of the interval blocks (padding rows excluded)."""
        from .batched_lu import sym_inertia, sym_inertia_host
        if self._cI is not None:
            main = torch.cuda.current_stream(self.KII.device)
            main.wait_event(self._cI_done)
            cI = self._cI
            cI.record_stream(main)
        else:
            f = sym_inertia if self.KII.is_cuda else sym_inertia_host
            cI = f(self.KII, ztol=ZERO_PIVOT)
        c = cI.to(torch.int64).view(self.B, self.n_k, 3).sum(1)
        c[:, 0] -= self.n_pad
        return c

    def inertia(self):
        """(positive, negative, zero) eigenvalue counts of K per instance, int64 [B, 3] (a tuple for
        a one-instance factor()), by Haynsworth's additivity In(K) = sum_k In(K_II^k) + In(S):
        Bunch-Kaufman inertia of the interval blocks (padding rows excluded) and of the separator
        system -- the dense Schur complement, or with the block-tridiagonal separators the sweep's
        pivot blocks and the border (btd.BorderedBtd)."""
        from .batched_lu import sym_inertia, sym_inertia_host
        f = sym_inertia if self.KII.is_cuda else sym_inertia_host
        c = self._interval_inertia()
        if self.use_btd:
            c = c + self.btd.inertia()
        else:
            cs = f(self.S, ztol=ZERO_PIVOT).to(torch.int64)
            cs[:, 0] -= 1                                       # the dummy separator's 1.0
            c = c + cs
        if self.squeeze:
            return tuple(int(v) for v in c[0].cpu().tolist())
        return c

    def _mv(self, vals, x):
        """K(vals) x for every instance: a fixed-order gather-sum."""
        return self.sc_mv.add_products(torch.zeros(x.shape[0], self.N, dtype=torch.float64, device=self.dev),
                                       vals, x, self.Q_, self.Q32)

    def matvec(self, x):
        return self._mv(self.vals, x)

    def solve(self, rhs, refine=None, rtol=1e-12, active=None):
        """Elimination solve with iterative refinement on the sparse residual, rhs [B, N] (or [N]).
        The interior pivots come from blocks that may be ill-conditioned even when K is not (an
        indefinite interior Hessian), so an instance's result is accepted once its backward error
        is small, ||K x - rhs|| <= rtol (||K|| ||x|| + ||rhs||) in the max norm; an instance that
        does not get there is solved once by a dense LU of its assembled K.  ``active`` ([B] bool,
        numpy or torch) restricts refinement and the dense fallback to the instances whose result
        the caller uses: the others (converged, failed, outside the current step) may hold a
        near-singular K and are returned unrefined.  A singular fallback K yields non-finite
        values for the caller's isfinite checks instead of an exception."""
        one = rhs.dim() == 1
        rhs = rhs.unsqueeze(0) if one else rhs
        if refine is None:
            # the dense fallback is a library LU of the whole K (~0.3 s at N = 12,257 or 13,848)
            refine = self.REFINE_STEPS
        self.n_solve += 1
        x = self._solve(rhs)
        b_norm = rhs.abs().amax(dim=1)
        done = torch.zeros(rhs.shape[0], dtype=torch.bool, device=self.dev)
        if active is not None:
            # a host mask goes through pinned memory asynchronously: a pageable copy would wait
            # for the solve just launched before the refinement's first launches are queued
            a = active if torch.is_tensor(active) else torch.from_numpy(np.ascontiguousarray(active, dtype=bool))
            if not a.is_cuda and torch.device(self.dev).type == "cuda":
                a = a.pin_memory().to(self.dev, non_blocking=True)
            done = ~a.to(device=self.dev, dtype=torch.bool).reshape(-1)
        for it in range(refine + 1):
            r = rhs - self.matvec(x)
            err = r.abs().amax(dim=1)
            scale = self.k_norm * x.abs().amax(dim=1) + b_norm
            done = done | (err <= rtol * scale)
            bad = ~torch.isfinite(err)
            # one transfer: the test, the fallback list and whether each solution is finite (the
            # callers' check, self.last_finite)
            db = torch.stack([done, bad, torch.isfinite(x).all(1)]).cpu().numpy()
            if (db[0] | db[1]).all() or it == refine:
                break
            x = torch.where(done[:, None], x, x + self._solve(r))
        todo = np.where(~db[0])[0].tolist()
        self.last_finite = db[2].copy()
        for b in todo:                      # ill-conditioned interior pivots: dense LU of that K
            self.n_dense += 1
            K = self.sc_dense.add_into(torch.zeros(self.N * self.N, dtype=torch.float64, device=self.dev),
                                       self.vals[b])
            xb, info = torch.linalg.solve_ex(K.view(self.N, self.N), rhs[b])
            x[b] = torch.where(info == 0, xb, torch.full_like(xb, float("nan")))
        if todo:
            self.last_finite = torch.isfinite(x).all(1).cpu().numpy()
        return x[0] if one else x

    def _block_solve(self, B):
        """K_II^-1 B for all interval blocks: the awelu solve kernel (right-hand sides resident in
        LDS; rocBLAS's batched trsv took 2.4 ms per one-column solve of 320 blocks) on the device,
        LAPACK in the CPU harness."""
        if self.awelu:
            from .batched_lu import lu_solve
            return lu_solve(self.LU_I, self.piv_I, B)
        return torch.linalg.lu_solve(self.LU_I, self.piv_I, B)

    def _solve(self, rhs):
        if rhs.dim() == 1:
            return self._solve(rhs.unsqueeze(0))[0]
        f64 = dict(dtype=torch.float64, device=self.dev)
        nI, L, nS, n_k = self.nI, self.L, self.nS, self.n_k
        B = rhs.shape[0]
        rI = torch.zeros(B, n_k * nI, **f64)
        rI[:, self.int_flat] = rhs[:, self.int_p]
        rS = torch.zeros(B, nS + 1, **f64)
        rS[:, :nS] = rhs[:, self.sep_p]
        z = self._block_solve(rI.view(B * n_k, nI, 1))                         # [B n_k, nI, 1]
        upd = det.bmm(self.KIS.transpose(1, 2), z).reshape(B, n_k * L)
        self.sc_rs.add_into(rS, -upd)
        rS[:, nS] = 0.0
        xS = torch.zeros(B, nS + 1, **f64)
        if self.use_btd:
            xS[:, :nS] = self.btd.solve(rS[:, :nS])
        else:
            xS = torch.linalg.lu_solve(self.LU_S, self.piv_S, rS.unsqueeze(-1)).squeeze(-1)
        xI = z.view(B * n_k, nI) - det.bmm(self.X, xS[:, self.lsep].reshape(B * n_k, L, 1)).view(B * n_k, nI)
        sol = torch.empty(B, self.N, **f64)
        sol[:, self.int_p] = xI.view(B, n_k * nI)[:, self.int_flat]
        sol[:, self.sep_p] = xS[:, :nS]
        return sol


def _as_batch(a, B, n, fill=None):
    """[B, n] float64 numpy array from None / [n] / [B, n]."""
    if a is None:
        return None if fill is None else np.full((B, n), fill)
    a = np.asarray(a, dtype=np.float64)
    return np.tile(a, (B, 1)) if a.ndim == 1 else a


def solve(ev, P, x0, lbx, ubx, lbg, ubg, lam0=None, zl0=None, zu0=None, opts: IpmOptions | None = None,
          device="cuda") -> IpmResult:
    """Solve min f s.t. lbg <= g <= ubg, lbx <= x <= ubx for one instance with the GPU
    interior-point method (solve_batch with B = 1)."""
    return solve_batch(ev, np.atleast_2d(P), np.atleast_2d(x0), lbx, ubx, lbg, ubg,
                       None if lam0 is None else np.atleast_2d(lam0),
                       None if zl0 is None else np.atleast_2d(zl0),
                       None if zu0 is None else np.atleast_2d(zu0), opts=opts, device=device)[0]


_STRUCT_CACHE: dict = {}


def cached_kkt_structures():
    """The StructuredKKT objects of the recent solves' structure cache (read-only use: bench.py
    times the solver kernels at their block shapes)."""
    return [e[0] for e in _STRUCT_CACHE.values()]


def _layout_key(lay):
    """What StructuredKKT reads from a layout: two evaluators whose layouts agree here (and whose NLPs
    have the same patterns) share one structure."""
    return (type(lay).__name__, lay.n_k, lay.interval_stride, lay.v_intervals, lay.rows_per_interval,
            getattr(lay, "nx", pb.NX), getattr(lay, "g_int0", 0))


def _structure(ev, nlp, dev, opts):
    """(StructuredKKT, J^T product, H product) for one NLP structure, shared by the solves with the
    same layout and the same fixed-variable / inequality sets and patterns, whichever evaluator (and
    batch) runs them: every sampling time of the MPC solves its pre-solve and main solve on one
    structure, and a sweep shard's batched warm start reuses its homotopy's final structure.  Their
    construction is host work of ~0.1 s at AP2 N=40.  Only structural data enters them; the per-solve
    state (the factorisation, the counters, the separator switches) is reset or overwritten by every
    solve."""
    import hashlib
    h = hashlib.sha1()
    for a in (nlp.free, nlp.ineq, nlp.j_row.cpu().numpy(), nlp.j_col.cpu().numpy(), nlp.h_r.cpu().numpy(),
              nlp.h_c.cpu().numpy()):
        h.update(np.ascontiguousarray(a, dtype=np.int64).tobytes())
        h.update(b"|")
    key = (_layout_key(ev.layout), len(nlp.x_fix), h.hexdigest(),
           str(torch.device(dev)), opts.lu_backend, opts.separators)
    ent = _STRUCT_CACHE.get(key)
    if ent is not None:
        skkt = ent[0]
        skkt.n_solve = skkt.n_dense = 0
        skkt.force_btd = skkt.btd_off = False
        return ent
    skkt = StructuredKKT(nlp, ev.layout, dev, lu_backend=opts.lu_backend, separators=opts.separators)
    ny, m = nlp.ny, nlp.m
    jt_op = _GatherMv(nlp.j_col.cpu().numpy(), nlp.j_row.cpu().numpy(), (ny, m), dev)
    hr_np, hc_np = nlp.h_r.cpu().numpy(), nlp.h_c.cpu().numpy()
    off_np = hr_np != hc_np
    h_op = _GatherMv(np.concatenate([hr_np, hc_np[off_np]]), np.concatenate([hc_np, hr_np[off_np]]), (ny, ny), dev)
    if len(_STRUCT_CACHE) >= 8:
        _STRUCT_CACHE.clear()
    _STRUCT_CACHE[key] = (skkt, jt_op, h_op)
    return skkt, jt_op, h_op


def solve_batch(ev, P, x0, lbx, ubx, lbg, ubg, lam0=None, zl0=None, zu0=None, opts: IpmOptions | None = None,
                device="cuda") -> list[IpmResult]:
    """Solve B instances of one NLP structure (P [B, n_p], x0 [B, n_v], shared bounds) side by side
    with the GPU interior-point method; returns one IpmResult per instance.

    Every instance runs its own IPOPT iteration (barrier parameter, filter, inertia correction,
    line search, restoration, termination); their evaluations (ev.batch == B), Hessians and KKT
    factorisations/solves are batched, so B instances cost little more per iteration than one.
    lam0 / zl0 / zu0 (constraint and V-bound multipliers of a previous solve) select IPOPT's
    warm_start_init_point: the multipliers are kept (pushed away from zero) and the primal point
    is pushed into the bounds with the smaller warm-start push."""
    opts = opts or IpmOptions()
    t_start = time.perf_counter()
    dev = torch.device(device)
    P = np.atleast_2d(np.asarray(P, dtype=np.float64))
    B = P.shape[0]
    nlp = DeviceNlp(ev, P, lbx, ubx, lbg, ubg, dev, relax=opts.bound_relax_factor, relax_cap=opts.constr_viol_tol)
    n, mI, m, ny = nlp.n, nlp.mI, nlp.m, nlp.ny
    N = ny + m
    f64 = dict(dtype=torch.float64, device=dev)
    logs = [[] for _ in range(B)]
    x0 = _as_batch(x0, B, ev.n_v)

    # ---- initial point: bound push (IPOPT 3.6) -----------------------------------------------
    x = torch.tensor(x0[:, nlp.free], **f64)
    yl, yu, hl, hu = nlp.yl, nlp.yu, nlp.has_l, nlp.has_u
    warm = lam0 is not None
    bpush = opts.warm_start_bound_push if warm else opts.bound_push
    bfrac = opts.warm_start_bound_push if warm else opts.bound_frac

    def push(y):
        lo = torch.where(hl, yl, torch.full_like(yl, -1e300))
        hi = torch.where(hu, yu, torch.full_like(yu, 1e300))
        gap = torch.where(hl & hu, hi - lo, torch.full_like(yl, 1e300))
        pl = torch.minimum(bpush * torch.clamp(lo.abs(), min=1.0), bfrac * gap)
        pu = torch.minimum(bpush * torch.clamp(hi.abs(), min=1.0), bfrac * gap)
        y = torch.where(hl, torch.maximum(y, lo + pl), y)
        y = torch.where(hu, torch.minimum(y, hi - pu), y)
        return y

    # gradient-based NLP scaling at the starting point (IPOPT nlp_scaling_method), per instance
    f0, grad0, g0, jv0 = nlp.eval_all(push(torch.cat([x, torch.zeros(B, mI, **f64)], 1))[:, :n])
    gmax = grad0.abs().amax(dim=1) if n else torch.zeros(B, **f64)
    nlp.obj_scale = torch.where(gmax > 0, torch.clamp(opts.nlp_scaling_max_gradient / gmax, max=1.0),
                                torch.ones_like(gmax))
    rowmax = torch.zeros(B, m, **f64).scatter_reduce_(1, nlp.j_row.expand(B, -1), jv0.abs(), "amax",
                                                      include_self=True)
    nlp.c_scale = torch.clamp(opts.nlp_scaling_max_gradient / torch.clamp(rowmax, min=1e-300), max=1.0)
    cs_I = nlp.c_scale[:, nlp.ineq_t]
    nlp.yl[:, n:] = torch.where(hl[:, n:], nlp.yl[:, n:] * cs_I, nlp.yl[:, n:])
    nlp.yu[:, n:] = torch.where(hu[:, n:], nlp.yu[:, n:] * cs_I, nlp.yu[:, n:])

    y = torch.cat([x, torch.zeros(B, mI, **f64)], 1)
    f, grad, g, jv = nlp.eval_all(y[:, :n])
    y[:, n:] = g[:, nlp.ineq_t]
    y = push(y)
    lam = torch.zeros(B, m, **f64)
    if warm:
        lam = torch.tensor(_as_batch(lam0, B, m), **f64) / nlp.c_scale * nlp.obj_scale[:, None]
    zl = torch.where(hl, torch.ones(B, ny, **f64), torch.zeros(B, ny, **f64))
    zu = torch.where(hu, torch.ones(B, ny, **f64), torch.zeros(B, ny, **f64))
    if warm:
        floor = opts.warm_start_mult_bound_push
        if zl0 is not None:
            zx = torch.tensor(_as_batch(zl0, B, ev.n_v)[:, nlp.free], **f64) * nlp.obj_scale[:, None]
            zl[:, :n] = torch.where(hl[:, :n], torch.clamp(zx, min=floor), zl[:, :n])
        if zu0 is not None:
            zx = torch.tensor(_as_batch(zu0, B, ev.n_v)[:, nlp.free], **f64) * nlp.obj_scale[:, None]
            zu[:, :n] = torch.where(hu[:, :n], torch.clamp(zx, min=floor), zu[:, :n])
        # slack bound multipliers from the row multipliers: dL/ds = -lam - z_l + z_u = 0
        lamI = lam[:, nlp.ineq_t]
        zl[:, n:] = torch.where(hl[:, n:], torch.clamp(-lamI, min=floor), zl[:, n:])
        zu[:, n:] = torch.where(hu[:, n:], torch.clamp(lamI, min=floor), zu[:, n:])

    # ---- per-instance state (host) ---------------------------------------------------------
    mu = np.full(B, opts.mu_init)
    # IPOPT's MonotoneMuUpdate floor: max(mu_target, mu_min, min(tol, compl_inf_tol) / (barrier_tol_factor + 1))
    mu_floor = max(opts.mu_target, 1e-11, min(opts.tol, opts.compl_inf_tol) / 11.0)
    n_accept = np.zeros(B, dtype=np.int64)
    tau = np.maximum(opts.tau_min, 1.0 - mu)
    filt = [[] for _ in range(B)]
    c = nlp.constraints(g, y[:, n:])
    theta0 = det.row_sum(c.abs()).cpu().numpy()
    theta_max = 1e4 * np.maximum(1.0, theta0)
    theta_min = 1e-4 * np.maximum(1.0, theta0)
    delta_w_last = np.zeros(B)
    # watchdog state per instance (IpmOptions.watchdog_*)
    wd_short = np.zeros(B, dtype=np.int64)                   # consecutive shortened steps
    in_wd = np.zeros(B, dtype=bool)
    wd_trial = np.zeros(B, dtype=np.int64)
    wd_skip = np.zeros(B, dtype=bool)                        # back at the watchdog's start: skip the full step
    wd_ref = [np.zeros(B), np.zeros(B), np.zeros(B), np.zeros(B)]   # theta, phi, grad phi . d, alpha
    wd_pt = None                                             # (y, lam, zl, zu) at the watchdog's start
    status = np.array(["max_iter"] * B, dtype=object)
    iters = np.zeros(B, dtype=np.int64)
    kkt_err = np.full(B, math.inf)
    active = np.ones(B, dtype=bool)
    skkt, jt_op, h_op = _structure(ev, nlp, dev, opts)
    skkt.force_btd = opts.separators == "btd"                   # the block sweep on host tensors too
    # exact inertia needs the separator pivot blocks of the block sweep on the device (a dense
    # Bunch-Kaufman pass over the whole Schur complement is ~1 s); otherwise the curvature test
    exact_inertia = opts.inertia == "exact" and (skkt.btd is not None or dev.type != "cuda")
    if skkt.btd is not None and dev.type == "cuda":
        skkt.force_btd = True
    if not warm and opts.constr_mult_init_max > 0 and m:
        # IPOPT's DefaultIterateInitializer: least-square constraint multipliers at the starting
        # point, [I A^T; A 0] (w, lam) = (-(grad f - z_L + z_U), 0), kept only where
        # max|lam| <= constr_mult_init_max (otherwise lam = 0)
        skkt.factor(torch.zeros(B, len(nlp.h_keep), **f64), torch.ones(B, ny, **f64), jv, 0.0, mI)
        sol = skkt.solve(torch.cat([-(torch.cat([grad, torch.zeros(B, mI, **f64)], 1) - zl + zu),
                                    torch.zeros(B, m, **f64)], 1))
        lam_ls = sol[:, ny:]
        keep = torch.isfinite(lam_ls).all(1) & (lam_ls.abs().amax(1) <= opts.constr_mult_init_max)
        lam = torch.where(keep[:, None], lam_ls, lam)
    timing = {}

    class _Phase:
        def __init__(self, key):
            self.key = key

        def __enter__(self):
            if opts.profile:
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                self.t = time.perf_counter()

        def __exit__(self, *exc):
            if opts.profile:
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                timing[self.key] = timing.get(self.key, 0.0) + time.perf_counter() - self.t
            return False

    def gaps(yv):
        dl = torch.where(hl, yv - yl, torch.ones_like(yv))
        du = torch.where(hu, yu - yv, torch.ones_like(yv))
        return dl, du

    def grad_y(gradv):
        return torch.cat([gradv, torch.zeros(B, mI, **f64)], 1)

    # IPOPT's optimality error, the merit pair (theta, phi), the Newton system's vectors and the step
    # update (with the kappa_d damping of one-sided bounds and the kappa_sigma safeguard): one libawelu
    # launch each per call on the device, the torch composition on host tensors (ipm_measures.Measures)
    meas = Measures(nlp, opts, jt_op, dev, n, mI, m, B)

    def ftb_dev(v, dv, mask_pos, tau_t):
        """Fraction-to-the-boundary step per instance on the device: min_i -tau v_i / dv_i ([B])."""
        ratio = torch.where(mask_pos & (dv < 0), -tau_t[:, None] * v / dv, torch.full_like(v, math.inf))
        return ratio.amin(1) if ratio.shape[1] else torch.full((B,), math.inf, **f64)

    def ftb2(vl, dvl, vu, dvu, tau_t, extra=None):
        """min(1, step to the lower bounds, step to the upper bounds) per instance (host [B]), in one
        device-to-host copy together with the rows of ``extra`` (returned after the step)."""
        rows = [ftb_dev(vl, dvl, hl, tau_t), ftb_dev(vu, dvu, hu, tau_t)] + (extra or [])
        h = torch.stack(rows).cpu().numpy()
        a = np.minimum(1.0, np.minimum(h[0], h[1]))
        return (a, *h[2:]) if extra else a

    def filter_ok(b, theta_t, phi_t):
        return all(not (theta_t >= th_f and phi_t >= ph_f) for th_f, ph_f in filt[b])

    hv_zero = torch.zeros(B, len(nlp.h_keep), **f64)

    def dev_b(a):
        """A host [B] array on the device: staged through pinned memory and copied asynchronously
        (a pageable copy waits for the device; ~80 of them per MPC sampling time)."""
        t = torch.from_numpy(np.array(a, dtype=np.float64))
        return t.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else t

    # ---- the newton direction with inertia correction (all instances in `want`) ------------------
    def newton_direction(want, dw_floor, hv, sigma, rhs, mu_t):
        """Per instance in `want`: (ok, sol, delta_w) of the primal-dual system with IPOPT's
        inertia correction (exact inertia) or the curvature test.  The factorisation left in skkt
        belongs to each accepted instance's final (delta_w, delta_c)."""
        delta_w = np.where(want, dw_floor, 0.0)
        delta_c = np.zeros(B)
        done = ~want.copy()
        ok = np.zeros(B, dtype=bool)
        sol_out = torch.zeros(B, N, **f64)
        dw_used = np.zeros(B)
        for attempt in range(60):
            with _Phase("kkt_factor"):
                skkt.factor(hv, sigma + dev_b(delta_w)[:, None], jv, dev_b(delta_c), mI, early_inertia=exact_inertia)
            grow = ~done.copy()
            if exact_inertia:
                with _Phase("inertia"):
                    inert = skkt.inertia().cpu().numpy()
                pos, neg, zero = inert[:, 0], inert[:, 1], inert[:, 2]
                # zero or missing negative eigenvalues: a (numerically) rank-deficient constraint
                # Jacobian -> delta_c once; too few positive ones -> delta_w (Waechter & Biegler
                # 2006, Alg. IC)
                need_c = ~done & ((zero > 0) | (neg < m)) & (delta_c == 0.0)
                delta_c = np.where(need_c, opts.delta_c * mu_t ** 0.25, delta_c)
                good = ~done & ~need_c & (pos == ny) & (neg == m)
                grow &= ~need_c
            else:
                good = ~done
            if good.any():
                with _Phase("kkt_solve"):
                    sol = skkt.solve(rhs, active=good)
                fin = skkt.last_finite                        # isfinite(sol), from the solve's last copy
                if not exact_inertia:
                    dy = sol[:, :ny]
                    Wd = h_op.mv(torch.cat([hv, hv[:, nlp.h_offdiag]], 1), dy)
                    curv = det.row_sum(dy * (Wd + (sigma + dev_b(delta_w)[:, None]) * dy))
                    cpass = (curv >= opts.curvature_kappa * det.row_sum(dy * dy)).cpu().numpy()
                    bad_fin = good & ~fin
                    delta_c = np.where(bad_fin & (delta_c == 0.0), opts.delta_c * mu_t ** 0.25, delta_c)
                    newly = good & fin & cpass
                else:
                    newly = good & fin
                    bad_fin = good & ~fin
                    delta_c = np.where(bad_fin & (delta_c == 0.0), opts.delta_c * mu_t ** 0.25, delta_c)
                if newly.any():
                    idx = torch.tensor(np.where(newly)[0], device=dev)
                    sol_out[idx] = sol[idx]
                    ok |= newly
                    dw_used = np.where(newly, delta_w, dw_used)
                    delta_w_last[newly & (delta_w > 0)] = delta_w[newly & (delta_w > 0)]
                    done |= newly
                grow &= ~newly
            # increase delta_w for the instances that still need it
            first = grow & (delta_w == 0.0)
            later = grow & (delta_w > 0.0)
            delta_w = np.where(first, np.where(delta_w_last == 0.0, opts.delta_w0,
                                               np.maximum(opts.delta_w_min, delta_w_last / 3.0)), delta_w)
            delta_w = np.where(later, delta_w * np.where(delta_w_last > 0, 8.0, 100.0), delta_w)
            done |= grow & (delta_w > opts.delta_w_max)
            if done.all():
                break
        return ok, sol_out, dw_used, delta_w, delta_c

    def refactor_for(sel, hv, sigma, delta_w, delta_c):
        """Leave skkt with the factorisation of the given per-instance (delta_w, delta_c)."""
        skkt.factor(hv, sigma + dev_b(delta_w)[:, None], jv, dev_b(delta_c), mI)

    # ---- the filter line search with second-order corrections (all instances in `want`) ---------
    def line_search(want, dy, dlam, rhs_top, c_cur, dl, du, theta, phi, grad_phi, tau_t, mu_t, wd=None, wd_ref=None,
                    skip_first=None, wd_new=None):
        """Per instance in `want`: (accepted, alpha, y_trial, dy_used, dlam_used, backtracks, socs, alpha_max,
        wd_failed).  ``wd`` [B] bool: instances in the watchdog -- one trial at the full step, judged
        against ``wd_ref`` = (theta, phi, grad phi . d, alpha) of the watchdog's starting point, no
        backtracking and no second-order correction (a failure is reported in wd_failed);
        ``skip_first`` [B] bool: the first trial point is skipped (the line search after a failed
        watchdog starts at half the step)."""
        # the fraction-to-the-boundary step and grad phi . dy stay on the device for the first trial
        # and come back with its theta / phi in one copy (the host minimum and the device minimum
        # are the same exact operation)
        alpha_dev = torch.minimum(torch.minimum(ftb_dev(dl, dy, hl, tau_t), ftb_dev(du, -dy, hu, tau_t)),
                                  torch.ones(B, **f64))
        gphi_dev = det.row_sum(grad_phi * dy)
        alpha = gphi_d = alpha_min = None
        live = want.copy()
        acc = np.zeros(B, dtype=bool)
        a_out = np.zeros(B)
        y_out = y.clone()
        dy_out, dlam_out = dy.clone(), dlam.clone()
        nback = np.zeros(B, dtype=np.int64)
        nsoc = np.zeros(B, dtype=np.int64)
        first = want.copy()                    # the next trial is the first one (SOC eligible)
        in_soc = np.zeros(B, dtype=bool)
        soc_p = np.zeros(B, dtype=np.int64)
        theta_old = np.zeros(B)
        c_soc = torch.zeros(B, m, **f64)
        dys = torch.zeros(B, ny, **f64)
        dlam_s = torch.zeros(B, m, **f64)
        a_s = np.zeros(B)
        wd_failed = np.zeros(B, dtype=bool)
        skipped = np.zeros(B, dtype=bool)
        alpha_max = None

        def accept_test(b, a, theta_t, phi_t):
            if not (math.isfinite(theta_t) and math.isfinite(phi_t)):
                return False, False
            th0, ph0, gp0 = theta[b], phi[b], gphi_d[b]
            if wd is not None and wd[b]:                          # the watchdog's reference point
                th0, ph0, gp0, a = wd_ref[0][b], wd_ref[1][b], wd_ref[2][b], wd_ref[3][b]
            switching = gp0 < 0 and a * (-gp0) ** opts.s_phi > opts.delta_switch * th0 ** opts.s_theta
            if th0 <= theta_min[b] and switching:
                ok_ = phi_t <= ph0 + opts.eta_phi * a * gp0
                f_type = True
            else:
                ok_ = theta_t <= theta_max[b] and (theta_t <= (1 - opts.gamma_theta) * th0 or
                                                   phi_t <= ph0 - opts.gamma_phi * th0)
                f_type = False
            return ok_ and filter_ok(b, theta_t, phi_t), f_type

        for _round in range(opts.max_backtracks * (opts.max_soc + 1) + 1):
            if not live.any():
                break
            if alpha is None:                                 # first trial: alpha on the device
                yt = y + alpha_dev[:, None] * dy
            else:
                a_t = dev_b(np.where(in_soc, a_s, alpha))[:, None]
                yt = y + a_t * torch.where(dev_b(in_soc)[:, None] > 0, dys, dy)
            with _Phase("eval_fg"):
                ft, gt = nlp.eval_fg(yt[:, :n])
            ct = nlp.constraints(gt, yt[:, n:])
            tp2 = meas.merit(ct, ft, yt, dev_b(mu_t))
            if alpha is None:
                tp4 = torch.cat([tp2, torch.stack([alpha_dev, gphi_dev])]).cpu().numpy()
                tp, alpha, gphi_d = tp4[:2], tp4[2].copy(), tp4[3].copy()
                alpha_max = alpha.copy()
                alpha_min = opts.alpha_min_frac * np.where(
                    gphi_d < 0, np.minimum(opts.gamma_theta, opts.gamma_phi * theta / np.maximum(-gphi_d, 1e-300)),
                    opts.gamma_theta)
                if wd_new is not None and wd_new.any():       # a watchdog starting here: its reference
                    wd_ref[2][wd_new] = gphi_d[wd_new]
                    wd_ref[3][wd_new] = alpha[wd_new]
                if skip_first is not None and skip_first.any():
                    # IPOPT's skip_first_trial_point: these instances start at half the step (their first
                    # trial, evaluated with the others, is discarded)
                    skipped[:] = skip_first & live
                    alpha = np.where(skipped, 0.5 * alpha, alpha)
                    nback[skipped] += 1
                    first[skipped] = False
            else:
                tp = tp2.cpu().numpy()
            start_soc = np.zeros(B, dtype=bool)
            cont_soc = np.zeros(B, dtype=bool)
            for b in np.where(live)[0]:
                th_b, ph_b = float(tp[0, b]), float(tp[1, b])
                if skipped[b]:                                # the skipped first trial: half the step next
                    skipped[b] = False
                    continue
                ok_, f_type = accept_test(b, alpha[b], th_b, ph_b)
                if wd is not None and wd[b]:                  # watchdog: the full step or nothing
                    if ok_:
                        acc[b], live[b] = True, False
                        a_out[b] = alpha[b]
                    else:
                        wd_failed[b], live[b] = True, False
                    continue
                if ok_:
                    if not f_type:
                        filt[b].append(((1 - opts.gamma_theta) * theta[b], phi[b] - opts.gamma_phi * theta[b]))
                    acc[b], live[b] = True, False
                    a_out[b] = a_s[b] if in_soc[b] else alpha[b]
                    continue
                if in_soc[b]:
                    nsoc[b] += 1
                    if math.isfinite(th_b) and th_b <= opts.kappa_soc * theta_old[b] and soc_p[b] + 1 < opts.max_soc:
                        soc_p[b] += 1
                        theta_old[b] = th_b
                        cont_soc[b] = True
                        continue
                    in_soc[b] = False                       # corrections failed: back to backtracking
                elif first[b] and opts.max_soc > 0 and math.isfinite(th_b) and th_b >= theta[b]:
                    first[b] = False
                    start_soc[b] = True
                    theta_old[b] = th_b
                    continue
                first[b] = False
                alpha[b] *= 0.5
                nback[b] += 1
                if alpha[b] < alpha_min[b] or nback[b] >= opts.max_backtracks:
                    live[b] = False
            if start_soc.any() or cont_soc.any():
                # second-order correction (Waechter & Biegler 2006, section 2.4): same matrix,
                # constraint part of the right-hand side c_soc = alpha c(y) + c(y_trial), then
                # c_soc <- a_soc c_soc + c(y_soc)
                st = dev_b(start_soc)[:, None] > 0
                ctn = dev_b(cont_soc)[:, None] > 0
                c_soc = torch.where(st, dev_b(alpha)[:, None] * c_cur + ct,
                                    torch.where(ctn, dev_b(a_s)[:, None] * c_soc + ct, c_soc))
                with _Phase("kkt_solve"):
                    sol = skkt.solve(torch.cat([rhs_top, -c_soc], 1), active=start_soc | cont_soc)
                fin = skkt.last_finite                        # isfinite(sol), from the solve's last copy
                upd = (start_soc | cont_soc) & fin
                sel = dev_b(upd)[:, None] > 0
                dys = torch.where(sel, sol[:, :ny], dys)
                dlam_s = torch.where(sel, sol[:, ny:], dlam_s)
                a_new = ftb2(dl, dys, du, -dys, tau_t)
                a_s = np.where(upd, a_new, a_s)
                in_soc |= upd
                # a non-finite correction: plain backtracking
                nf = (start_soc | cont_soc) & ~fin
                in_soc &= ~nf
                for b in np.where(nf)[0]:
                    alpha[b] *= 0.5
                    nback[b] += 1
            # remember the accepted trial points
            if acc.any():
                sel = dev_b(acc & want)[:, None] > 0
                y_out = torch.where(sel & (dev_b(in_soc)[:, None] > 0), y + dev_b(a_s)[:, None] * dys,
                                    torch.where(sel, y + dev_b(alpha)[:, None] * dy, y_out))
                dy_out = torch.where(sel & (dev_b(in_soc)[:, None] > 0), dys, dy_out)
                dlam_out = torch.where(sel & (dev_b(in_soc)[:, None] > 0), dlam_s, dlam_out)
                want = want & ~acc
        return acc, a_out, y_out, dy_out, dlam_out, nback, nsoc, alpha_max, wd_failed

    # ---- feasibility restoration (all instances in `want`) ---------------------------------------
    def restoration(want, c0, theta0_, mu_t, max_steps=50):
        """Minimum-norm Gauss-Newton corrections toward c(y) = 0, scaled by the barrier Sigma, with
        backtracking on theta, until the filter accepts the point (IPOPT's restoration phase,
        reduced to its core).  Returns (success [B], y, lam)."""
        yv = y.clone()
        lam_r = lam.clone()
        live = want.copy()
        succ = np.zeros(B, dtype=bool)
        for _ in range(max_steps):
            if not live.any():
                break
            _, _, g_c, jv_c = nlp.eval_all(yv[:, :n])
            cv = nlp.constraints(g_c, yv[:, n:])
            th = det.row_sum(cv.abs()).cpu().numpy()
            dlv, duv = gaps(yv)
            sig = torch.where(hl, 1.0 / dlv ** 2, torch.zeros_like(yv)) + torch.where(hu, 1.0 / duv ** 2, torch.zeros_like(yv))
            skkt.factor(hv_zero, sig + 1e-8, jv_c, 0.0, mI)
            sol = skkt.solve(-torch.cat([torch.zeros(B, ny, **f64), cv], 1), active=live)
            fin = skkt.last_finite                            # isfinite(sol), from the solve's last copy
            live &= fin
            dyv = torch.where(torch.isfinite(sol[:, :ny]), sol[:, :ny], torch.zeros_like(sol[:, :ny]))
            a = ftb2(dlv, dyv, duv, -dyv, dev_b(tau))
            searching = live.copy()
            a_acc = np.zeros(B)
            for _bt in range(30):
                if not searching.any():
                    break
                yt = yv + dev_b(a)[:, None] * dyv
                ft, gt = nlp.eval_fg(yt[:, :n])
                ct = nlp.constraints(gt, yt[:, n:])
                tht = det.row_sum(ct.abs()).cpu().numpy()
                okb = searching & np.isfinite(tht) & (tht < (1 - 1e-4 * a) * th)
                a_acc = np.where(okb, a, a_acc)
                searching &= ~okb
                a = np.where(searching, 0.5 * a, a)
            live &= ~searching                                  # no decrease found: failed
            if not live.any():
                break
            sel = dev_b(live)[:, None] > 0
            yv = torch.where(sel, yv + dev_b(a_acc)[:, None] * dyv, yv)
            lam_r = torch.where(sel, lam_r + dev_b(a_acc)[:, None] * sol[:, ny:], lam_r)
            ft, gt = nlp.eval_fg(yv[:, :n])
            ct = nlp.constraints(gt, yv[:, n:])
            tp = meas.merit(ct, ft, yv, dev_b(mu_t)).cpu().numpy()
            for b in np.where(live)[0]:
                if tp[0, b] <= 0.9 * theta0_[b] and filter_ok(b, tp[0, b], tp[1, b]):
                    succ[b], live[b] = True, False
            if opts.verbose:
                print(f"      restoration: theta {np.round(tp[0][want], 6).tolist()} a {a_acc[want].tolist()} "
                      f"live {live[want].tolist()}", flush=True)
        return succ, yv, lam_r

    # ---- main loop -------------------------------------------------------------------------------
    it = 0
    while it < opts.max_iter:
        c = nlp.constraints(g, y[:, n:])
        # one transfer for the loop head: the convergence errors, the barrier problem's error at the
        # current mu (the first pass of the barrier update below) and theta / phi at the current mu
        # (the line search's reference values, unless mu changes)
        mu_head = dev_b(mu)
        head = meas.head(grad, jv, c, y, lam, zl, zu, f, mu_head).cpu().numpy()
        kkt_err, e_d, e_p, e_c, u_d, u_p, u_c = head[:7]
        e_mu_head, theta_head, phi_head = head[7], head[8], head[9]
        # IPOPT's OptimalityErrorConvergenceCheck: the scaled error and the unscaled tests
        conv = active & (kkt_err <= opts.tol) & (u_d <= opts.dual_inf_tol) & (u_p <= opts.constr_viol_tol) & \
            (u_c <= opts.compl_inf_tol)
        status[conv] = "solve_succeeded"
        active &= ~conv
        acceptable = (kkt_err <= opts.acceptable_tol) & (u_d <= opts.acceptable_dual_inf_tol) & \
            (u_p <= opts.acceptable_constr_viol_tol) & (u_c <= opts.acceptable_compl_inf_tol)
        n_accept = np.where(active & acceptable, n_accept + 1, 0)
        if opts.acceptable_iter > 0:
            acc_stop = active & (n_accept >= opts.acceptable_iter)
            status[acc_stop] = "solved_to_acceptable_level"
            active &= ~acc_stop
        if not active.any():
            break
        # barrier update (monotone), per instance
        mu_changed = False
        for pass_ in range(50):
            e_mu = e_mu_head if pass_ == 0 else meas.barrier_error(grad, jv, c, y, lam, zl, zu, f, dev_b(mu))
            upd = active & (e_mu <= opts.kappa_eps * mu) & (mu > mu_floor * 1.0000001)
            if not upd.any():
                break
            mu_changed = True
            mu = np.where(upd, np.maximum(mu_floor, np.minimum(opts.kappa_mu * mu, mu ** opts.theta_mu)), mu)
            tau = np.maximum(opts.tau_min, 1.0 - mu)
            for b in np.where(upd)[0]:
                filt[b] = []
            in_wd &= ~upd                                     # a new barrier problem: line search reset
            wd_short[upd] = 0
            wd_skip &= ~upd
        # ---- Newton system ----------------------------------------------------------------------
        with _Phase("hessian"):
            hv = nlp.hess(y[:, :n], lam)
        mu_d = dev_b(mu)
        dl, du, sigma, grad_phi, rhs = meas.newton(grad, jv, c, y, lam, zl, zu, mu_d)
        rhs_top = rhs[:, :ny]
        if mu_changed:
            theta, phi = meas.merit(c, f, y, mu_d).cpu().numpy()
        else:
            theta, phi = theta_head, phi_head
        pending = active.copy()
        wd_new = np.zeros(B, dtype=bool)
        if opts.watchdog_shortened_iter_trigger > 0:
            wd_new = active & ~in_wd & ~wd_skip & (wd_short >= opts.watchdog_shortened_iter_trigger)
            if wd_new.any():
                in_wd |= wd_new
                wd_trial[wd_new] = 0
                wd_short[wd_new] = 0
                wd_ref[0][wd_new] = theta[wd_new]
                wd_ref[1][wd_new] = phi[wd_new]
                seln = dev_b(wd_new)[:, None] > 0
                if wd_pt is None:
                    wd_pt = [t.clone() for t in (y, lam, zl, zu)]
                wd_pt = [torch.where(seln, t, r) for t, r in zip((y, lam, zl, zu), wd_pt)]
        wd_restore = np.zeros(B, dtype=bool)
        acc_all = np.zeros(B, dtype=bool)
        alpha_acc = np.zeros(B)
        y_new, dy_new, dlam_new = y.clone(), torch.zeros(B, ny, **f64), torch.zeros(B, m, **f64)
        dw_rec = np.zeros(B)
        nback = np.zeros(B, dtype=np.int64)
        nsoc = np.zeros(B, dtype=np.int64)
        tau_d = dev_b(tau)
        for dw_floor in (0.0, 1e-2, 1.0, 1e2):
            if not pending.any():
                break
            ok, sol, dw_used, dw_fin, dc_fin = newton_direction(pending, dw_floor, hv, sigma, rhs, mu)
            want = pending & ok
            if want.any():
                # the factorisation in skkt is the last attempt's: the accepted (delta_w, delta_c)
                # of every instance that found a direction (others were still growing)
                acc, a_o, y_o, dy_o, dl_o, nb_, ns_, a_max, wd_fail = line_search(
                    want, sol[:, :ny], sol[:, ny:], rhs_top, c, dl, du, theta, phi, grad_phi, tau_d, mu,
                    wd=in_wd & want, wd_ref=wd_ref, skip_first=wd_skip & want, wd_new=wd_new & want)
                # steps shortened by the line search count toward the watchdog's trigger
                norm_acc = acc & ~in_wd
                short = norm_acc & (a_o < a_max * (1.0 - 1e-14))
                wd_short = np.where(short, wd_short + 1, np.where(norm_acc, 0, wd_short))
                in_wd &= ~acc                                     # a watchdog step accepted: the watchdog ends
                if wd_fail.any():
                    wd_trial[wd_fail] += 1
                    back = wd_fail & (wd_trial > opts.watchdog_trial_iter_max)
                    go_on = wd_fail & ~back
                    # within the watchdog's trials: the full step is taken anyway
                    if go_on.any():
                        sel_g = dev_b(go_on)[:, None] > 0
                        dyg = sol[:, :ny]
                        y_o = torch.where(sel_g, y + dev_b(np.where(go_on, a_max, 0.0))[:, None] * dyg, y_o)
                        dy_o = torch.where(sel_g, dyg, dy_o)
                        dl_o = torch.where(sel_g, sol[:, ny:], dl_o)
                        a_o = np.where(go_on, a_max, a_o)
                        acc = acc | go_on
                    # too many: back to the watchdog's starting point, whose line search skips the full step
                    in_wd &= ~back
                    wd_restore |= back
                    pending &= ~back
                sel = dev_b(acc)[:, None] > 0
                y_new = torch.where(sel, y_o, y_new)
                dy_new = torch.where(sel, dy_o, dy_new)
                dlam_new = torch.where(sel, dl_o, dlam_new)
                alpha_acc = np.where(acc, a_o, alpha_acc)
                dw_rec = np.where(acc, dw_used, dw_rec)
                nback += nb_
                nsoc += ns_
                acc_all |= acc
                pending &= ~acc
        # ---- restoration for the instances without an acceptable step ---------------------------
        rest_ok = np.zeros(B, dtype=bool)
        wd_skip[:] = False
        if pending.any():
            in_wd &= ~pending                                 # no watchdog across a restoration phase
            wd_short[pending] = 0
            succ, y_r, lam_r = restoration(pending, c, theta, mu)
            failed = pending & ~succ
            status[failed] = "restoration_failed"
            active &= ~failed
            rest_ok = succ
            if succ.any():
                for b in np.where(succ)[0]:
                    filt[b].append(((1 - opts.gamma_theta) * theta[b], phi[b] - opts.gamma_phi * theta[b]))
                sel = dev_b(succ)[:, None] > 0
                y = torch.where(sel, y_r, y)
                lam = torch.where(sel, lam_r, lam)
        # ---- accepted steps: primal, multipliers, bound multipliers; the kappa_sigma safeguard -------
        # (a watchdog that failed returns its instances to the watchdog's starting point, whose next
        # direction is the one the watchdog started with, and skips the full step there)
        restore = (wd_restore, wd_pt) if wd_restore.any() else None
        y, lam, zl, zu, az_dev = meas.step(acc_all, y, y_new, dy_new, lam, dlam_new, zl, zu, dl, du, mu_d, tau_d,
                                           alpha_acc, restore)
        if restore is not None:
            wd_skip |= wd_restore
        with _Phase("eval_all"):
            f, grad, g, jv = nlp.eval_all(y[:, :n])
        if rest_ok.any():
            # IPOPT after restoration: constraint multipliers by least squares on the dual
            # infeasibility, [I A^T; A 0] (w, lam) = (-(grad f - z_L + z_U), 0)
            skkt.factor(hv_zero, torch.ones(B, ny, **f64), jv, 0.0, mI)
            sol = skkt.solve(torch.cat([-(grad_y(grad) - zl + zu), torch.zeros(B, m, **f64)], 1), active=rest_ok)
            fin = torch.isfinite(sol).all(1)
            sel = (dev_b(rest_ok)[:, None] > 0) & fin[:, None]
            lam = torch.where(sel, sol[:, ny:], lam)
        it += 1
        stepped = acc_all | rest_ok
        iters += stepped
        f_host, alpha_z = torch.stack([f / nlp.obj_scale, az_dev]).cpu().numpy()
        for b in np.where(stepped)[0]:
            rec = dict(it=int(iters[b]), f=float(f_host[b]), inf_pr=float(e_p[b]), inf_du=float(e_d[b]), mu=float(mu[b]),
                       alpha=float(alpha_acc[b]) if acc_all[b] else 0.0,
                       alpha_z=float(alpha_z[b]) if acc_all[b] else 0.0,
                       delta_w=float(dw_rec[b]) if acc_all[b] else -1.0,
                       backtracks=int(nback[b]), soc=int(nsoc[b]))
            logs[b].append(rec)
        if opts.callback is not None:
            # IPOPT's intermediate callback (awebox's iteration_callback, opti/preparation.py:305-313):
            # the full V of every instance after the iteration, and which instances stepped
            opts.callback(it, nlp.full_x(y[:, :n]), stepped.copy())
        if opts.verbose:
            shown = np.where(active | (pending & ~rest_ok))[0]
            for b0 in (shown if B <= 4 else shown[:1]):
                print(f"{it:4d} active={int(active.sum())} [b{b0}] f={f_host[b0]: .8e} pr={e_p[b0]:.2e} "
                      f"du={e_d[b0]:.2e} mu={mu[b0]:.1e} a={alpha_acc[b0]:.2e} dw={dw_rec[b0]:.1e} "
                      f"bt={nback[b0]} soc={nsoc[b0]} th={theta[b0]:.2e}"
                      + (" RESTORATION" if pending[b0] else ""), flush=True)
    for b in range(B):
        if status[b] == "max_iter" and kkt_err[b] <= opts.acceptable_tol:
            status[b] = "solved_to_acceptable_level"
    c = nlp.constraints(g, y[:, n:])
    yh = y[:, :n].cpu().numpy()
    lam_out = (lam * nlp.c_scale / nlp.obj_scale[:, None]).cpu().numpy()
    viol = (c / nlp.c_scale).abs().amax(1).cpu().numpy() if m else np.zeros(B)
    zl_h = (zl[:, :n] / nlp.obj_scale[:, None]).cpu().numpy()
    zu_h = (zu[:, :n] / nlp.obj_scale[:, None]).cpu().numpy()
    f_out = (f / nlp.obj_scale).cpu().numpy()
    seconds = time.perf_counter() - t_start
    out = []
    for b in range(B):
        xf = nlp.x_fix.copy()
        xf[nlp.free] = yh[b]
        zl_v = np.zeros(len(xf))
        zu_v = np.zeros(len(xf))
        zl_v[nlp.free] = zl_h[b]
        zu_v[nlp.free] = zu_h[b]
        out.append(IpmResult(x=xf, lam_g=lam_out[b], f=float(f_out[b]), status=str(status[b]),
                             iterations=int(iters[b]), kkt_error=float(kkt_err[b]), constr_viol=float(viol[b]),
                             seconds=seconds, zl=zl_v, zu=zu_v, log=logs[b], kkt_solves=skkt.n_solve,
                             kkt_dense=skkt.n_dense, timing=timing))
    return out
