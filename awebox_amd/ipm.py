"""Primal-dual interior-point NLP solver on the GPU.

The reference hands the collocation NLP to IPOPT through ``casadi.nlpsol`` (opti/preparation.py:
366-400) and drives it through the homotopy (opti/optimization.py:273-382).  IPOPT is not
available here, so this module restates the IPOPT algorithm (Waechter & Biegler, Math. Prog.
106, 2006) at the level the AP2 problem needs, with every piece of data on the device:

* NLP functions, gradient, Jacobian and the exact Hessian of the Lagrangian come from the HIP
  evaluator (awebox_amd.evaluator) on device tensors;
* the primal-dual KKT system [W + Sigma + dw I, A^T; A, -dc I] is solved by structured
  elimination (StructuredKKT: batched LU of the interval interiors on the awelu kernel, a dense
  or block-tridiagonal Schur complement on the separators), assembled in a fixed summation order
  (deterministic gather-sum tables); the inertia correction uses the curvature test of Chiang &
  Zavala (2016) instead of an inertia-revealing factorisation;
* fixed variables (lbx == ubx) are removed (IPOPT's fixed_variable_treatment=make_parameter);
  inequality rows get slacks; gradient-based NLP scaling, bound push, monotone Fiacco-McCormick
  barrier update, fraction-to-the-boundary rule and the filter line search follow IPOPT's
  defaults (tol 1e-8, mu_init 0.1, kappa_mu 0.2, theta_mu 1.5, tau_min 0.99);
* after a failed line search: a retry with stronger regularisation, then a reduced feasibility
  restoration (Gauss-Newton steps on ||c|| inside the bounds until the filter accepts).

What is left out: second-order corrections, IPOPT's full restoration-phase NLP, and quasi-Newton
options.
"""
from __future__ import annotations

import math
import time
import warnings
from dataclasses import dataclass, field

import numpy as np
import torch

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
    kkt: str = "structured"          # "structured" (interval elimination + Schur) or "dense"
    lu_backend: str = "awelu"        # interval-block LU: "awelu" (batched_lu.hip) or "torch" (rocSOLVER)
    separators: str = "btd"          # separator system: "dense" LU or "btd" (awebox_amd/btd.py block sweep)
    deterministic: bool = True       # KKT assembly by gather-sum tables instead of atomic scatter-adds
    inertia: str = "exact"           # inertia correction: "curvature" test (Chiang & Zavala) or "exact" (IPOPT:
                                     # In(K) = In(K_II) + In(S) from symmetric eigenvalues of the blocks)
    profile: bool = False            # synchronise and time the solver's phases (IpmResult.timing)
    verbose: bool = False


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
    """Evaluator-backed NLP restricted to the free variables, with slacks for inequality rows."""

    def __init__(self, ev, P, lbx, ubx, lbg, ubg, device):
        self.ev, self.dev = ev, device
        n_v, n_g = ev.n_v, ev.n_g
        self.P = torch.tensor(np.asarray(P, dtype=np.float64).reshape(1, -1), device=device)
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
        # bounds of y = [x_free; s]
        yl = np.concatenate([lbx[self.free], lbg[self.ineq]])
        yu = np.concatenate([ubx[self.free], ubg[self.ineq]])
        self.yl = torch.tensor(yl, device=device)
        self.yu = torch.tensor(yu, device=device)
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
        B = 1
        self.V = torch.tensor(self.x_fix.reshape(1, -1), device=device)
        self.f = torch.zeros(B, dtype=torch.float64, device=device)
        self.g = torch.zeros(B, n_g, dtype=torch.float64, device=device)
        self.grad = torch.zeros(B, n_v, dtype=torch.float64, device=device)
        self.jac = torch.zeros(B, ev.nnz, dtype=torch.float64, device=device)
        self.H = torch.zeros(B, ev.nnz_h, dtype=torch.float64, device=device)
        self.sig = torch.ones(B, dtype=torch.float64, device=device)
        self.free_t = torch.tensor(self.free, device=device)
        self.ineq_t = torch.tensor(self.ineq, device=device)
        self.obj_scale = 1.0
        self.c_scale = torch.ones(n_g, dtype=torch.float64, device=device)

    def full_x(self, x):
        self.V[0, self.free_t] = x
        return self.V

    def eval_all(self, x):
        """f, grad_f (reduced), c(y) pieces: g(x) and the Jacobian values (reduced, scaled)."""
        self.ev.eval_nlp_device(self.full_x(x), self.P, self.f, self.g, self.grad, self.jac)
        f = self.f[0] * self.obj_scale
        grad = self.grad[0, self.free_t] * self.obj_scale
        g = self.g[0] * self.c_scale
        jv = self.jac[0, self.j_keep] * self.c_scale[self.j_row]
        return f, grad, g, jv

    def eval_fg(self, x):
        self.ev.eval_nlp_device(self.full_x(x), self.P, self.f, self.g, self.grad, self.jac)
        return self.f[0] * self.obj_scale, self.g[0] * self.c_scale

    def hess(self, x, lam):
        """Hessian of obj_scale f + (c_scale lam)^T g, reduced upper values."""
        lam_unscaled = (lam * self.c_scale).reshape(1, -1).contiguous()
        self.sig[0] = self.obj_scale
        self.ev.eval_hess_device(self.full_x(x), self.P, self.sig, lam_unscaled, self.H)
        return self.H[0, self.h_keep]

    def constraints(self, g, s):
        """c(y) = [g_E - target; g_I - s] (scaled rows)."""
        c = g - self.g_target * self.c_scale
        c = c.clone()
        c[self.ineq_t] = c[self.ineq_t] - s
        return c


class _Csr:
    """Fixed COO pattern as a CSR operator: y = A(vals) x through a sparse matrix-vector product
    (no atomics; fp64 scatter-adds with many duplicates are slow on the GPU)."""

    def __init__(self, rows, cols, shape, dev):
        rows = np.asarray(rows, dtype=np.int64)
        cols = np.asarray(cols, dtype=np.int64)
        order = np.lexsort((cols, rows))
        self.perm = torch.tensor(order, device=dev)
        self.col = torch.tensor(cols[order], device=dev)
        self.crow = torch.tensor(np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=shape[0]))]),
                                 dtype=torch.int64, device=dev)
        self.shape = shape

    def mv(self, vals, x):
        with warnings.catch_warnings():
            warnings.filterwarnings("ignore", message="Sparse CSR tensor support is in beta state")
            A = torch.sparse_csr_tensor(self.crow, self.col, vals[self.perm], size=self.shape)
        return (A @ x.unsqueeze(1)).squeeze(1)


class _ScatterSum:
    """out[..., dst[i]] += vals[..., i] for a fixed index pattern, deterministically and without
    atomics: the duplicates of every destination are pre-grouped on the host into gather tables
    (one per power-of-two bucket of the multiplicity, padding -> a zero slot), so a few gathers,
    row sums and plain indexed stores replace index_put_(accumulate=True) / index_add_, whose
    atomics add duplicates in a run-dependent order (the homotopy path is
    sensitive to that roundoff).  Leading (batch) dimensions of ``out`` and ``vals`` are kept."""

    def __init__(self, dst, dev):
        dst = np.asarray(dst, dtype=np.int64).reshape(-1)
        self.n_src = len(dst)
        order = np.argsort(dst, kind="stable")
        uniq, start, count = np.unique(dst[order], return_index=True, return_counts=True)
        self.buckets = []
        lo, width = 0, 1
        while lo < (count.max() if len(count) else 0):
            sel = np.where((count > lo) & (count <= width))[0]
            if len(sel):
                table = np.full((len(sel), width), len(dst), dtype=np.int64)
                for w in range(width):
                    has = count[sel] > w
                    table[has, w] = order[start[sel][has] + w]
                self.buckets.append((torch.tensor(uniq[sel], device=dev), torch.tensor(table, device=dev)))
            lo, width = width, 2 * width

    def add_into(self, out, vals):
        ext = torch.cat([vals, vals.new_zeros(vals.shape[:-1] + (1,))], dim=-1)
        for d, table in self.buckets:
            out[..., d] += ext[..., table].sum(dim=-1)
        return out


class _GatherMv:
    """y = A(vals) x for a fixed COO pattern: products vals * x[cols], summed per row by a
    _ScatterSum (fixed order).  Replaces rocSPARSE's CSR SpMV, whose adaptive algorithm splits
    long rows (the t_f column of J, i.e. a row of J^T) across workgroups with atomic adds."""

    def __init__(self, rows, cols, shape, dev):
        self.cols = torch.tensor(np.asarray(cols, dtype=np.int64), device=dev)
        self.sum = _ScatterSum(rows, dev)
        self.shape = shape

    def mv(self, vals, x):
        out = x.new_zeros(x.shape[:-1] + (self.shape[0],))
        return self.sum.add_into(out, vals * x[..., self.cols])


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


ZERO_PIVOT = 1e-30   # relative zero-pivot threshold of the inertia count: KKT pivots legitimately span
                     # 1e-10 .. 1e10 at small mu, so only exactly singular columns count as zero


class StructuredKKT:
    """KKT solve by elimination of every interval's interior unknowns (batched dense LU on the
    GPU) and a dense Schur complement on the separators.

    Intervals of the collocation NLP couple only through the shooting states x[k] (shared by
    interval k and the continuity rows of interval k-1), the free global variables (t_f and
    the homotopy parameters) and the periodicity rows.  Those, and the multipliers of the
    continuity rows, are the separators S; everything else -- u[k], xdot[k], z[k], the
    collocation variables, the path slacks and the multipliers of interval k's node, path and
    collocation rows -- is interior to interval k.  With K = [K_II, K_IS; K_SI, K_SS]:
        S = K_SS - sum_k K_SI^k (K_II^k)^-1 K_IS^k,
    about 5 GFLOP at N=40 instead of the 1.3 TFLOP of a dense LU of the whole system."""

    def __init__(self, nlp, lay, dev, lu_backend="awelu", separators="btd", deterministic=False):
        n, ny, m = nlp.n, nlp.ny, nlp.m
        self.lu_backend = lu_backend
        N = ny + m
        self.N, self.dev = N, dev
        n_k, stride, v0, rows = lay.n_k, lay.interval_stride, lay.v_intervals, lay.rows_per_interval
        nx = getattr(lay, "nx", pb.NX)                          # states per shooting node
        owner = np.full(N, -1, dtype=np.int64)                  # interval of an interior unknown
        for p, v in enumerate(nlp.free):
            if v >= v0:
                k, o = divmod(v - v0, stride)
                if k < n_k and o >= nx:
                    owner[p] = k
        for i, r in enumerate(nlp.ineq):
            owner[n + i] = r // rows if r < n_k * rows else -1     # global rows (t_f bounds): separators
        # interval rows, except the continuity rows: an interval has more rows than interior
        # unknowns (x[k], x[k+1] close the count), so their multipliers join the separators
        rr = np.arange(m)
        owner[ny + rr] = np.where((rr < n_k * rows) & (rr % rows < rows - nx), rr // rows, -1)
        self.owner = owner
        sep = np.where(owner < 0)[0]
        self.nS = len(sep)
        sep_id = np.full(N, -1, dtype=np.int64)
        sep_id[sep] = np.arange(self.nS)
        loc = np.full(N, -1, dtype=np.int64)
        counts = np.zeros(n_k, dtype=np.int64)
        for p in np.where(owner >= 0)[0]:
            loc[p] = counts[owner[p]]
            counts[owner[p]] += 1
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
        self.csr = _Csr(P_, Q_, (N, N), dev)
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
        self.dst_ii = torch.tensor(oP[ii] * nI * nI + loc[P_[ii]] * nI + loc[Q_[ii]], device=dev)
        isi = np.where(is_)[0]
        self.sel_is = torch.tensor(isi, device=dev)
        self.dst_is = torch.tensor(oP[isi] * nI * L + loc[P_[isi]] * L + lpos[oP[isi], sep_id[Q_[isi]]], device=dev)
        self.sel_ss = torch.tensor(np.where(ss)[0], device=dev)
        self.dst_ss = torch.tensor(sep_id[P_[ss]] * (nS + 1) + sep_id[Q_[ss]], device=dev)
        pad = [(k, j) for k in range(n_k) for j in range(int(counts[k]), nI)]
        self.pad_flat = torch.tensor([k * nI * nI + j * nI + j for k, j in pad], dtype=torch.int64, device=dev)
        r_idx = self.lsep[:, :, None].expand(n_k, L, L)
        c_idx = self.lsep[:, None, :].expand(n_k, L, L)
        self.schur_flat = (r_idx * (nS + 1) + c_idx).reshape(-1)
        int_p = np.where(owner >= 0)[0]
        self.int_p = torch.tensor(int_p, device=dev)
        self.sc = None
        if deterministic:
            self.sc = [_ScatterSum(t.cpu().numpy(), dev) for t in (self.dst_ii, self.dst_is, self.dst_ss,
                                                                    self.schur_flat)]
            self.sc_mv = _ScatterSum(P_, dev)
            self.sc_dense = _ScatterSum(P_ * N + Q_, dev)
            self.sc_rs = _ScatterSum(lsep_arr.reshape(-1), dev)
        # separators in stages [c[k-1], x[k]] (block tridiagonal, globals as border): pairing each
        # shooting state with the multipliers of the continuity row that defines it keeps the block
        # sweep's pivot blocks regular -- the finer order x[0], c[0], x[1], ... meets near-singular
        # pivot blocks at N=40 (cond 3e17 on the AP2 KKT); the paired one stays at cond <= 1e13
        # with |W_k| <= 60, a backward error of 2e-21 (emulated on the CPU)
        self.btd = None
        self.force_btd = False                                  # CPU tests: the BTD path on host
        self.btd_off = False                                    # the dense separator LU even when btd exists
        from .batched_lu import BTD_MAX_M
        if lu_backend == "awelu" and separators == "btd" and 2 * nx <= BTD_MAX_M:
            stage_of = np.full(self.nS, -1, dtype=np.int64)
            pos_of = np.zeros(self.nS, dtype=np.int64)
            free = np.asarray(nlp.free.cpu().numpy() if torch.is_tensor(nlp.free) else nlp.free)
            for q, p in enumerate(sep):
                if p < n:
                    v = int(free[p])
                    if v >= v0:
                        k, o = divmod(v - v0, stride)
                        if o < nx and k <= n_k:
                            stage_of[q], pos_of[q] = k, nx + o
                elif p >= ny:
                    r = p - ny
                    if r < n_k * rows and r % rows >= rows - nx:
                        stage_of[q], pos_of[q] = r // rows + 1, r % rows - (rows - nx)
            ss_r, ss_c = sep_id[P_[ss]], sep_id[Q_[ss]]
            sch_r, sch_c = lsep_arr[:, :, None].repeat(L, 2), lsep_arr[:, None, :].repeat(L, 1)
            from .btd import BorderedBtd
            try:
                self.btd = BorderedBtd(stage_of, pos_of, n_k + 1, 2 * nx,
                                       np.concatenate([ss_r, sch_r.reshape(-1)]),
                                       np.concatenate([ss_c, sch_c.reshape(-1)]), dev,
                                       deterministic=deterministic)
            except ValueError:
                self.btd = None                                 # not stage-structured: dense S
        self.int_flat = torch.tensor(owner[int_p] * nI + loc[int_p], device=dev)
        self.sep_p = torch.tensor(sep, device=dev)

    def factor(self, hv, diag, jv, delta_c, mI):
        f64 = dict(dtype=torch.float64, device=self.dev)
        m = self.N - diag.numel()
        vals = torch.cat([hv, hv[self.off_mask], diag, jv, jv, -torch.ones(2 * mI, **f64),
                          torch.full((m,), -float(delta_c), **f64)])
        self.vals = vals
        self.k_norm = float(self._mv(vals.abs(), torch.ones(self.N, **f64)).max().item())
        nI, L, nS, n_k = self.nI, self.L, self.nS, self.n_k
        KII = torch.zeros(n_k * nI * nI, **f64)
        if self.sc:
            self.sc[0].add_into(KII, vals[self.sel_ii])
        else:
            KII.index_put_((self.dst_ii,), vals[self.sel_ii], accumulate=True)
        KII[self.pad_flat] = 1.0
        KII = KII.view(n_k, nI, nI)
        self.KII = KII
        KIS = torch.zeros(n_k * nI * L, **f64)
        if self.sc:
            self.sc[1].add_into(KIS, vals[self.sel_is])
        else:
            KIS.index_put_((self.dst_is,), vals[self.sel_is], accumulate=True)
        KIS = KIS.view(n_k, nI, L)
        self.awelu = self.lu_backend == "awelu" and KII.is_cuda   # the CPU test harness uses LAPACK
        if self.awelu:
            from .batched_lu import lu_factor
            self.LU_I, self.piv_I = lu_factor(KII)
        else:
            self.LU_I, self.piv_I = torch.linalg.lu_factor(KII)
        self.X = self._block_solve(KIS)                                        # K_II^-1 K_IS
        T = KIS.transpose(1, 2) @ self.X                                       # [n_k, L, L]
        self.KIS = KIS
        if self.btd is not None and not self.btd_off and (KII.is_cuda or self.force_btd):
            self.btd.factor(torch.cat([vals[self.sel_ss], -T.reshape(-1)]))
            self.use_btd = True
            return
        self.use_btd = False
        S = torch.zeros((nS + 1) * (nS + 1), **f64)
        if self.sc:
            self.sc[2].add_into(S, vals[self.sel_ss])
            self.sc[3].add_into(S, -T.reshape(-1))
        else:
            S.index_put_((self.dst_ss,), vals[self.sel_ss], accumulate=True)
            S.index_put_((self.schur_flat,), -T.reshape(-1), accumulate=True)
        S = S.view(nS + 1, nS + 1)
        S[nS, :] = 0.0
        S[:, nS] = 0.0
        S[nS, nS] = 1.0
        self.S = S
        self.LU_S, self.piv_S = torch.linalg.lu_factor(S)

    def inertia(self):
        """(positive, negative, zero) eigenvalue counts of K by Haynsworth's additivity,
        In(K) = sum_k In(K_II^k) + In(S): Bunch-Kaufman inertia of the interval blocks (padding
        rows excluded) and of the separator system -- the dense Schur complement S, or with the
        block-tridiagonal separators the sweep's pivot blocks and the border (btd.BorderedBtd)."""
        from .batched_lu import sym_inertia, sym_inertia_host
        f = sym_inertia if self.KII.is_cuda else sym_inertia_host
        c = f(self.KII, ztol=ZERO_PIVOT).to(torch.int64).sum(0)
        c[0] -= len(self.pad_flat)
        if self.use_btd:
            c = c + self.btd.inertia()[0]
        else:
            cs = f(self.S.unsqueeze(0), ztol=ZERO_PIVOT).to(torch.int64)[0]
            cs[0] -= 1                                          # the dummy separator's 1.0
            c = c + cs
        pos, neg, zero = (int(v) for v in c.cpu().tolist())
        return pos, neg, zero

    def _mv(self, vals, x):
        """K(vals) x: a fixed-order gather-sum when deterministic, rocSPARSE CSR otherwise."""
        if self.sc:
            return self.sc_mv.add_into(torch.zeros(self.N, dtype=torch.float64, device=self.dev), vals * x[self.Q_])
        return self.csr.mv(vals, x)

    def matvec(self, x):
        return self._mv(self.vals, x)

    def solve(self, rhs, refine=3, rtol=1e-12):
        """Elimination solve with iterative refinement on the sparse residual.  The interior
        pivots come from blocks that may be ill-conditioned even when K is not (an indefinite
        interior Hessian), so the result is accepted once its backward error is small,
        ||K x - rhs|| <= rtol (||K|| ||x|| + ||rhs||) in the max norm; otherwise the system is
        solved once by a dense LU of the assembled K."""
        self.n_solve += 1
        x = self._solve(rhs)
        b_norm = float(rhs.abs().max().item())
        self.backward = []
        for _ in range(refine + 1):
            r = rhs - self.matvec(x)
            err = float(r.abs().max().item())
            if not math.isfinite(err):
                break
            scale = self.k_norm * float(x.abs().max().item()) + b_norm
            self.backward.append(err / scale)
            if err <= rtol * scale:
                return x
            x = x + self._solve(r)
        # ill-conditioned interior pivots: one dense LU of the assembled K for this system
        self.n_dense += 1
        K = torch.zeros(self.N * self.N, dtype=torch.float64, device=self.dev)
        if self.sc:
            self.sc_dense.add_into(K, self.vals)
        else:
            K.index_put_((self.P_ * self.N + self.Q_,), self.vals, accumulate=True)
        return torch.linalg.solve(K.view(self.N, self.N), rhs)

    def _block_solve(self, B):
        """K_II^-1 B for all interval blocks: triangular solves on the LU factors (rocBLAS on the
        device, LAPACK in the CPU harness).  The awelu solve kernel (RTI's choice) is not used
        here: it did not change the per-iteration time, and its roundoff moved the bench's 2-point
        AP2 sweep to another local solution at 8 m/s (3,874 W over 60 s instead of 3,799 W over
        29 s)."""
        return torch.linalg.lu_solve(self.LU_I, self.piv_I, B)

    def _solve(self, rhs):
        f64 = dict(dtype=torch.float64, device=self.dev)
        nI, L, nS, n_k = self.nI, self.L, self.nS, self.n_k
        rI = torch.zeros(n_k * nI, **f64)
        rI[self.int_flat] = rhs[self.int_p]
        rI = rI.view(n_k, nI, 1)
        rS = torch.zeros(nS + 1, **f64)
        rS[:nS] = rhs[self.sep_p]
        z = self._block_solve(rI)                                              # [n_k, nI, 1]
        upd = (self.KIS.transpose(1, 2) @ z).reshape(-1)                      # [n_k * L]
        if self.sc:
            self.sc_rs.add_into(rS, -upd)
        else:
            rS = rS.index_add(0, self.lsep.reshape(-1), -upd)
        rS[nS] = 0.0
        if self.use_btd:
            xS = torch.zeros(nS + 1, **f64)
            xS[:nS] = self.btd.solve(rS[:nS])
        else:
            xS = torch.linalg.lu_solve(self.LU_S, self.piv_S, rS.view(-1, 1)).view(-1)
        xI = z.view(n_k, nI) - (self.X @ xS[self.lsep].unsqueeze(-1)).view(n_k, nI)
        sol = torch.empty(self.N, **f64)
        sol[self.int_p] = xI.reshape(-1)[self.int_flat]
        sol[self.sep_p] = xS[:nS]
        return sol


def solve(ev, P, x0, lbx, ubx, lbg, ubg, lam0=None, zl0=None, zu0=None, opts: IpmOptions | None = None,
          device="cuda") -> IpmResult:
    """Solve min f s.t. lbg <= g <= ubg, lbx <= x <= ubx with the GPU interior-point method.

    lam0 / zl0 / zu0 (constraint and V-bound multipliers of a previous solve) select IPOPT's
    warm_start_init_point: the multipliers are kept (pushed away from zero) and the primal point
    is pushed into the bounds with the smaller warm-start push."""
    opts = opts or IpmOptions()
    t_start = time.perf_counter()
    dev = torch.device(device)
    nlp = DeviceNlp(ev, P, lbx, ubx, lbg, ubg, dev)
    n, mI, m, ny = nlp.n, nlp.mI, nlp.m, nlp.ny
    N = ny + m
    f64 = dict(dtype=torch.float64, device=dev)
    log = []

    # ---- initial point: bound push (IPOPT 3.6) -----------------------------------------------
    x = torch.tensor(np.asarray(x0, dtype=np.float64)[nlp.free], **f64)
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

    # gradient-based NLP scaling at the starting point (IPOPT nlp_scaling_method)
    f0, grad0, g0, jv0 = nlp.eval_all(push(torch.cat([x, torch.zeros(mI, **f64)]))[:n])
    gmax = float(grad0.abs().max().item()) if n else 0.0
    nlp.obj_scale = min(1.0, opts.nlp_scaling_max_gradient / gmax) if gmax > 0 else 1.0
    rowmax = torch.zeros(m, **f64).scatter_reduce_(0, nlp.j_row, jv0.abs(), "amax", include_self=True)
    nlp.c_scale = torch.clamp(opts.nlp_scaling_max_gradient / torch.clamp(rowmax, min=1e-300), max=1.0)
    # slack bounds live in the scaled constraint space
    cs_I = nlp.c_scale[nlp.ineq_t]
    nlp.yl[n:] = torch.where(nlp.has_l[n:], nlp.yl[n:] * cs_I, nlp.yl[n:])
    nlp.yu[n:] = torch.where(nlp.has_u[n:], nlp.yu[n:] * cs_I, nlp.yu[n:])

    y = torch.cat([x, torch.zeros(mI, **f64)])
    f, grad, g, jv = nlp.eval_all(y[:n])
    y[n:] = g[nlp.ineq_t]
    y = push(y)
    lam = torch.zeros(m, **f64)
    if lam0 is not None:
        lam = torch.tensor(np.asarray(lam0, dtype=np.float64), **f64) / nlp.c_scale * nlp.obj_scale
    zl = torch.where(hl, torch.ones(ny, **f64), torch.zeros(ny, **f64))
    zu = torch.where(hu, torch.ones(ny, **f64), torch.zeros(ny, **f64))
    if warm:
        floor = opts.warm_start_mult_bound_push
        if zl0 is not None:
            zx = torch.tensor(np.asarray(zl0, dtype=np.float64)[nlp.free], **f64) * nlp.obj_scale
            zl[:n] = torch.where(hl[:n], torch.clamp(zx, min=floor), zl[:n])
        if zu0 is not None:
            zx = torch.tensor(np.asarray(zu0, dtype=np.float64)[nlp.free], **f64) * nlp.obj_scale
            zu[:n] = torch.where(hu[:n], torch.clamp(zx, min=floor), zu[:n])
        # slack bound multipliers from the row multipliers: dL/ds = -lam - z_l + z_u = 0
        lamI = lam[nlp.ineq_t]
        zl[n:] = torch.where(hl[n:], torch.clamp(-lamI, min=floor), zl[n:])
        zu[n:] = torch.where(hu[n:], torch.clamp(lamI, min=floor), zu[n:])
    mu = opts.mu_init
    mu_floor = max(opts.mu_target, opts.tol / 10)
    tau = max(opts.tau_min, 1.0 - mu)
    filt = []
    c = nlp.constraints(g, y[n:])
    theta0 = float(c.abs().sum().item())
    theta_max = 1e4 * max(1.0, theta0)
    theta_min = 1e-4 * max(1.0, theta0)
    delta_w_last = 0.0
    skkt = None
    if opts.kkt == "structured" and getattr(ev, "layout", None) is not None:
        try:
            skkt = StructuredKKT(nlp, ev.layout, dev, lu_backend=opts.lu_backend, separators=opts.separators,
                                 deterministic=opts.deterministic)
            skkt.force_btd = opts.separators == "btd"           # the block sweep on host tensors too
        except ValueError:
            skkt = None
    K = torch.zeros(N, N, **f64) if skkt is None else None
    # exact inertia needs the separator pivot blocks of the block sweep on the device (a dense
    # Bunch-Kaufman pass over the whole Schur complement is ~1 s); otherwise the curvature test
    exact_inertia = opts.inertia == "exact" and skkt is not None and (skkt.btd is not None or not dev.type == "cuda")
    timing = {}

    class _Phase:
        def __init__(self, key):
            self.key = key

        def __enter__(self):
            if opts.profile:
                if torch.cuda.is_available() and str(dev).startswith("cuda"):
                    torch.cuda.synchronize()
                self.t = time.perf_counter()

        def __exit__(self, *exc):
            if opts.profile:
                if torch.cuda.is_available() and str(dev).startswith("cuda"):
                    torch.cuda.synchronize()
                timing[self.key] = timing.get(self.key, 0.0) + time.perf_counter() - self.t
            return False
    status = "max_iter"
    it = 0
    kkt_err = math.inf

    def gaps(yv):
        dl = torch.where(hl, yv - yl, torch.ones_like(yv))
        du = torch.where(hu, yu - yv, torch.ones_like(yv))
        return dl, du

    def barrier_phi(fv, yv):
        dl, du = gaps(yv)
        return fv - mu * (torch.log(dl[hl]).sum() + torch.log(du[hu]).sum())

    def grad_y(gradv):
        return torch.cat([gradv, torch.zeros(mI, **f64)])

    Op = _GatherMv if opts.deterministic else _Csr
    jt_op = Op(nlp.j_col.cpu().numpy(), nlp.j_row.cpu().numpy(), (ny, m), dev)
    hr_np, hc_np = nlp.h_r.cpu().numpy(), nlp.h_c.cpu().numpy()
    off_np = hr_np != hc_np
    h_op = Op(np.concatenate([hr_np, hc_np[off_np]]), np.concatenate([hc_np, hr_np[off_np]]), (ny, ny), dev)

    def A_T_lam(jvv, lamv):
        r = jt_op.mv(jvv, lamv)
        r[n:] -= lamv[nlp.ineq_t]
        return r

    def errors(gradv, jvv, cv, yv, lamv, zlv, zuv, mu_):
        dl, du = gaps(yv)
        dual = grad_y(gradv) + A_T_lam(jvv, lamv) - zlv + zuv
        compl_l = torch.where(hl, dl * zlv - mu_, torch.zeros_like(yv))
        compl_u = torch.where(hu, du * zuv - mu_, torch.zeros_like(yv))
        nb = int(hl.sum().item() + hu.sum().item())
        s_d = max(opts.s_max, (lamv.abs().sum() + zlv.abs().sum() + zuv.abs().sum()).item() / max(1, m + nb)) / opts.s_max
        s_c = max(opts.s_max, (zlv.abs().sum() + zuv.abs().sum()).item() / max(1, nb)) / opts.s_max
        e_dual = dual.abs().max().item() / s_d
        e_pr = cv.abs().max().item() if m else 0.0
        e_c = max(compl_l.abs().max().item(), compl_u.abs().max().item()) / s_c
        return max(e_dual, e_pr, e_c), e_dual, e_pr, e_c

    def assemble(Kmat, hv, sigma, delta_w, delta_c):
        Kmat.zero_()
        if hv is not None:
            Kmat[nlp.h_r, nlp.h_c] = hv
            Kmat[nlp.h_c[nlp.h_offdiag], nlp.h_r[nlp.h_offdiag]] = hv[nlp.h_offdiag]
        idx = torch.arange(ny, device=dev)
        Kmat[idx, idx] += sigma + delta_w
        _dense_A(nlp, jv, ny, Kmat)
        if delta_c > 0:
            idm = torch.arange(ny, N, device=dev)
            Kmat[idm, idm] = -delta_c

    def max_step(v, dv, mask_pos):
        ratio = torch.where(mask_pos & (dv < 0), -tau * v / dv, torch.full_like(v, math.inf))
        return min(1.0, float(ratio.min().item())) if ratio.numel() else 1.0

    hv_zero = torch.zeros(len(nlp.h_keep), **f64)

    def restoration(y0, c0, theta0_, phi0_, max_steps=50):
        """Minimum-norm Gauss-Newton corrections toward c(y) = 0, scaled by the barrier Sigma,
        with backtracking on theta; returns (y, lam) once the point is acceptable to the filter."""
        yv, cv, th = y0, c0, theta0_
        lam_r = lam
        for _ in range(max_steps):
            _, _, g_c, jv_c = nlp.eval_all(yv[:n])
            cv = nlp.constraints(g_c, yv[n:])
            th = float(cv.abs().sum().item())
            dlv, duv = gaps(yv)
            sig = torch.where(hl, 1.0 / dlv ** 2, torch.zeros_like(yv)) + torch.where(hu, 1.0 / duv ** 2, torch.zeros_like(yv))
            rhs = -torch.cat([torch.zeros(ny, **f64), cv])
            try:
                if skkt is not None:
                    skkt.factor(hv_zero, sig + 1e-8, jv_c, 0.0, mI)
                    sol = skkt.solve(rhs)
                else:
                    assemble_jv(K, jv_c, sig + 1e-8)
                    sol = torch.linalg.solve(K, rhs)
            except RuntimeError:
                return None
            dyv = sol[:ny]
            a = min(max_step(dlv, dyv, hl), max_step(duv, -dyv, hu))
            for _ in range(30):
                yt = yv + a * dyv
                ft, gt = nlp.eval_fg(yt[:n])
                ct = nlp.constraints(gt, yt[n:])
                tht = float(ct.abs().sum().item())
                if math.isfinite(tht) and tht < (1 - 1e-4 * a) * th:
                    break
                a *= 0.5
            else:
                return None
            yv = yt
            lam_r = lam_r + a * sol[ny:]
            pht = float(barrier_phi(ft, yt).item())
            if tht <= 0.9 * theta0_ and all(not (tht >= th_f and pht >= ph_f) for th_f, ph_f in filt):
                return yv, lam_r
        return None

    def assemble_jv(Kmat, jv_c, diag):
        Kmat.zero_()
        idx = torch.arange(ny, device=dev)
        Kmat[idx, idx] = diag
        _dense_A(nlp, jv_c, ny, Kmat)

    while it < opts.max_iter:
        c = nlp.constraints(g, y[n:])
        kkt_err, e_d, e_p, e_c = errors(grad, jv, c, y, lam, zl, zu, opts.mu_target)
        if kkt_err <= opts.tol:
            status = "solve_succeeded"
            break
        # barrier update (monotone)
        while True:
            e_mu = errors(grad, jv, c, y, lam, zl, zu, mu)[0]
            if e_mu > opts.kappa_eps * mu or mu <= mu_floor * 1.0000001:
                break
            mu = max(mu_floor, min(opts.kappa_mu * mu, mu ** opts.theta_mu))
            tau = max(opts.tau_min, 1.0 - mu)
            filt = []
        # ---- Newton system --------------------------------------------------------------------
        with _Phase("hessian"):
            hv = nlp.hess(y[:n], lam)
        dl, du = gaps(y)
        sigma = torch.where(hl, zl / dl, torch.zeros_like(y)) + torch.where(hu, zu / du, torch.zeros_like(y))
        grad_phi = grad_y(grad) - torch.where(hl, mu / dl, torch.zeros_like(y)) + torch.where(hu, mu / du, torch.zeros_like(y))
        theta = float(c.abs().sum().item())
        phi = float(barrier_phi(f, y).item())

        def newton_direction(dw_floor):
            """(dy, dlam, delta_w) with the curvature-tested inertia correction."""
            nonlocal delta_w_last
            rhs = -torch.cat([grad_phi + A_T_lam(jv, lam), c])
            delta_w = dw_floor
            delta_c = 0.0
            for attempt in range(60):
                try:
                    with _Phase("kkt_factor"):
                        if skkt is not None:
                            skkt.factor(hv, sigma + delta_w, jv, delta_c, mI)
                        else:
                            assemble(K, hv, sigma, delta_w, delta_c)
                    if exact_inertia:
                        # IPOPT's inertia correction (Waechter & Biegler 2006, Alg. IC): a singular
                        # matrix gets delta_c once, a wrong inertia a larger delta_w
                        with _Phase("inertia"):
                            pos, neg, zero = skkt.inertia()
                        # zero or missing negative eigenvalues: a (numerically) rank-deficient
                        # constraint Jacobian -> delta_c; too few positive ones -> delta_w
                        if (zero > 0 or neg < m) and delta_c == 0.0:
                            delta_c = opts.delta_c * mu ** 0.25
                            continue
                        ok = pos == ny and neg == m
                        if ok:
                            with _Phase("kkt_solve"):
                                sol = skkt.solve(rhs)
                            if not bool(torch.isfinite(sol).all().item()):
                                ok = False
                        if ok:
                            if delta_w > 0:
                                delta_w_last = delta_w
                            return sol[:ny], sol[ny:], delta_w
                    else:
                        with _Phase("kkt_solve"):
                            sol = skkt.solve(rhs) if skkt is not None else torch.linalg.solve(K, rhs)
                        ok = bool(torch.isfinite(sol).all().item())
                        if ok:
                            dy = sol[:ny]
                            Wd = h_op.mv(torch.cat([hv, hv[nlp.h_offdiag]]), dy)
                            curv = float((dy * (Wd + (sigma + delta_w) * dy)).sum().item())
                            if curv >= opts.curvature_kappa * float((dy * dy).sum().item()):
                                if delta_w > 0:
                                    delta_w_last = delta_w
                                return sol[:ny], sol[ny:], delta_w
                        else:
                            delta_c = opts.delta_c * mu ** 0.25
                except RuntimeError:
                    delta_c = opts.delta_c * mu ** 0.25
                if delta_w == 0.0:
                    delta_w = opts.delta_w0 if delta_w_last == 0.0 else max(opts.delta_w_min, delta_w_last / 3.0)
                else:
                    delta_w *= 8.0 if delta_w_last > 0 else 100.0
                if delta_w > opts.delta_w_max:
                    return None
            return None

        def acceptable(alpha, theta_t, phi_t, gphi_d):
            """IPOPT's filter acceptance of a trial point (switching condition + Armijo, or
            sufficient decrease of theta or phi, and acceptability to the filter)."""
            if not (math.isfinite(theta_t) and math.isfinite(phi_t)):
                return False, False
            switching = gphi_d < 0 and alpha * (-gphi_d) ** opts.s_phi > opts.delta_switch * theta ** opts.s_theta
            if theta <= theta_min and switching:
                ok = phi_t <= phi + opts.eta_phi * alpha * gphi_d
                f_type = True
            else:
                ok = theta_t <= theta_max and (theta_t <= (1 - opts.gamma_theta) * theta or
                                               phi_t <= phi - opts.gamma_phi * theta)
                f_type = False
            ok = ok and all(not (theta_t >= th_f and phi_t >= ph_f) for th_f, ph_f in filt)
            return ok, f_type

        def trial(yt):
            with _Phase("eval_fg"):
                ft, gt = nlp.eval_fg(yt[:n])
            ct = nlp.constraints(gt, yt[n:])
            return ct, float(ct.abs().sum().item()), float(barrier_phi(ft, yt).item())

        def line_search(dy, dlam, rhs_top):
            """Filter line search from the fraction-to-the-boundary step, with IPOPT's second-order
            corrections when the first trial is rejected with theta_trial >= theta.  Returns
            (alpha, y_trial, dy, dlam) -- dy/dlam replaced by the corrected step when a
            correction was accepted -- or None."""
            nonlocal filt
            alpha = min(max_step(dl, dy, hl), max_step(du, -dy, hu))
            ls_info["alpha_max"] = alpha
            if opts.verbose and alpha < 1.0:
                rl = torch.where(hl & (dy < 0), -tau * dl / dy, torch.full_like(dy, math.inf))
                ru = torch.where(hu & (dy > 0), tau * du / dy, torch.full_like(dy, math.inf))
                r2 = torch.minimum(rl, ru)
                ls_info["ftb_index"] = int(r2.argmin().item())
            ls_info["backtracks"] = 0
            ls_info["soc"] = 0
            gphi_d = float((grad_phi * dy).sum().item())
            alpha_min = opts.alpha_min_frac * min(opts.gamma_theta, opts.gamma_phi * theta / max(-gphi_d, 1e-300)
                                                   if gphi_d < 0 else opts.gamma_theta)
            for bt in range(opts.max_backtracks):
                yt = y + alpha * dy
                ct, theta_t, phi_t = trial(yt)
                ok, f_type = acceptable(alpha, theta_t, phi_t, gphi_d)
                if ok:
                    if not f_type:
                        filt.append(((1 - opts.gamma_theta) * theta, phi - opts.gamma_phi * theta))
                    return alpha, yt, dy, dlam
                if bt == 0 and opts.max_soc > 0 and skkt is not None and math.isfinite(theta_t) and theta_t >= theta:
                    # second-order correction (Waechter & Biegler 2006, section 2.4): same matrix,
                    # constraint part of the right-hand side c_soc = alpha c(y) + c(y_trial)
                    c_soc = alpha * c + ct
                    theta_old = theta_t
                    for _p in range(opts.max_soc):
                        with _Phase("kkt_solve"):
                            sol = skkt.solve(torch.cat([rhs_top, -c_soc]))
                        if not bool(torch.isfinite(sol).all().item()):
                            break
                        dys = sol[:ny]
                        a_s = min(max_step(dl, dys, hl), max_step(du, -dys, hu))
                        ys = y + a_s * dys
                        cs_, theta_s, phi_s = trial(ys)
                        ls_info["soc"] += 1
                        ok, f_type = acceptable(alpha, theta_s, phi_s, gphi_d)
                        if ok:
                            if not f_type:
                                filt.append(((1 - opts.gamma_theta) * theta, phi - opts.gamma_phi * theta))
                            return a_s, ys, dys, sol[ny:]
                        if not math.isfinite(theta_s) or theta_s > opts.kappa_soc * theta_old:
                            break
                        theta_old = theta_s
                        c_soc = a_s * c_soc + cs_
                if opts.verbose and bt < 8:
                    print(f"     ls bt={bt} alpha={alpha:.3e} theta {theta:.6e}->{theta_t:.6e} phi {phi:.10e}->{phi_t:.10e} "
                          f"gphi_d={gphi_d:.3e} theta_min={theta_min:.2e} filt={len(filt)}", flush=True)
                alpha *= 0.5
                ls_info["backtracks"] += 1
                if alpha < alpha_min:
                    break
            return None

        accepted = None
        delta_w = 0.0
        ls_info = {}
        for dw_floor in (0.0, 1e-2, 1.0, 1e2):
            nd = newton_direction(dw_floor)
            if nd is None:
                continue
            dy, dlam, delta_w = nd
            accepted = line_search(dy, dlam, -(grad_phi + A_T_lam(jv, lam)))
            if accepted is not None:
                break
        if accepted is None:
            # feasibility restoration: Gauss-Newton steps on ||c|| inside the bounds until the
            # filter accepts the point (IPOPT's restoration phase, reduced to its core)
            rest = restoration(y, c, theta, phi)
            if rest is None:
                status = "restoration_failed"
                break
            y, lam = rest
            filt.append(((1 - opts.gamma_theta) * theta, phi - opts.gamma_phi * theta))
            dl, du = gaps(y)
            f, grad, g, jv = nlp.eval_all(y[:n])
            if skkt is not None and exact_inertia:
                # IPOPT after restoration: bound multipliers kept within the kappa_sigma band of the
                # new point, constraint multipliers by least squares on the dual infeasibility,
                # [I A^T; A 0] (w, lam) = (-(grad f - z_L + z_U), 0)
                zl = torch.where(hl, torch.clamp(zl, min=mu / (opts.kappa_sigma * dl), max=opts.kappa_sigma * mu / dl), zl)
                zu = torch.where(hu, torch.clamp(zu, min=mu / (opts.kappa_sigma * du), max=opts.kappa_sigma * mu / du), zu)
                try:
                    skkt.factor(hv_zero, torch.ones(ny, **f64), jv, 0.0, mI)
                    sol = skkt.solve(torch.cat([-(grad_y(grad) - zl + zu), torch.zeros(m, **f64)]))
                    if bool(torch.isfinite(sol).all().item()):
                        lam = sol[ny:]
                except RuntimeError:
                    pass
            else:
                zl = torch.where(hl, torch.clamp(mu / dl, max=1e3), zl)
                zu = torch.where(hu, torch.clamp(mu / du, max=1e3), zu)
            it += 1
            log.append(dict(it=it, f=float(f.item()) / nlp.obj_scale, inf_pr=e_p, inf_du=e_d, mu=mu,
                            alpha=0.0, alpha_z=0.0, delta_w=-1.0))
            if opts.verbose:
                print(f"{it:4d} restoration theta {theta:.3e} -> {float(nlp.constraints(g, y[n:]).abs().sum().item()):.3e}",
                      flush=True)
            continue
        alpha, yt, dy, dlam = accepted
        dzl = torch.where(hl, mu / dl - zl - zl / dl * dy, torch.zeros_like(y))
        dzu = torch.where(hu, mu / du - zu + zu / du * dy, torch.zeros_like(y))
        alpha_z = min(max_step(zl, dzl, hl), max_step(zu, dzu, hu))
        y = yt
        lam = lam + alpha * dlam
        zl = zl + alpha_z * dzl
        zu = zu + alpha_z * dzu
        # kappa_sigma safeguard
        dl, du = gaps(y)
        zl = torch.where(hl, torch.clamp(zl, min=mu / (opts.kappa_sigma * dl), max=opts.kappa_sigma * mu / dl), zl)
        zu = torch.where(hu, torch.clamp(zu, min=mu / (opts.kappa_sigma * du), max=opts.kappa_sigma * mu / du), zu)
        with _Phase("eval_all"):
            f, grad, g, jv = nlp.eval_all(y[:n])
        it += 1
        rec = dict(it=it, f=float(f.item()) / nlp.obj_scale, inf_pr=e_p, inf_du=e_d, mu=mu, alpha=alpha,
                   alpha_z=alpha_z, delta_w=delta_w, **ls_info)
        log.append(rec)
        if opts.verbose:
            print(f"{it:4d} f={rec['f']: .8e} pr={e_p:.2e} du={e_d:.2e} mu={mu:.1e} a={alpha:.2e} dw={delta_w:.1e}",
                  flush=True)
    if status == "max_iter" and kkt_err <= opts.acceptable_tol:
        status = "solved_to_acceptable_level"
    xf = nlp.x_fix.copy()
    xf[nlp.free] = y[:n].cpu().numpy()
    lam_out = (lam * nlp.c_scale / nlp.obj_scale).cpu().numpy()
    c = nlp.constraints(g, y[n:])
    zl_v = np.zeros(len(xf))
    zu_v = np.zeros(len(xf))
    zl_v[nlp.free] = (zl[:n] / nlp.obj_scale).cpu().numpy()
    zu_v[nlp.free] = (zu[:n] / nlp.obj_scale).cpu().numpy()
    return IpmResult(x=xf, lam_g=lam_out, f=float(f.item()) / nlp.obj_scale, status=status, iterations=it,
                     kkt_error=kkt_err, constr_viol=float((c / nlp.c_scale).abs().max().item()) if m else 0.0,
                     seconds=time.perf_counter() - t_start, zl=zl_v, zu=zu_v, log=log,
                     kkt_solves=skkt.n_solve if skkt is not None else 0,
                     kkt_dense=skkt.n_dense if skkt is not None else 0, timing=timing)
