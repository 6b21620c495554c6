"""Bordered block-tridiagonal separator systems of the structured KKT solve.

After the interval interiors are eliminated (ipm.StructuredKKT, rti.BatchedRti), the separators
are the shooting states x[k], the multipliers c[k] of the continuity rows and a few global
unknowns (free globals such as t_f, the multipliers of the periodicity and global rows).  In
stages [c[k-1], x[k]] the separator matrix is block tridiagonal -- interval k's Schur complement
touches only (x[k], c[k]) and the globals, the continuity row k couples c[k] with x[k+1] -- apart
from the globals, which form a border:
    S = [T  E]      T block tridiagonal (nb = N + 1 blocks of 2 n_x),
        [F  C]      E, F, C the couplings with the n_G border unknowns.
Pairing x[k] with c[k-1] is the Riccati structure of the stage-wise KKT and keeps the sweep's pivot
blocks regular; the finer order x[0], c[0], x[1], ... breaks down at N=40.
Solve:  Z = T^-1 E,  C' = C - F Z,  x_G = C'^-1 (r_G - F T^-1 r_T),  x_T = T^-1 r_T - Z x_G,
with T factorised once per KKT matrix by the awelu block sweep (awelu_btd_factor_batched) and
C' (n_G x n_G) by the awelu LU.  This replaces a dense LU of S (n_S = 1,886 at AP2 N=40,
2,100 for the dual kites at N=20), whose library factorisation is dominated by host-side launch
overhead (~17 ms of CPU time against 1.4 ms of GPU time per factorisation on MI355X,
profiles/r01/ipm_profile_n40_awelu_solve.log).

Host tensors (the CPU test harness) take the same assembly and solve the blocks with dense
LAPACK calls; device tensors use the awelu kernels and fail loudly without them.
"""
from __future__ import annotations

import numpy as np
import torch

from . import det


class BorderedBtd:
    """Separator system with ``stage_of[q]`` (block index, -1 = border) and ``pos_of[q]`` (row
    within the block) for the n_S separators; the matrix entries arrive as value vectors aligned
    with the coordinate lists given at construction (duplicates are summed)."""

    def __init__(self, stage_of, pos_of, nb, m, rows, cols, dev, deterministic=True):
        stage_of, pos_of = np.asarray(stage_of), np.asarray(pos_of)
        rows, cols = np.asarray(rows), np.asarray(cols)
        nS = len(stage_of)
        valid = (rows < nS) & (cols < nS)
        gid = np.full(nS, -1, dtype=np.int64)
        border = np.where(stage_of < 0)[0]
        gid[border] = np.arange(len(border))
        self.nS, self.nb, self.m, self.nG, self.dev = nS, nb, m, len(border), dev
        slot = np.where(stage_of >= 0, stage_of * m + pos_of, -1)
        r_ok, c_ok = np.where(valid, rows, 0), np.where(valid, cols, 0)
        sr, sc = stage_of[r_ok], stage_of[c_ok]
        tt = valid & (sr >= 0) & (sc >= 0)
        if np.any(np.abs(sr[tt] - sc[tt]) > 1):
            raise ValueError("separator couplings are not block tridiagonal in stage order")
        tg = valid & (sr >= 0) & (sc < 0)
        gt = valid & (sr < 0) & (sc >= 0)
        gg = valid & (sr < 0) & (sc < 0)
        n_t = nb * m
        t = lambda a: torch.tensor(a, dtype=torch.int64, device=dev)  # noqa: E731
        self.src_tt, self.dst_tt = t(np.where(tt)[0]), t(((sr[tt] * 3 + 1 + sc[tt] - sr[tt]) * m + pos_of[r_ok[tt]]) * m
                                                           + pos_of[c_ok[tt]])
        self.src_tg, self.dst_tg = t(np.where(tg)[0]), t(slot[r_ok[tg]] * self.nG + gid[c_ok[tg]])
        self.src_gt, self.dst_gt = t(np.where(gt)[0]), t(gid[r_ok[gt]] * n_t + slot[c_ok[gt]])
        self.src_gg, self.dst_gg = t(np.where(gg)[0]), t(gid[r_ok[gg]] * self.nG + gid[c_ok[gg]])
        used = np.zeros((nb, m), dtype=bool)
        used[stage_of[stage_of >= 0], pos_of[stage_of >= 0]] = True
        if used.sum() != (stage_of >= 0).sum():
            raise ValueError("two separators share a block position")
        T0 = np.zeros((nb, 3, m, m))
        a_, i_ = np.where(~used)
        T0[a_, 1, i_, i_] = 1.0                           # unused block positions (fixed variables)
        self.n_unused = len(a_)
        self.T0 = torch.tensor(T0.reshape(-1), dtype=torch.float64, device=dev)
        sep_t = np.where(stage_of >= 0)[0]
        self.sep_t, self.slot_t = t(sep_t), t(slot[sep_t])
        self.sep_g = t(border)
        self.sc = None
        if deterministic:                                  # fixed-order sums of duplicate entries
            from .ipm import scatter_sum
            self.sc = [scatter_sum(d.cpu().numpy(), dev) for d in (self.dst_tt, self.dst_tg, self.dst_gt, self.dst_gg)]

    # ---------------------------------------------------------------------------------------
    def factor(self, vals):
        """vals [n_entries] (or [B, n_entries]): the separator matrix entries."""
        squeeze = vals.dim() == 1
        v = vals.unsqueeze(0) if squeeze else vals
        B, nb, m, nG = v.shape[0], self.nb, self.m, self.nG
        n_t = nb * m
        f64 = dict(dtype=torch.float64, device=self.dev)
        T = self.T0.repeat(B, 1)
        E = torch.zeros(B, n_t * nG, **f64)
        Fm = torch.zeros(B, nG * n_t, **f64)
        C = torch.zeros(B, nG * nG, **f64)
        parts = ((T, self.src_tt, self.dst_tt), (E, self.src_tg, self.dst_tg), (Fm, self.src_gt, self.dst_gt),
                 (C, self.src_gg, self.dst_gg))
        for i, (out, src, dst) in enumerate(parts):
            if self.sc is not None:
                self.sc[i].add_into_sel(out, v, src)
            else:
                out.index_add_(1, dst, v[:, src])
        T = T.view(B, nb, 3, m, m)
        self.B = B
        self.squeeze = squeeze
        from .batched_lu import BTD_MAX_M
        self.fused = T.is_cuda and m <= BTD_MAX_M
        if self.fused:
            from .batched_lu import btd_factor
            self.Tf = btd_factor(T)
        else:
            # the forward sweep of T^-1 E rides along with the block recursion (see _factor_blocks)
            Yf = self._factor_blocks(T, E.view(B, nb, m, nG) if nG else None)
        self.Fm = Fm.view(B, nG, n_t)
        if nG:
            if self.fused:
                self.Z = self._t_solve(E.view(B, n_t, nG))                 # T^-1 E
            else:
                self.Z = self._t_backward(Yf)
            Cp = C.view(B, nG, nG) - det.bmm(self.Fm, self.Z)
            self.Cp = Cp
            self.Cf = self._lu(Cp)

    def inertia(self):
        """[B, 3] (positive, negative, zero) eigenvalue counts of the separator matrix S: the pivot
        blocks D'_k of the block sweep (Bunch-Kaufman on the blocks themselves, not on their
        explicit inverses, whose signs are unreliable when a block is nearly singular) plus the border's
        Schur complement C' (Haynsworth additivity); the identity rows of unused block positions
        are taken out."""
        from .batched_lu import sym_inertia, sym_inertia_host
        from .ipm import ZERO_PIVOT
        B, nb, m = self.B, self.nb, self.m
        f = sym_inertia if self.dev_is_cuda() else sym_inertia_host
        if self.fused:
            F, Dinv = self.Tf                              # F's diagonal slots hold the pivot blocks D'_k
            c = f(F[:, :, 1].reshape(B * nb, m, m), ztol=ZERO_PIVOT).view(B, nb, 3).sum(1)
        else:
            c = f(self.Dp.reshape(B * nb, m, m), ztol=ZERO_PIVOT).view(B, nb, 3).sum(1)
        c = c.to(torch.int64)
        c[:, 0] -= self.n_unused
        if self.nG:
            cc = (sym_inertia if self.Cp.is_cuda else sym_inertia_host)(self.Cp.contiguous(), ztol=ZERO_PIVOT)
            c = c + cc.to(torch.int64)
        return c

    def dev_is_cuda(self):
        return torch.device(self.dev).type == "cuda"

    def _factor_blocks(self, T, X=None):
        """The block sweep by a block recursion over batched dense operations (blocks larger than
        the fused kernels' LDS limit, and host tensors): D'_0 = D_0, W_k = D'_k^-1 U_k,
        D'_k = D_k - L_k W_{k-1}, with an LU (partial pivoting) of every pivot block -- the awelu
        kernels on the device, LAPACK on the host.

        With X [B, nb, m, r] (the border columns E) the forward sweep of T^-1 X runs in the same
        stages, Y_k = D'_k^-1 (X_k - L_k Y_{k-1}): L_k multiplies [W_{k-1} | Y_{k-1}] in one product
        and D'_k^-1 is applied to [U_k | X_k - L_k Y_{k-1}] in one solve, so the sweep costs no
        launches of its own.  Every entry is the same sum as in separate calls (products summed over
        k in sequence, solves column by column), so Y is bitwise _t_solve's forward sweep.  Returns
        the list of Y_k (None without X)."""
        B, nb, m = T.shape[0], self.nb, self.m
        self.T_blocks = T
        Dp, LUs, Ws, Y = [], [], [], []
        D = T[:, 0, 1]
        rk = X[:, 0] if X is not None else None
        for k in range(nb):
            if k > 0:
                if X is None:
                    D = T[:, k, 1] - det.bmm(T[:, k, 0], Ws[k - 1])
                else:
                    P = det.bmm(T[:, k, 0], torch.cat([Ws[k - 1], Y[k - 1]], 2))
                    D = T[:, k, 1] - P[:, :, :m]
                    rk = X[:, k] - P[:, :, m:]
            LU = self._lu(D.contiguous())
            Dp.append(D)
            LUs.append(LU)
            if k < nb - 1:
                if X is None:
                    Ws.append(self._lu_solve(LU, T[:, k, 2].contiguous()))
                else:
                    S = self._lu_solve(LU, torch.cat([T[:, k, 2], rk], 2).contiguous())
                    Ws.append(S[:, :, :m])
                    Y.append(S[:, :, m:])
            elif X is not None:
                Y.append(self._lu_solve(LU, rk.contiguous()))
        self.Dp = torch.stack(Dp, 1)
        self.LUs, self.Ws = LUs, Ws
        return Y if X is not None else None

    def _t_backward(self, Y):
        """The backward sweep of T^-1 X from the forward sweep's Y_k: x_k = Y_k - W_k x_{k+1}."""
        B, nb, m = self.B, self.nb, self.m
        Y = list(Y)
        for k in range(nb - 2, -1, -1):
            Y[k] = Y[k] - det.bmm(self.Ws[k], Y[k + 1])
        return torch.stack(Y, 1).reshape(B, nb * m, -1)

    AWELU_SOLVE = True          # device: the awelu solve kernel (False: rocSOLVER getrs, A/B only)

    def _lu_solve(self, LU, X):
        """D'^-1 X from an LU of the pivot block (LAPACK convention: the awelu factors on the
        device).  On the device the awelu solve kernel: one workgroup per (block, right-hand-side
        chunk), the same operations per entry whatever the batch, so the block recursion rounds the
        same for one instance as inside a batch (rocSOLVER's getrs calls rocBLAS trsm, whose kernel
        choice follows the batch count).  Round 5 measured the library getrs ahead for the dual
        kites' 100 x 100 blocks (the dual homotopy's first 62 iterations 3.8 s against 4.3 s,
        profiles/r05/solver/dual_solve_ab); batch invariance decides.  Host tensors: LAPACK."""
        if X.is_cuda and self.AWELU_SOLVE:
            from .batched_lu import lu_solve
            return lu_solve(LU[0], LU[1], X)
        return torch.linalg.lu_solve(LU[0], LU[1], X)

    def _t_solve(self, X):
        B, nb, m = self.B, self.nb, self.m
        if self.fused:
            from .batched_lu import btd_solve
            F, Dinv = self.Tf
            return btd_solve(F, Dinv, X.reshape(B, nb, m, -1)).view(B, nb * m, -1)
        Xb = X.reshape(B, nb, m, -1)
        T = self.T_blocks
        Y = []
        for k in range(nb):                                # forward: Y_k = D'_k^-1 (X_k - L_k Y_{k-1})
            rk = Xb[:, k] if k == 0 else Xb[:, k] - det.bmm(T[:, k, 0], Y[k - 1])
            Y.append(self._lu_solve(self.LUs[k], rk.contiguous()))
        for k in range(nb - 2, -1, -1):                    # backward: x_k = Y_k - W_k x_{k+1}
            Y[k] = Y[k] - det.bmm(self.Ws[k], Y[k + 1])
        return torch.stack(Y, 1).reshape(B, nb * m, -1)

    @staticmethod
    def _lu(A):
        if A.is_cuda:
            from .batched_lu import lu_factor
            return lu_factor(A)
        return torch.linalg.lu_factor(A)

    def _c_solve(self, X):
        if X.is_cuda:
            from .batched_lu import lu_solve
            return lu_solve(*self.Cf, X)
        return torch.linalg.lu_solve(*self.Cf, X)

    def solve(self, r):
        """r [n_S] (or [B, n_S]) -> S^-1 r."""
        r2 = r.unsqueeze(0) if r.dim() == 1 else r
        B, n_t = r2.shape[0], self.nb * self.m
        rT = torch.zeros(B, n_t, dtype=torch.float64, device=r.device)
        rT[:, self.slot_t] = r2[:, self.sep_t]
        z = self._t_solve(rT.unsqueeze(-1)).squeeze(-1)
        x = torch.empty_like(r2)
        if self.nG:
            rG = r2[:, self.sep_g] - det.bmv(self.Fm, z)
            xG = self._c_solve(rG.unsqueeze(-1)).squeeze(-1)
            z = z - det.bmv(self.Z, xG)
            x[:, self.sep_g] = xG
        x[:, self.sep_t] = z[:, self.slot_t]
        return x[0] if r.dim() == 1 else x
