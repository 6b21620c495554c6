"""Cyclic reduction (CR) of the separator chain vs the sequential Riccati block recursion, on
KKT-like stage chains [c[k-1], x[k]] (continuity coupling +-I, symmetric indefinite state blocks,
random couplings between neighbouring stages).  CR eliminates the odd positions of the chain
level by level (ceil(log2 nb) levels of batched LUs instead of nb dependent ones), but its
intermediate Schur complements of indefinite chains can be nearly singular even when the whole
matrix is well conditioned: at nb = 7, m = 52 (cond 1.3e4) the level-2 pivot block reaches cond
1e8 and the last one 1.9e9, and CR's solution is off by 4e-8 relative, against 6e-12 for the
Riccati order, whose pivot blocks stay below cond 3e5.  The product therefore keeps the Riccati
order (awebox_amd/btd.py); this lab prints the comparison.

    python tools/btd_cr_lab.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from awebox_amd.btd import BorderedBtd  # noqa: E402


class CrBtd(BorderedBtd):
    """BorderedBtd with the block recursion replaced by cyclic reduction (host tensors)."""

    def _factor_blocks(self, T):
        self._factor_cr(T)

    def _t_solve(self, X):
        B, nb, m = self.B, self.nb, self.m
        return self._solve_cr(X.reshape(B, nb, m, -1)).reshape(B, nb * m, -1)

    # ---- cyclic reduction -------------------------------------------------------------------
    def _factor_cr(self, T):
        """Block cyclic reduction of the chain: per level the blocks at odd positions of the
        current chain (never adjacent, so they form a block-diagonal set) are eliminated at once
        -- one batched LU of all of them, one batched solve for D_e^-1 [L_e | U_e] -- and their
        neighbours receive the Schur updates
            D_k -= L_k D_e^-1 U_e + U_k D_f^-1 L_f,   L_k <- -L_k D_e^-1 L_e,   U_k <- -U_k D_f^-1 U_f
        (e = k - 1, f = k + 1 in the current chain), leaving a block-tridiagonal chain of the even
        positions; ceil(log2 nb) levels instead of nb sequential stages.  The pivot blocks of all
        levels and the last remaining block give the inertia (Haynsworth additivity over the
        elimination order).  Used for blocks beyond the fused kernels' LDS limit (the dual kites'
        separators, m = 100), whose sequential block recursion took nb dependent batched LUs and
        library triangular solves per factorisation."""
        B, nb, m = T.shape[0], self.nb, self.m
        L, D, U = T[:, :, 0], T[:, :, 1], T[:, :, 2]
        levels, pivs = [], []
        while D.shape[1] > 1:
            n = D.shape[1]
            eo = torch.arange(1, n, 2, device=D.device)          # eliminated (odd positions)
            ke = torch.arange(0, n, 2, device=D.device)          # kept (even positions)
            ne = len(eo)
            De = D[:, eo].contiguous()
            LUe = self._lu(De.reshape(B * ne, m, m))
            GH = self._lu_solve(LUe, torch.cat([L[:, eo], U[:, eo]], 3).reshape(B * ne, m, 2 * m))
            GH = GH.view(B, ne, m, 2 * m)
            G, H = GH[..., :m], GH[..., m:]                       # D_e^-1 L_e, D_e^-1 U_e
            Dk, Lk, Uk = D[:, ke].clone(), L[:, ke], U[:, ke]
            nk = len(ke)
            # left neighbour of kept block i is eliminated block i - 1, right neighbour block i
            left = torch.arange(nk, device=D.device) - 1          # index into eo, -1 = none
            right = torch.arange(nk, device=D.device)
            hl = left >= 0
            hr = right < ne
            il, ir = torch.where(hl)[0], torch.where(hr)[0]
            Dk[:, il] -= Lk[:, il] @ H[:, left[il]]
            Dk[:, ir] -= Uk[:, ir] @ G[:, right[ir]]
            Ln = torch.zeros_like(Lk)
            Un = torch.zeros_like(Uk)
            Ln[:, il] = -(Lk[:, il] @ G[:, left[il]])
            Un[:, ir] = -(Uk[:, ir] @ H[:, right[ir]])
            levels.append(dict(eo=eo, ke=ke, LUe=LUe, G=G, H=H, Lk=Lk, Uk=Uk, il=il, ir=ir, left=left, right=right))
            pivs.append(De)
            D, L, U = Dk, Ln, Un
        LUf = self._lu(D[:, 0].contiguous())
        pivs.append(D)
        self.cr_levels, self.cr_last = levels, LUf
        self.cr_piv = torch.cat(pivs, 1)                          # [B, nb, m, m]

    def _solve_cr(self, X):
        """T^-1 X [B, nb, m, k] with _factor_cr's levels: the right-hand sides reduced level by level
        (r_k -= L_k D_e^-1 r_e + U_k D_f^-1 r_f), the last block solved, then the eliminated blocks
        recovered in reverse (x_e = D_e^-1 r_e - G_e x_left - H_e x_right)."""
        B, m, k = X.shape[0], self.m, X.shape[3]
        r = X
        ys = []
        for lv in self.cr_levels:
            eo, ke, il, ir = lv["eo"], lv["ke"], lv["il"], lv["ir"]
            ne = len(eo)
            ye = self._lu_solve(lv["LUe"], r[:, eo].reshape(B * ne, m, k).contiguous()).view(B, ne, m, k)
            rk = r[:, ke].clone()
            rk[:, il] -= lv["Lk"][:, il] @ ye[:, lv["left"][il]]
            rk[:, ir] -= lv["Uk"][:, ir] @ ye[:, lv["right"][ir]]
            ys.append(ye)
            r = rk
        x = self._lu_solve(self.cr_last, r[:, 0].contiguous()).unsqueeze(1)
        for lv, ye in zip(reversed(self.cr_levels), reversed(ys)):
            eo, ke = lv["eo"], lv["ke"]
            n = len(eo) + len(ke)
            xe = ye.clone()
            # eliminated block e = 2 i + 1 sits between kept blocks i and i + 1
            i_e = torch.arange(len(eo), device=x.device)
            xe -= lv["G"] @ x[:, i_e]
            has_r = i_e + 1 < len(ke)
            ir_e = torch.where(has_r)[0]
            xe[:, ir_e] -= lv["H"][:, ir_e] @ x[:, ir_e + 1]
            full = torch.empty(B, n, m, k, dtype=x.dtype, device=x.device)
            full[:, ke] = x
            full[:, eo] = xe
            x = full
        return x


def chain(nb, m, B, seed):
    rng = np.random.default_rng(seed)
    h = m // 2
    S = np.zeros((B, nb * m, nb * m))
    for k in range(nb):
        o = k * m
        S[:, o:o + h, o + h:o + m] = np.eye(h)
        S[:, o + h:o + m, o:o + h] = np.eye(h)
        Q = rng.standard_normal((B, h, h))
        S[:, o + h:o + m, o + h:o + m] = Q + Q.transpose(0, 2, 1)
        if k + 1 < nb:
            A = 0.5 * rng.standard_normal((B, m, m))
            S[:, o:o + m, o + m:o + 2 * m] = A
            S[:, o + m:o + 2 * m, o:o + m] = A.transpose(0, 2, 1)
    rows, cols = np.nonzero(np.any(S != 0, axis=0))
    stage_of = np.repeat(np.arange(nb), m)
    pos_of = np.tile(np.arange(m), nb)
    return stage_of, pos_of, rows, cols, S[:, rows, cols], S


def main():
    for nb, m in [(7, 52), (21, 60), (21, 100)]:
        stage_of, pos_of, rows, cols, vals, S = chain(nb, m, 1, nb * 100 + m)
        r = np.random.default_rng(1).standard_normal((1, S.shape[1]))
        x_ref = np.linalg.solve(S, r[..., None])[..., 0]
        out = {"nb": nb, "m": m, "cond": float(np.linalg.cond(S[0]))}
        for name, cls in (("riccati", BorderedBtd), ("cr", CrBtd)):
            bt = cls(stage_of, pos_of, nb, m, rows, cols, "cpu")
            bt.factor(torch.tensor(vals))
            x = bt.solve(torch.tensor(r)).numpy()
            piv = bt.cr_piv if name == "cr" else bt.Dp
            out[name] = {"rel_err": float(np.abs(x - x_ref).max() / np.abs(x_ref).max()),
                         "max_pivot_cond": float(max(np.linalg.cond(piv[0, k].numpy()) for k in range(nb)))}
        print(out)


if __name__ == "__main__":
    main()
