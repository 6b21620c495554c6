"""Hessian of the Lagrangian by coloured central differences of the exact GPU gradient.

For evaluators without a second-order kernel (the dual-kite NLP of config 3/4) the interior-point
solver still needs ``nlp_hess_l`` (awebox's default is the exact Hessian, ``default.py:323``).
The Lagrangian gradient grad f + J^T lambda comes exactly from the HIP evaluator, so its
directional differences give Hessian columns.  Structure of the collocation NLP makes this cheap:

* every g row and objective term of interval k depends only on the interval's own columns
  (x[k], u[k], xdot[k], z[k], coll_var[k]) and the globals (V.theta, phi, xi); x[n_k] enters only
  linear rows;
* so column position p of ALL intervals can share one colour (no row of interval k sees a column
  of another interval), while each global column gets a colour of its own.  Rows of globals are
  taken from the global columns by symmetry.

n_colours = n_globals + interval stride (348 for the dual kites at d=4, 164 for AP2); one Hessian
costs 2 n_colours gradient evaluations, done as ONE batched launch of the evaluator (for B
instances at once: B x 2 n_colours), and one fixed-order gather-sum for J^T lambda.  The pattern is dense per interval block (upper triangle).
Truncation error of central differences with h = 1e-5 (1 + |x|) is O(h^2) of the third
derivatives: ~1e-9 relative, checked against the exact AP2 Hessian kernel on the GPU
(tests/test_fd_hessian.py).
"""
from __future__ import annotations

import numpy as np


class FdHessian:
    """Adds ``sparsity_hess`` / ``nnz_h`` / ``eval_hess_device`` to an evaluator ``ev`` (any batch).

    ``make_batched(B)`` must return an evaluator of the same NLP for B instances; ``layout``
    provides ``n_k``, ``interval_stride``, ``v_intervals``, ``n_v``.
    """

    def __init__(self, ev, make_batched, layout, device="cuda", rel_step=1e-5, tail=False):
        """``tail``: the columns after the last interval (x[n_k]) get the colours of the first
        interval positions and a dense block of their own -- for an objective that is nonlinear
        in x[n_k] (the MPC's terminal cost, pmpc.py:356-358); such columns may enter g only
        linearly (the continuity rows).  Without it they have no Hessian entries."""
        import torch
        self.ev = ev
        self.layout = layout
        self.dev = device
        self.rel_step = rel_step
        lay = layout
        n_v, v0, stride, n_k = lay.n_v, lay.v_intervals, lay.interval_stride, lay.n_k
        self.n_glob = v0
        self.n_col = v0 + stride
        # colour of every column, and its "row block" (interval of a non-global column)
        colour = np.full(n_v, -1, dtype=np.int64)
        colour[:v0] = np.arange(v0)
        own = np.arange(v0, v0 + n_k * stride)
        colour[own] = v0 + (own - v0) % stride
        n_tail = n_v - v0 - n_k * stride if tail else 0
        if n_tail > stride:
            raise ValueError("tail longer than an interval")
        tail_cols = np.arange(v0 + n_k * stride, v0 + n_k * stride + n_tail)
        colour[tail_cols] = v0 + (tail_cols - v0 - n_k * stride)
        self.n_blocks = n_k + (1 if n_tail else 0)
        self.colour = colour
        # upper-triangular pattern: globals x everything below, interval blocks dense
        cols, rows = [], []
        for c in range(v0):
            cols.append(np.full(c + 1, c))
            rows.append(np.arange(c + 1))
        for k in range(self.n_blocks):
            b = v0 + k * stride
            for p in range(stride if k < n_k else n_tail):
                c = b + p
                cols.append(np.full(v0 + p + 1, c))
                rows.append(np.concatenate([np.arange(v0), np.arange(b, c + 1)]))
        col = np.concatenate(cols)
        row = np.concatenate(rows)
        order = np.lexsort((row, col))
        col, row = col[order], row[order]
        self.hcolind = np.zeros(n_v + 1, dtype=np.int32)
        np.add.at(self.hcolind, col + 1, 1)
        self.hcolind = np.cumsum(self.hcolind).astype(np.int32)
        self.hrow = row.astype(np.int32)
        self.nnz_h = len(row)
        # value sources: (colour, row) of the difference matrix for each entry, averaged with the
        # symmetric (colour of row, col) where both columns are interval-own
        glob_c = col < v0
        glob_r = (row < v0) & ~glob_c
        t = torch
        self.src_a_col = t.tensor(np.where(glob_r, colour[row], colour[col]), device=device)
        self.src_a_row = t.tensor(np.where(glob_r, col, row), device=device)
        both = ~glob_c & ~glob_r
        self.both = t.tensor(both, device=device)
        self.src_b_col = t.tensor(np.where(both, colour[row], 0), device=device)
        self.src_b_row = t.tensor(np.where(both, col, 0), device=device)
        # J^T lambda: a fixed-order gather-sum of the entries' products into their columns
        colind, jrow = ev.sparsity_jac()
        self.jrow = t.tensor(jrow.astype(np.int64), device=device)
        from .ipm import _ScatterSum
        self.jt_sum = _ScatterSum(np.repeat(np.arange(n_v), np.diff(colind)), device)
        self.make_batched = make_batched
        self.evb, self.nb_inst = None, 0
        self.colour_t = t.tensor(colour, device=device)
        f64 = dict(dtype=t.float64, device=device)
        mask = np.zeros((self.n_col, n_v))
        valid = colour >= 0
        mask[colour[valid], np.where(valid)[0]] = 1.0
        self.mask = t.tensor(mask, **f64)              # [n_col, n_v] direction of each colour

    def _buffers(self, B):
        """A batched evaluator of B x 2 n_col perturbed instances (built on first use per B)."""
        import torch as t
        if self.nb_inst != B:
            nb = 2 * self.n_col * B
            f64 = dict(dtype=t.float64, device=self.dev)
            self.evb = None
            self.evb = self.make_batched(nb)
            ev, n_v = self.ev, self.layout.n_v
            self.Vb = t.zeros(nb, n_v, **f64)
            self.Pb = t.zeros(nb, ev.n_p, **f64)
            self.fb = t.zeros(nb, **f64)
            self.gb = t.zeros(nb, ev.n_g, **f64)
            self.gradb = t.zeros(nb, n_v, **f64)
            self.jacb = t.zeros(nb, ev.nnz, **f64)
            self.nb_inst = B

    # ---- evaluator surface used by the solver --------------------------------------------
    def __getattr__(self, name):
        return getattr(self.ev, name)

    def sparsity_hess(self):
        return self.hcolind.copy(), self.hrow.copy()

    def eval_hess_device(self, V, P, sigma, lam_g, H, stream=None):
        """Upper-triangular CCS values of sigma f + lam_g^T g at V for every instance: V [B, n_v],
        P [B, n_p], sigma [B], lam_g [B, n_g], H [B, nnz_h]; one batched launch of B x 2 n_col
        perturbed evaluations."""
        import torch
        x = V.reshape(-1, self.layout.n_v)
        B, nc = x.shape[0], self.n_col
        self._buffers(B)
        h = self.rel_step * (1.0 + x.abs())                           # [B, n_v]
        dirs = self.mask[None, :, :] * h[:, None, :]                 # [B, n_col, n_v]
        Vb = self.Vb.view(B, 2, nc, -1)
        Vb[:, 0] = x[:, None, :] + dirs
        Vb[:, 1] = x[:, None, :] - dirs
        self.Pb.view(B, 2 * nc, -1)[:] = P.reshape(B, 1, -1)
        self.evb.eval_nlp_device(self.Vb, self.Pb, self.fb, self.gb, self.gradb, self.jacb, stream=stream)
        lam = lam_g.reshape(B, -1)
        prod = self.jacb.view(B, 2 * nc, -1) * lam[:, self.jrow][:, None, :]      # [B, 2 n_col, nnz]
        jtl = self.jt_sum.add_into(torch.zeros(B, 2 * nc, x.shape[1], dtype=torch.float64, device=x.device), prod)
        gl = sigma.reshape(B, 1, 1) * self.gradb.view(B, 2 * nc, -1) + jtl
        step = 2.0 * h                                               # [B, n_v]
        D = gl[:, :nc] - gl[:, nc:]                                  # [B, n_col, n_v]
        # divide each colour row by the step of the column it perturbs for that entry
        va = D[:, self.src_a_col, self.src_a_row]
        ca = torch.where(self.src_a_col < self.n_glob, self.src_a_col, self._col_of(self.src_a_col, self.src_a_row))
        va = va / step[:, ca]
        vb = D[:, self.src_b_col, self.src_b_row]
        cb = self._col_of(self.src_b_col, self.src_b_row)
        vb = vb / step[:, cb]
        H.reshape(B, -1)[:] = torch.where(self.both, 0.5 * (va + vb), va)

    def _col_of(self, colour, row):
        """The column of `colour` perturbed in the row block of `row` (interval-own columns)."""
        lay = self.layout
        v0, stride = lay.v_intervals, lay.interval_stride
        k = ((row - v0).clamp(min=0) // stride).clamp(max=self.n_blocks - 1)
        return v0 + k * stride + (colour - v0).clamp(min=0)
