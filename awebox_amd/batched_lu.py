"""ctypes binding of ``libawelu.so``: batched in-place LU with partial pivoting of mid-sized fp64
matrices (the interval blocks of ipm.StructuredKKT), in torch.linalg.lu_factor's convention so
that torch.linalg.lu_solve consumes the result."""
from __future__ import annotations

import ctypes
import os

_LIB = None
_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libawelu.so")
MAX_N = 1024
BTD_MAX_M = 48                  # block size limit of the block-tridiagonal kernels (LDS)


def load_library(path: str = _PATH):
    global _LIB
    if _LIB is None:
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not built; run `python -m awebox_amd.build`")
        lib = ctypes.CDLL(path)
        lib.awelu_factor_batched.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p]
        lib.awelu_solve_batched.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p]
        lib.awelu_btd_factor_batched.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
        lib.awelu_btd_solve_batched.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 4
        lib.awelu_sym_inertia_batched.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_double,
                                                  ctypes.c_void_p, ctypes.c_void_p]
        lib.awelu_gather_sum.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_longlong] + \
            [ctypes.c_void_p] * 2 + [ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
        ll, vp = ctypes.c_longlong, ctypes.c_void_p
        lib.awelu_row_sum.argtypes = [ll, ll, vp, ll, vp, vp]
        lib.awelu_bmm.argtypes = [ctypes.c_int] * 4 + [vp, ll, ll, ll] * 3 + [vp]
        lib.awelu_gather_sum_wide.argtypes = [ctypes.c_int] * 2 + [vp] * 5 + [ll] + [vp] * 2 + [ll, vp, ll, vp]
        lib.awelu_last_error.restype = ctypes.c_char_p
        _LIB = lib
    return _LIB


def lu_factor(A):
    """(LU, pivots) of a contiguous float64 CUDA tensor [batch, n, n] (or [n, n]); A is copied."""
    import torch
    if A.dtype != torch.float64 or not A.is_cuda:
        raise ValueError("lu_factor needs a float64 CUDA tensor")
    squeeze = A.dim() == 2
    LU = (A.unsqueeze(0) if squeeze else A).contiguous().clone()
    b, n, n2 = LU.shape
    if n != n2 or n > MAX_N:
        raise ValueError(f"square blocks with n <= {MAX_N} expected, got {tuple(LU.shape)}")
    piv = torch.empty(b, n, dtype=torch.int32, device=LU.device)
    lib = load_library()
    s = torch.cuda.current_stream(LU.device).cuda_stream
    rc = lib.awelu_factor_batched(n, b, ctypes.c_void_p(LU.data_ptr()), ctypes.c_void_p(piv.data_ptr()),
                                  ctypes.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"awelu_factor_batched: {lib.awelu_last_error().decode()}")
    return (LU[0], piv[0]) if squeeze else (LU, piv)


def lu_solve(LU, piv, B):
    """A^-1 B from lu_factor's (LU, piv): LU [batch, n, n], piv int32 [batch, n], B [batch, n, nrhs]
    float64 CUDA tensors (also unbatched [n, n], [n], [n, nrhs]); returns a new tensor."""
    import torch
    if LU.dtype != torch.float64 or B.dtype != torch.float64 or piv.dtype != torch.int32 or not LU.is_cuda:
        raise ValueError("lu_solve needs float64 CUDA factors / right-hand sides and int32 pivots")
    squeeze = LU.dim() == 2
    LU3 = (LU.unsqueeze(0) if squeeze else LU).contiguous()
    piv2 = (piv.unsqueeze(0) if squeeze else piv).contiguous()
    X = (B.unsqueeze(0) if squeeze else B).contiguous().clone()
    b, n, _ = LU3.shape
    if X.dim() != 3 or X.shape[0] != b or X.shape[1] != n or piv2.shape != (b, n):
        raise ValueError(f"shape mismatch: LU {tuple(LU3.shape)}, piv {tuple(piv2.shape)}, B {tuple(X.shape)}")
    lib = load_library()
    s = torch.cuda.current_stream(LU3.device).cuda_stream
    rc = lib.awelu_solve_batched(n, X.shape[2], b, ctypes.c_void_p(LU3.data_ptr()), ctypes.c_void_p(piv2.data_ptr()),
                                 ctypes.c_void_p(X.data_ptr()), ctypes.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"awelu_solve_batched: {lib.awelu_last_error().decode()}")
    return X[0] if squeeze else X


def btd_factor(T):
    """Factor block-tridiagonal systems T [batch, nb, 3, m, m] (sub-, main, super-diagonal block of
    every block row; float64 CUDA, m <= 48).  Returns (F, Dinv): F = T with W_k in the super-diagonal
    slots, Dinv [batch, nb, m, m] the inverted pivot blocks; T is not modified."""
    import torch
    if T.dtype != torch.float64 or not T.is_cuda or T.dim() != 5 or T.shape[2] != 3 or T.shape[3] != T.shape[4]:
        raise ValueError(f"btd_factor needs a float64 CUDA tensor [batch, nb, 3, m, m], got {tuple(T.shape)}")
    b, nb, _, m, _ = T.shape
    F = T.contiguous().clone()
    Dinv = torch.empty(b, nb, m, m, dtype=torch.float64, device=T.device)
    lib = load_library()
    s = torch.cuda.current_stream(T.device).cuda_stream
    rc = lib.awelu_btd_factor_batched(nb, m, b, ctypes.c_void_p(F.data_ptr()), ctypes.c_void_p(Dinv.data_ptr()),
                                      ctypes.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"awelu_btd_factor_batched: {lib.awelu_last_error().decode()}")
    return F, Dinv


def btd_solve(F, Dinv, X):
    """T^-1 X with btd_factor's (F, Dinv); X [batch, nb, m, nrhs] float64 CUDA.  Returns a new tensor."""
    import torch
    b, nb, _, m, _ = F.shape
    if X.dtype != torch.float64 or not X.is_cuda or X.dim() != 4 or X.shape[:3] != (b, nb, m):
        raise ValueError(f"shape mismatch: F {tuple(F.shape)}, X {tuple(X.shape)}")
    Xw = X.contiguous().clone()
    lib = load_library()
    s = torch.cuda.current_stream(F.device).cuda_stream
    rc = lib.awelu_btd_solve_batched(nb, m, X.shape[3], b, ctypes.c_void_p(F.data_ptr()),
                                     ctypes.c_void_p(Dinv.data_ptr()), ctypes.c_void_p(Xw.data_ptr()),
                                     ctypes.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"awelu_btd_solve_batched: {lib.awelu_last_error().decode()}")
    return Xw


def btd_dense(T):
    """The dense matrices [batch, nb m, nb m] of block-tridiagonal T [batch, nb, 3, m, m]."""
    import torch
    b, nb, _, m, _ = T.shape
    A = torch.zeros(b, nb * m, nb * m, dtype=T.dtype, device=T.device)
    for k in range(nb):
        for s_, dk in ((0, -1), (1, 0), (2, 1)):
            if 0 <= k + dk < nb:
                A[:, k * m:(k + 1) * m, (k + dk) * m:(k + dk + 1) * m] = T[:, k, s_]
    return A


def gather_sum(lsrc, lw, ldst, vals, out, rows, x=None, cols=None):
    """out[r][ldst] += the lane lists' sums of vals[r][lsrc] (times x[r][cols[lsrc]] with x), for
    r < rows: ipm._ScatterSum's fixed-order sums in one launch (awelu_gather_sum).  All device
    tensors: lsrc / ldst int32, lw uint8 (one entry per lane), vals / out / x float64 contiguous
    with ``rows`` leading rows, cols int32."""
    import torch
    L = lsrc.numel()
    if L == 0 or rows == 0:
        return out
    lib = load_library()
    s = torch.cuda.current_stream(out.device).cuda_stream
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
    rc = lib.awelu_gather_sum(L, rows, ptr(lsrc), ptr(lw), ptr(ldst), ptr(vals), vals.shape[-1], ptr(x), ptr(cols),
                              x.shape[-1] if x is not None else 0, ptr(out), out.shape[-1], ctypes.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"awelu_gather_sum: {lib.awelu_last_error().decode()}")
    return out


def gather_sum_wide(wsrc, woff, ww, wdst, vals, out, rows, x=None, cols=None):
    """The wide lists (more than 64 sources) of ipm._ScatterSum's sums in one launch
    (awelu_gather_sum_wide): out[r][wdst[l]] += list l's sum of vals[r][wsrc] (times x[r][cols[wsrc]])
    in det.row_sum's order.  wsrc / woff / ww / wdst int32 device tensors."""
    import torch
    nl = wdst.numel()
    if nl == 0 or rows == 0:
        return out
    lib = load_library()
    s = torch.cuda.current_stream(out.device).cuda_stream
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)  # noqa: E731
    rc = lib.awelu_gather_sum_wide(nl, rows, ptr(wsrc), ptr(woff), ptr(ww), ptr(wdst), ptr(vals), vals.shape[-1],
                                   ptr(x), ptr(cols), x.shape[-1] if x is not None else 0, ptr(out), out.shape[-1],
                                   ctypes.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"awelu_gather_sum_wide: {lib.awelu_last_error().decode()}")
    return out


def sym_inertia(A, ztol=1e-13):
    """(positive, negative, zero) eigenvalue counts [batch, 3] (int32, on the device) of symmetric
    float64 CUDA matrices A [batch, n, n] (lower triangle read; A is not modified)."""
    import torch
    if A.dtype != torch.float64 or not A.is_cuda or A.dim() != 3 or A.shape[1] != A.shape[2]:
        raise ValueError(f"sym_inertia needs a float64 CUDA tensor [batch, n, n], got {tuple(A.shape)}")
    b, n, _ = A.shape
    W = A.contiguous().clone()
    counts = torch.empty(b, 3, dtype=torch.int32, device=A.device)
    lib = load_library()
    s = torch.cuda.current_stream(A.device).cuda_stream
    rc = lib.awelu_sym_inertia_batched(n, b, ctypes.c_void_p(W.data_ptr()), ctypes.c_double(ztol),
                                       ctypes.c_void_p(counts.data_ptr()), ctypes.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"awelu_sym_inertia_batched: {lib.awelu_last_error().decode()}")
    return counts


def sym_inertia_host(A, ztol=1e-13):
    """The same counts from symmetric eigenvalues (host tensors: the CPU test harness)."""
    import torch
    ev = torch.linalg.eigvalsh(0.5 * (A + A.transpose(-1, -2)))
    scale = A.abs().amax(dim=(-1, -2), keepdim=False).clamp(min=1e-300).unsqueeze(-1)
    pos = (ev > ztol * scale).sum(-1)
    neg = (ev < -ztol * scale).sum(-1)
    return torch.stack([pos, neg, ev.shape[-1] - pos - neg], dim=-1).to(torch.int32)
