"""Batch-invariant reductions and products of the interior-point solver (DESIGN.md section 9,
"Batch invariance").

The reference solves every sweep point and every homotopy run as its own IPOPT problem
(awebox/sweep.py:148-172 calls opti/optimization.py:363 once per point), so its answer for one
point cannot depend on how many points are solved.  ipm.solve_batch solves B instances side by side;
to keep that property, every operation that mixes the entries of one instance must round the same
whatever B is.  Elementwise torch operations and index gathers already do.  torch's row reductions
(``x.sum(1)``) pick their strategy from the tensor's shape, and rocBLAS picks its GEMM kernel from
the batch count, so their last bits change with B -- enough for the final homotopy step to end on a
different local optimum (profiles/r05/ensemble/batch_homotopy.log: 35.9 s alone, 51.7 s at B = 128).

This module gives each such operation one fixed order that depends only on the length being
reduced:

* ``row_sum(x)``: thread t of 256 adds x[t], x[t + 256], ... in sequence, then the 256 partial sums
  as an adjacent-pair tree (libawelu ``awelu_row_sum``);
* ``tree_sum(x)``: the adjacent-pair tree over a power-of-two last dimension (the order of the
  narrow gather-sum kernel ``awelu_gather_sum``);
* ``bmm(A, B)``: every entry summed over k in sequence, product and sum rounded separately
  (libawelu ``awelu_bmm``).

On the GPU the libawelu kernels run (and fail loudly without the library); on host tensors -- the CPU
test harness -- and wherever ``emulate=True`` is asked for, the same order is restated with
elementwise torch operations, so a GPU kernel can be checked bitwise against its restatement
(tests/test_det_gpu.py) and the CPU harness is batch-invariant by the same construction
(tests/test_det.py)."""
from __future__ import annotations

import ctypes
import math
import os

import torch

ROW_SUM_THREADS = 256
# AWE_DET_OFF=1: torch's own reductions and matmul instead (A/B measurements only: batch-dependent)
_OFF = os.environ.get("AWE_DET_OFF", "0") == "1"


def _lib():
    from .batched_lu import load_library
    return load_library()


def _check(rc, name):
    if rc != 0:
        raise RuntimeError(f"{name}: {_lib().awelu_last_error().decode()}")


# ---- row sums --------------------------------------------------------------------------------------
def row_sum(x: torch.Tensor, emulate: bool = False) -> torch.Tensor:
    """Sum over the last dimension of float64 ``x`` [..., n] in the fixed order of awelu_row_sum."""
    if x.dtype != torch.float64:
        raise ValueError("row_sum needs float64")
    if _OFF and not emulate:
        return x.sum(-1)
    n = x.shape[-1]
    lead = x.shape[:-1]
    R = math.prod(lead)
    if x.is_cuda and not emulate:
        x2 = x.reshape(R, n)
        if n and x2.stride(-1) != 1:
            x2 = x2.contiguous()
        if n == 0:
            return torch.zeros(lead, dtype=torch.float64, device=x.device)
        out = torch.empty(R, dtype=torch.float64, device=x.device)
        if R:
            ldx = x2.stride(0) if R > 1 else max(n, 1)
            s = torch.cuda.current_stream(x.device).cuda_stream
            _check(_lib().awelu_row_sum(R, n, ctypes.c_void_p(x2.data_ptr()), ldx,
                                        ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s)), "awelu_row_sum")
        return out.reshape(lead)
    return _row_sum_ref(x.reshape(R, n)).reshape(lead)


def _row_sum_ref(x2: torch.Tensor) -> torch.Tensor:
    R, n = x2.shape
    T = ROW_SUM_THREADS
    J = -(-n // T)
    acc = torch.zeros(R, T, dtype=torch.float64, device=x2.device)
    if J:
        pad = torch.zeros(R, J * T, dtype=torch.float64, device=x2.device)
        pad[:, :n] = x2
        v = pad.view(R, J, T)
        for j in range(J):
            acc = acc + v[:, j]
    return _tree(acc)


def _tree(acc: torch.Tensor) -> torch.Tensor:
    """Adjacent-pair tree over the power-of-two last dimension: ((a0 + a1) + (a2 + a3)) + .."""
    while acc.shape[-1] > 1:
        acc = acc[..., 0::2] + acc[..., 1::2]
    return acc[..., 0]


def tree_sum(x: torch.Tensor) -> torch.Tensor:
    """Sum over a power-of-two last dimension as an adjacent-pair tree (awelu_gather_sum's order for
    a list of that width)."""
    w = x.shape[-1]
    if w & (w - 1):
        raise ValueError("tree_sum needs a power-of-two last dimension")
    return _tree(x)


# ---- batched products ------------------------------------------------------------------------------
def bmm(A: torch.Tensor, B: torch.Tensor, emulate: bool = False) -> torch.Tensor:
    """A @ B for float64 [batch, M, K] and [batch, K, N] (any strides, e.g. transposed views; a 2-D
    operand pair is one matrix), every entry summed over k in sequence (awelu_bmm).  Returns a new
    contiguous [batch, M, N] (or [M, N]) tensor."""
    if A.dtype != torch.float64 or B.dtype != torch.float64:
        raise ValueError("bmm needs float64")
    if _OFF and not emulate:
        return A @ B
    squeeze = A.dim() == 2
    A3 = A.unsqueeze(0) if squeeze else A
    B3 = B.unsqueeze(0) if squeeze else B
    if A3.dim() != 3 or B3.dim() != 3 or A3.shape[0] != B3.shape[0] or A3.shape[2] != B3.shape[1]:
        raise ValueError(f"bmm shape mismatch: {tuple(A.shape)} @ {tuple(B.shape)}")
    nb, M, K = A3.shape
    N = B3.shape[2]
    if A3.is_cuda and not emulate:
        C = torch.empty(nb, M, N, dtype=torch.float64, device=A.device)
        if nb and M and N:
            s = torch.cuda.current_stream(A.device).cuda_stream
            sa, sb, sc = A3.stride(), B3.stride(), C.stride()
            _check(_lib().awelu_bmm(nb, M, N, K, ctypes.c_void_p(A3.data_ptr()), sa[0], sa[1], sa[2],
                                    ctypes.c_void_p(B3.data_ptr()), sb[0], sb[1], sb[2],
                                    ctypes.c_void_p(C.data_ptr()), sc[0], sc[1], sc[2], ctypes.c_void_p(s)),
                   "awelu_bmm")
        return C[0] if squeeze else C
    C = torch.zeros(nb, M, N, dtype=torch.float64, device=A.device)
    for k in range(K):
        C = C + A3[:, :, k:k + 1] * B3[:, k:k + 1, :]
    return C[0] if squeeze else C


def bmv(A: torch.Tensor, x: torch.Tensor, emulate: bool = False) -> torch.Tensor:
    """A @ x for [batch, M, K] and [batch, K] -> [batch, M] (bmm with one column)."""
    return bmm(A, x.unsqueeze(-1), emulate=emulate).squeeze(-1)
