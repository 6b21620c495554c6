"""ctypes binding of ``libawelu.so``: batched in-place LU with partial pivoting of mid-sized fp64
matrices (the interval blocks of ipm.StructuredKKT), in torch.linalg.lu_factor's convention so
that torch.linalg.lu_solve consumes the result."""
from __future__ import annotations

import ctypes
import os

_LIB = None
_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libawelu.so")
MAX_N = 1024


def load_library(path: str = _PATH):
    global _LIB
    if _LIB is None:
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not built; run `python -m awebox_amd.build`")
        lib = ctypes.CDLL(path)
        lib.awelu_factor_batched.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p]
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
