"""ctypes binding of the dual-kite CPU port (oracle/cpu/libdualcpu.so) -- TEST AND BASELINE
INFRASTRUCTURE (see oracle/cpu/dual_cpu.cpp); never used by the product."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_LIB = None
_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpu", "libdualcpu.so")


def load():
    global _LIB
    if _LIB is None:
        from oracle.cpu.build import build
        build()
        lib = ctypes.CDLL(_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        vp = ctypes.c_void_p
        lib.dualcpu_create.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ctypes.POINTER(vp)]
        lib.dualcpu_sizes.argtypes = [vp, ip, ip, ip, ip]
        lib.dualcpu_sparsity.argtypes = [vp, ip, ip]
        lib.dualcpu_eval_nlp.argtypes = [vp, ctypes.c_int, dp, dp, dp, dp, dp, dp, ctypes.c_int]
        lib.dualcpu_destroy.argtypes = [vp]
        lib.dualcpu_last_error.restype = ctypes.c_char_p
        _LIB = lib
    return _LIB


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class DualCpuPort:
    def __init__(self, consts):
        self.lib = load()
        c = np.ascontiguousarray(consts.consts, dtype=np.float64)
        h = ctypes.c_void_p()
        if self.lib.dualcpu_create(consts.cfg.n_k, consts.cfg.d, _dp(c), c.size, ctypes.byref(h)) != 0:
            raise RuntimeError(self.lib.dualcpu_last_error().decode())
        self.h = h
        s = [ctypes.c_int() for _ in range(4)]
        self.lib.dualcpu_sizes(self.h, *[ctypes.byref(x) for x in s])
        self.n_v, self.n_g, self.n_p, self.nnz = (x.value for x in s)
        self.colind = np.zeros(self.n_v + 1, dtype=np.int32)
        self.row = np.zeros(self.nnz, dtype=np.int32)
        ip = ctypes.POINTER(ctypes.c_int)
        self.lib.dualcpu_sparsity(self.h, self.colind.ctypes.data_as(ip), self.row.ctypes.data_as(ip))

    def __del__(self):
        try:
            self.lib.dualcpu_destroy(self.h)
        except Exception:
            pass

    def eval_nlp(self, V, P, threads=0):
        V = np.ascontiguousarray(np.atleast_2d(V), dtype=np.float64)
        P = np.ascontiguousarray(np.atleast_2d(P), dtype=np.float64)
        B = V.shape[0]
        f = np.zeros(B)
        g = np.zeros((B, self.n_g))
        gr = np.zeros((B, self.n_v))
        jac = np.zeros((B, self.nnz))
        self.lib.dualcpu_eval_nlp(self.h, B, _dp(V), _dp(P), _dp(f), _dp(g), _dp(gr), _dp(jac), int(threads))
        return {"f": f, "g": g, "grad_f": gr, "jac": jac}

    def jac_csc(self, values):
        import scipy.sparse as sp
        return sp.csc_matrix((np.asarray(values), self.row, self.colind), shape=(self.n_g, self.n_v))
