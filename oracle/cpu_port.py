"""ctypes binding of the CPU port (oracle/cpu/libap2cpu.so) -- TEST AND BASELINE INFRASTRUCTURE.

The CPU port runs the evaluator's algorithm (shared node model and tables, vector-dual forward
mode, OpenMP over (instance, interval)) on the host.  bench.py times it as the CPU baseline
(kind "port"); tests compare it with the independent oracle (ap2_oracle.py) so that the
colouring / gather-list / objective logic is exercised without a GPU.  Never used by the product.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "cpu", "libap2cpu.so")
_LIB = None


def load():
    global _LIB
    if _LIB is None:
        from oracle.cpu.build import build
        build()
        lib = ctypes.CDLL(_LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        vp = ctypes.c_void_p
        lib.ap2cpu_create.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ctypes.POINTER(vp)]
        lib.ap2cpu_sizes.argtypes = [vp, ip, ip, ip, ip]
        lib.ap2cpu_sparsity.argtypes = [vp, ip, ip]
        lib.ap2cpu_eval_nlp.argtypes = [vp, ctypes.c_int, dp, dp, dp, dp, dp, dp, ctypes.c_int]
        lib.ap2cpu_destroy.argtypes = [vp]
        lib.ap2cpu_hess_init.argtypes = [vp, ip]
        lib.ap2cpu_hess_sparsity.argtypes = [vp, ip, ip]
        lib.ap2cpu_eval_hess.argtypes = [vp, ctypes.c_int, dp, dp, dp, dp, dp, ctypes.c_int]
        lib.ap2cpu_node.argtypes = [vp, dp, dp, ctypes.c_double, dp, dp]
        lib.ap2cpu_last_error.restype = ctypes.c_char_p
        _LIB = lib
    return _LIB


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class CpuPort:
    def __init__(self, consts):
        self.lib = load()
        cfg = consts.cfg
        c = np.ascontiguousarray(consts.consts, dtype=np.float64)
        h = ctypes.c_void_p()
        if self.lib.ap2cpu_create(cfg.n_k, cfg.d, _dp(c), c.size, ctypes.byref(h)) != 0:
            raise RuntimeError(self.lib.ap2cpu_last_error().decode())
        self.h = h
        n = [ctypes.c_int() for _ in range(4)]
        self.lib.ap2cpu_sizes(h, *(ctypes.byref(x) for x in n))
        self.n_v, self.n_g, self.n_p, self.nnz = (x.value for x in n)
        self.colind = np.zeros(self.n_v + 1, dtype=np.int32)
        self.row = np.zeros(self.nnz, dtype=np.int32)
        ip = ctypes.POINTER(ctypes.c_int)
        self.lib.ap2cpu_sparsity(h, self.colind.ctypes.data_as(ip), self.row.ctypes.data_as(ip))

    def eval_nlp(self, V, P, threads=0):
        V = np.ascontiguousarray(np.atleast_2d(V), dtype=np.float64)
        P = np.ascontiguousarray(np.atleast_2d(P), dtype=np.float64)
        B = V.shape[0]
        f = np.zeros(B)
        g = np.zeros((B, self.n_g))
        grad = np.zeros((B, self.n_v))
        jac = np.zeros((B, self.nnz))
        self.lib.ap2cpu_eval_nlp(self.h, B, _dp(V), _dp(P), _dp(f), _dp(g), _dp(grad), _dp(jac), int(threads))
        return {"f": f, "g": g, "grad_f": grad, "jac": jac}

    def node(self, w_sc, theta0, gamma=1.0):
        """Rows [36] (24 eq, 9 ineq, power, beta, pad) of the shared node model at the scaled node
        vector w_sc [59] and their Jacobian [36, 59]."""
        w = np.ascontiguousarray(w_sc, dtype=np.float64)
        th = np.ascontiguousarray(theta0, dtype=np.float64)
        rows = np.zeros(36)
        jac = np.zeros((36, w.size))
        self.lib.ap2cpu_node(self.h, _dp(w), _dp(th), float(gamma), _dp(rows), _dp(jac))
        return rows, jac

    def hess_init(self):
        if getattr(self, "hnnz", None) is None:
            n = ctypes.c_int()
            if self.lib.ap2cpu_hess_init(self.h, ctypes.byref(n)) != 0:
                raise RuntimeError(self.lib.ap2cpu_last_error().decode())
            self.hnnz = n.value
            self.hcolind = np.zeros(self.n_v + 1, dtype=np.int32)
            self.hrow = np.zeros(self.hnnz, dtype=np.int32)
            ip = ctypes.POINTER(ctypes.c_int)
            self.lib.ap2cpu_hess_sparsity(self.h, self.hcolind.ctypes.data_as(ip), self.hrow.ctypes.data_as(ip))

    def eval_hess(self, V, P, sigma, lam, threads=0):
        """Upper-triangular CCS values of the Hessian of sigma f + lam^T g, [B, nnz_h]."""
        self.hess_init()
        V = np.ascontiguousarray(np.atleast_2d(V), dtype=np.float64)
        P = np.ascontiguousarray(np.atleast_2d(P), dtype=np.float64)
        lam = np.ascontiguousarray(np.atleast_2d(lam), dtype=np.float64)
        B = V.shape[0]
        sig = np.ascontiguousarray(np.broadcast_to(np.asarray(sigma, dtype=np.float64), (B,)))
        H = np.zeros((B, self.hnnz))
        rc = self.lib.ap2cpu_eval_hess(self.h, B, _dp(V), _dp(P), _dp(sig), _dp(lam), _dp(H), int(threads))
        if rc != 0:
            raise RuntimeError(self.lib.ap2cpu_last_error().decode())
        return H

    def hess_csc(self, values):
        """Full symmetric scipy matrix from upper-triangular values."""
        import scipy.sparse as sp
        U = sp.csc_matrix((np.asarray(values), self.hrow, self.hcolind), shape=(self.n_v, self.n_v))
        return (U + sp.triu(U, 1).T).tocsc()

    def jac_csc(self, values):
        import scipy.sparse as sp
        return sp.csc_matrix((np.asarray(values), self.row, self.colind), shape=(self.n_g, self.n_v))

    def __del__(self):
        try:
            self.lib.ap2cpu_destroy(self.h)
        except Exception:
            pass
