"""Python side of the tracking-MPC boundary: ctypes binding of ``libawempc.so`` (include/awempc.h).

``MpcEvaluator`` exposes the NLP oracle surface the MPC's IPOPT solver reaches through
``ct.nlpsol('solver', 'ipopt', {'x': V, 'p': p, 'f': f, 'g': g})`` in ``awebox/pmpc.py:193-217``
(``nlp_f`` / ``nlp_g`` / ``nlp_grad_f`` / ``nlp_jac_g``, with x = V and p = the MPC parameter struct
``[x0, ref, u_ref, Q, R, P]``), plus the batched device path used for many MPC instances at once.

There is no CPU fallback: a missing library or device raises ``AwegpuUnavailable``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import kite3 as k3
from .evaluator import AWE_ERR_NODEVICE, AWE_OK, AwegpuError, AwegpuUnavailable, _dptr

_LIB = None
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libawempc.so")

EXPORTED_SYMBOLS = ["awempc_create", "awempc_destroy", "awempc_last_error", "awempc_sizes",
                    "awempc_sparsity_jac", "awempc_sparsity_jac_static", "awempc_eval_nlp",
                    "awempc_eval_nlp_host", "awempc_last_kernel_ms", "awempc_hess_init", "awempc_sparsity_hess",
                    "awempc_sparsity_hess_static", "awempc_eval_hess", "awempc_eval_hess_host", "awempc_last_hess_ms",
                    "awempc_gen_status", "awempc_eval_nlp_im", "awempc_last_kernel_ms_im"]


def load_library(path: str = _LIB_PATH):
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise AwegpuUnavailable(f"{path} not built; run `python -m awebox_amd.build`")
    lib = ctypes.CDLL(path)
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int)
    h = ctypes.c_void_p
    lib.awempc_create.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(h)]
    lib.awempc_destroy.argtypes = [h]
    lib.awempc_last_error.restype = ctypes.c_char_p
    lib.awempc_sizes.argtypes = [h, ip, ip, ip, ip]
    lib.awempc_sparsity_jac.argtypes = [h, ip, ip]
    lib.awempc_sparsity_jac_static.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ip, ip, ip]
    lib.awempc_eval_nlp.argtypes = [h] + [ctypes.c_void_p] * 7
    lib.awempc_eval_nlp_host.argtypes = [h, dp, dp, dp, dp, dp, dp]
    lib.awempc_last_kernel_ms.argtypes = [h, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.awempc_hess_init.argtypes = [h, ip]
    lib.awempc_sparsity_hess.argtypes = [h, ip, ip]
    lib.awempc_sparsity_hess_static.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ip, ip, ip]
    lib.awempc_eval_hess.argtypes = [h] + [ctypes.c_void_p] * 6
    lib.awempc_eval_hess_host.argtypes = [h, dp, dp, dp, dp, dp]
    lib.awempc_last_hess_ms.argtypes = [h, ctypes.POINTER(ctypes.c_float)]
    lib.awempc_gen_status.argtypes = [h, ip]
    lib.awempc_eval_nlp_im.argtypes = [h] + [ctypes.c_void_p] * 6 + [ctypes.c_size_t, ctypes.c_void_p]
    lib.awempc_last_kernel_ms_im.argtypes = [h] + [ctypes.POINTER(ctypes.c_float)] * 3
    _LIB = lib
    return lib


def sparsity_jac_static(consts: k3.Kite3Constants):
    """CCS pattern (colind, row) of the MPC J_g, derived on the CPU (no device)."""
    lib = load_library()
    cfg = consts.cfg
    c = np.ascontiguousarray(consts.consts, dtype=np.float64)
    nnz = ctypes.c_int()
    ip = ctypes.POINTER(ctypes.c_int)
    if lib.awempc_sparsity_jac_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz), None, None) != AWE_OK:
        raise AwegpuError(lib.awempc_last_error().decode())
    lay = k3.MpcLayout(cfg.n_k, cfg.d)
    colind = np.zeros(lay.n_v + 1, dtype=np.int32)
    row = np.zeros(nnz.value, dtype=np.int32)
    if lib.awempc_sparsity_jac_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz),
                                      colind.ctypes.data_as(ip), row.ctypes.data_as(ip)) != AWE_OK:
        raise AwegpuError(lib.awempc_last_error().decode())
    return colind, row


def sparsity_hess_static(consts: k3.Kite3Constants):
    """Upper-triangular CCS pattern (colind, row) of the MPC nlp_hess_l, derived on the CPU."""
    lib = load_library()
    cfg = consts.cfg
    c = np.ascontiguousarray(consts.consts, dtype=np.float64)
    nnz = ctypes.c_int()
    ip = ctypes.POINTER(ctypes.c_int)
    if lib.awempc_sparsity_hess_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz), None, None) != AWE_OK:
        raise AwegpuError(lib.awempc_last_error().decode())
    lay = k3.MpcLayout(cfg.n_k, cfg.d)
    colind = np.zeros(lay.n_v + 1, dtype=np.int32)
    row = np.zeros(nnz.value, dtype=np.int32)
    if lib.awempc_sparsity_hess_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz),
                                       colind.ctypes.data_as(ip), row.ctypes.data_as(ip)) != AWE_OK:
        raise AwegpuError(lib.awempc_last_error().decode())
    return colind, row


class MpcEvaluator:
    """HIP evaluator of the 3-DOF tracking-MPC NLP for ``batch`` (V, p) instances."""

    def __init__(self, consts: k3.Kite3Constants | None = None, batch: int = 1):
        self.consts = consts or k3.build_constants()
        cfg = self.consts.cfg
        self.layout = k3.MpcLayout(cfg.n_k, cfg.d)
        self.batch = int(batch)
        self._lib = load_library()
        c = np.ascontiguousarray(self.consts.consts, dtype=np.float64)
        handle = ctypes.c_void_p()
        self._check(self._lib.awempc_create(cfg.n_k, cfg.d, _dptr(c), c.size, self.batch, ctypes.byref(handle)))
        self._h = handle
        n_v, n_g, n_p, nnz = (ctypes.c_int() for _ in range(4))
        self._check(self._lib.awempc_sizes(self._h, ctypes.byref(n_v), ctypes.byref(n_g), ctypes.byref(n_p),
                                           ctypes.byref(nnz)))
        self.n_v, self.n_g, self.n_p, self.nnz = n_v.value, n_g.value, n_p.value, nnz.value
        assert (self.n_v, self.n_g, self.n_p) == (self.layout.n_v, self.layout.n_g, self.layout.n_p)
        self._colind = np.zeros(self.n_v + 1, dtype=np.int32)
        self._row = np.zeros(self.nnz, dtype=np.int32)
        ip = ctypes.POINTER(ctypes.c_int)
        self._check(self._lib.awempc_sparsity_jac(self._h, self._colind.ctypes.data_as(ip),
                                                  self._row.ctypes.data_as(ip)))

    def _check(self, rc):
        if rc != AWE_OK:
            msg = self._lib.awempc_last_error().decode()
            if rc == AWE_ERR_NODEVICE:
                raise AwegpuUnavailable(msg)
            raise AwegpuError(f"awempc error {rc}: {msg}")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.awempc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sparsity_jac(self):
        return self._colind.copy(), self._row.copy()

    def jac_csc(self, values):
        import scipy.sparse as sp
        return sp.csc_matrix((np.asarray(values), self._row, self._colind), shape=(self.n_g, self.n_v))

    # ---------------------------------------------- device path ------------------------
    @property
    def generated_available(self) -> bool:
        """Whether the generated instance-minor path (awempc_eval_nlp_im) serves these constants."""
        ok = ctypes.c_int()
        self._check(self._lib.awempc_gen_status(self._h, ctypes.byref(ok)))
        return bool(ok.value)

    def eval_nlp_device(self, V, p, f, g, grad_f, jac, stream=None):
        """f, g, grad f, J_g for all instances; float64 CUDA tensors V [B, n_v], p [B, n_p], f [B],
        g [B, n_g] (contiguous) and grad_f [B, n_v], jac [B, nnz]: both contiguous (awempc_eval_nlp,
        the dual-number kernel), or both instance-minor views ``x_t.t()`` of contiguous [n, ld] tensors
        with one ld >= B (awempc_eval_nlp_im, the generated node code; ``alloc_grad`` / ``alloc_jac``)."""
        import torch
        for t, n in ((V, self.n_v), (p, self.n_p), (f, 1), (g, self.n_g)):
            if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous() or t.numel() != self.batch * n:
                raise ValueError("device tensors must be contiguous float64 CUDA tensors of the batch shape")
        for t, n in ((grad_f, self.n_v), (jac, self.nnz)):
            if t.dtype != torch.float64 or not t.is_cuda or tuple(t.shape) != (self.batch, n):
                raise ValueError("grad_f and jac must be float64 CUDA tensors [batch, n]")
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        im = lambda t: t.stride(0) == 1 and t.stride(1) >= self.batch   # noqa: E731
        if self.batch == 1 or (jac.is_contiguous() and grad_f.is_contiguous()):
            self._check(self._lib.awempc_eval_nlp(self._h, V.data_ptr(), p.data_ptr(), f.data_ptr(), g.data_ptr(),
                                                  grad_f.data_ptr(), jac.data_ptr(), ctypes.c_void_p(s)))
        elif im(jac) and im(grad_f) and jac.stride(1) == grad_f.stride(1):
            self._check(self._lib.awempc_eval_nlp_im(self._h, V.data_ptr(), p.data_ptr(), f.data_ptr(), g.data_ptr(),
                                                     grad_f.data_ptr(), jac.data_ptr(), int(jac.stride(1)),
                                                     ctypes.c_void_p(s)))
        else:
            raise ValueError("jac and grad_f must both be contiguous or both instance-minor views "
                             "(strides (1, ld), one ld)")

    def alloc_jac(self, device="cuda", instance_minor=None):
        """A J_g value tensor [B, nnz]: instance-minor (the transposed view of [nnz, B], written by the
        generated path with coalesced stores) when the generated path serves this handle and B > 1,
        unless asked otherwise."""
        import torch
        if instance_minor is None:
            instance_minor = self.batch > 1 and self.generated_available
        if instance_minor:
            return torch.zeros(self.nnz, self.batch, dtype=torch.float64, device=device).t()
        return torch.zeros(self.batch, self.nnz, dtype=torch.float64, device=device)

    def alloc_grad(self, device="cuda", instance_minor=None):
        """A grad f tensor [B, n_v] in the layout of ``alloc_jac``."""
        import torch
        if instance_minor is None:
            instance_minor = self.batch > 1 and self.generated_available
        if instance_minor:
            return torch.zeros(self.n_v, self.batch, dtype=torch.float64, device=device).t()
        return torch.zeros(self.batch, self.n_v, dtype=torch.float64, device=device)

    def last_kernel_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        self._check(self._lib.awempc_last_kernel_ms(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def last_kernel_ms_im(self):
        """(input transposition, node kernels, finalize) of the last instance-minor evaluation, ms."""
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        self._check(self._lib.awempc_last_kernel_ms_im(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    # ---------------------------------------------- nlp_hess_l ---------------------------
    @property
    def nnz_h(self):
        if getattr(self, "_hcolind", None) is None:
            n = ctypes.c_int()
            self._check(self._lib.awempc_hess_init(self._h, ctypes.byref(n)))
            self._hcolind = np.zeros(self.n_v + 1, dtype=np.int32)
            self._hrow = np.zeros(n.value, dtype=np.int32)
            ip = ctypes.POINTER(ctypes.c_int)
            self._check(self._lib.awempc_sparsity_hess(self._h, self._hcolind.ctypes.data_as(ip),
                                                       self._hrow.ctypes.data_as(ip)))
        return len(self._hrow)

    def sparsity_hess(self):
        """Upper-triangular CCS pattern of nlp_hess_l: (colind[n_v+1], row[nnz_h])."""
        _ = self.nnz_h
        return self._hcolind.copy(), self._hrow.copy()

    def hess_csc(self, values, full=True):
        import scipy.sparse as sp
        _ = self.nnz_h
        U = sp.csc_matrix((np.asarray(values), self._hrow, self._hcolind), shape=(self.n_v, self.n_v))
        return (U + sp.triu(U, 1).T).tocsc() if full else U

    def eval_hess_device(self, V, p, sigma, lam_g, H, stream=None):
        """Upper-triangular values of the Hessian of sigma f + lam^T g for all instances; contiguous
        float64 CUDA tensors [B, n_v], [B, n_p], [B], [B, n_g], [B, nnz_h]."""
        import torch
        nh = self.nnz_h
        for t, n in ((V, self.n_v), (p, self.n_p), (sigma, 1), (lam_g, self.n_g), (H, nh)):
            if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous() or t.numel() != self.batch * n:
                raise ValueError("device tensors must be contiguous float64 CUDA tensors of the batch shape")
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._check(self._lib.awempc_eval_hess(self._h, V.data_ptr(), p.data_ptr(), sigma.data_ptr(),
                                               lam_g.data_ptr(), H.data_ptr(), ctypes.c_void_p(s)))

    def eval_hess(self, V, p, sigma, lam_g):
        """Host arrays in, host array out: H [B, nnz_h] (upper triangle, CCS)."""
        nh = self.nnz_h
        V = np.ascontiguousarray(np.asarray(V, dtype=np.float64).reshape(self.batch, self.n_v))
        p = np.ascontiguousarray(np.asarray(p, dtype=np.float64).reshape(self.batch, self.n_p))
        sig = np.ascontiguousarray(np.broadcast_to(np.asarray(sigma, dtype=np.float64), (self.batch,)))
        lam = np.ascontiguousarray(np.asarray(lam_g, dtype=np.float64).reshape(self.batch, self.n_g))
        H = np.zeros((self.batch, nh))
        self._check(self._lib.awempc_eval_hess_host(self._h, _dptr(V), _dptr(p), _dptr(sig), _dptr(lam), _dptr(H)))
        return H

    def nlp_hess_l(self, x, p, lam_f, lam_g):
        """CasADi nlp_hess_l: Hessian of lam_f f + lam_g^T g (upper triangle, CCS values)."""
        if self.batch != 1:
            raise ValueError("the oracle-named entry points evaluate one instance (batch=1)")
        return self.eval_hess(np.asarray(x).reshape(1, -1), np.asarray(p).reshape(1, -1), lam_f,
                              np.asarray(lam_g).reshape(1, -1))[0]

    def last_hess_ms(self):
        a = ctypes.c_float()
        self._check(self._lib.awempc_last_hess_ms(self._h, ctypes.byref(a)))
        return a.value

    # ---------------------------------------------- host path --------------------------
    def eval_nlp(self, V, p):
        V = np.ascontiguousarray(np.asarray(V, dtype=np.float64).reshape(self.batch, self.n_v))
        p = np.ascontiguousarray(np.asarray(p, dtype=np.float64).reshape(self.batch, self.n_p))
        f = np.zeros(self.batch)
        g = np.zeros((self.batch, self.n_g))
        grad = np.zeros((self.batch, self.n_v))
        jac = np.zeros((self.batch, self.nnz))
        self._check(self._lib.awempc_eval_nlp_host(self._h, _dptr(V), _dptr(p), _dptr(f), _dptr(g), _dptr(grad),
                                                   _dptr(jac)))
        return {"f": f, "g": g, "grad_f": grad, "jac": jac}

    def eval_f(self, V, P):
        """Host arrays in: f [B] (the derivative kernel; there is no value-only kernel for this NLP)."""
        return self.eval_nlp(V, P)["f"]

    def eval_g(self, V, P):
        """Host arrays in: g [B, n_g] (the derivative kernel)."""
        return self.eval_nlp(V, P)["g"]

    # ---- CasADi nlpsol oracle names (one instance) -----------------------------------
    def _single(self, x, p):
        if self.batch != 1:
            raise ValueError("the oracle-named entry points evaluate one instance (batch=1)")
        return self.eval_nlp(np.asarray(x).reshape(1, -1), np.asarray(p).reshape(1, -1))

    def nlp_f(self, x, p):
        return float(self._single(x, p)["f"][0])

    def nlp_g(self, x, p):
        return self._single(x, p)["g"][0]

    def nlp_grad_f(self, x, p):
        out = self._single(x, p)
        return float(out["f"][0]), out["grad_f"][0]

    def nlp_jac_g(self, x, p):
        out = self._single(x, p)
        return out["g"][0], self.jac_csc(out["jac"][0])
