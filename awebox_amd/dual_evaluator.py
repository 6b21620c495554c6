"""ctypes binding of ``libawedual.so`` (include/awedual.h): the multi-kite NLP oracle surface.

``DualEvaluator`` serves ``nlp_f`` / ``nlp_g`` / ``nlp_grad_f`` / ``nlp_jac_g`` / ``nlp_hess_l`` for the dual-kite
power-cycle NLP (config 3) with CasADi's argument meaning (x = V, p = P) and J_g in CCS
(awebox/opti/preparation.py:366-400), plus the batched device-pointer path used by the sweep
driver and ``bench.py``.  No CPU fallback: a missing library or device raises
``AwegpuUnavailable``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import dual as du
from .evaluator import AWE_ERR_NODEVICE, AWE_OK, AwegpuError, AwegpuUnavailable, _dptr

_LIB = None
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libawedual.so")

EXPORTED_SYMBOLS = ["adl_create", "adl_destroy", "adl_last_error", "adl_sizes", "adl_sparsity_jac",
                    "adl_sparsity_jac_static", "adl_colour_counts", "adl_eval_nlp", "adl_eval_nlp_host",
                    "adl_last_kernel_ms", "adl_node_eval_host", "adl_hess_nnz", "adl_sparsity_hess",
                    "adl_sparsity_hess_static", "adl_eval_hess", "adl_eval_hess_host", "adl_last_hess_ms",
                    "adl_gen_status", "adl_eval_nlp_im", "adl_last_kernel_ms_im"]


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
    lib.adl_create.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(h)]
    lib.adl_destroy.argtypes = [h]
    lib.adl_last_error.restype = ctypes.c_char_p
    lib.adl_sizes.argtypes = [h, ip, ip, ip, ip]
    lib.adl_sparsity_jac.argtypes = [h, ip, ip]
    lib.adl_sparsity_jac_static.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ip, ip, ip]
    lib.adl_colour_counts.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ip, ip, ip, ip]
    lib.adl_eval_nlp.argtypes = [h] + [ctypes.c_void_p] * 7
    lib.adl_eval_nlp_host.argtypes = [h, dp, dp, dp, dp, dp, dp]
    lib.adl_last_kernel_ms.argtypes = [h, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.adl_node_eval_host.argtypes = [dp, dp, dp, ctypes.c_int, dp, dp]
    lib.adl_hess_nnz.argtypes = [h, ip]
    lib.adl_sparsity_hess.argtypes = [h, ip, ip]
    lib.adl_sparsity_hess_static.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ip, ip, ip]
    lib.adl_eval_hess.argtypes = [h] + [ctypes.c_void_p] * 6
    lib.adl_eval_hess_host.argtypes = [h, dp, dp, dp, dp, dp]
    lib.adl_last_hess_ms.argtypes = [h, ctypes.POINTER(ctypes.c_float)]
    lib.adl_gen_status.argtypes = [h, ip]
    lib.adl_eval_nlp_im.argtypes = [h] + [ctypes.c_void_p] * 6 + [ctypes.c_size_t, ctypes.c_void_p]
    lib.adl_last_kernel_ms_im.argtypes = [h] + [ctypes.POINTER(ctypes.c_float)] * 4
    _LIB = lib
    return lib


def _err(lib):
    return lib.adl_last_error().decode()


def sparsity_jac_static(consts: du.MultiConstants):
    """CCS pattern (colind, row) of J_g derived on the CPU -- no device needed."""
    lib = load_library()
    cfg = consts.cfg
    c = np.ascontiguousarray(consts.consts, dtype=np.float64)
    nnz = ctypes.c_int()
    ip = ctypes.POINTER(ctypes.c_int)
    if lib.adl_sparsity_jac_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz), None, None) != AWE_OK:
        raise AwegpuError(_err(lib))
    lay = du.layout_for(consts)
    colind = np.zeros(lay.n_v + 1, dtype=np.int32)
    row = np.zeros(nnz.value, dtype=np.int32)
    if lib.adl_sparsity_jac_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz),
                                   colind.ctypes.data_as(ip), row.ctypes.data_as(ip)) != AWE_OK:
        raise AwegpuError(_err(lib))
    return colind, row


def sparsity_hess_static(consts: du.MultiConstants):
    """Upper-triangular CCS pattern (colind, row) of nlp_hess_l derived on the CPU."""
    lib = load_library()
    cfg = consts.cfg
    c = np.ascontiguousarray(consts.consts, dtype=np.float64)
    nnz = ctypes.c_int()
    ip = ctypes.POINTER(ctypes.c_int)
    if lib.adl_sparsity_hess_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz), None, None) != AWE_OK:
        raise AwegpuError(_err(lib))
    lay = du.layout_for(consts)
    colind = np.zeros(lay.n_v + 1, dtype=np.int32)
    row = np.zeros(nnz.value, dtype=np.int32)
    if lib.adl_sparsity_hess_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz),
                                    colind.ctypes.data_as(ip), row.ctypes.data_as(ip)) != AWE_OK:
        raise AwegpuError(_err(lib))
    return colind, row


def colour_counts(consts: du.MultiConstants):
    """(colours at the shooting node, at a Radau node, tangent entries of each) -- CPU only."""
    lib = load_library()
    c = np.ascontiguousarray(consts.consts, dtype=np.float64)
    out = [ctypes.c_int() for _ in range(4)]
    if lib.adl_colour_counts(consts.cfg.n_k, consts.cfg.d, _dptr(c), c.size, *[ctypes.byref(o) for o in out]) != AWE_OK:
        raise AwegpuError(_err(lib))
    return tuple(o.value for o in out)


def node_eval_host(w: np.ndarray, theta0: np.ndarray, consts: du.MultiConstants):
    """Diagnostics (CPU): values [75] and Jacobian [75, 127] of one node of the HIP model's
    source, evaluated on the host in dual arithmetic (the kernel's model code, not the oracle)."""
    lib = load_library()
    w = np.ascontiguousarray(w, dtype=np.float64)
    th = np.ascontiguousarray(theta0, dtype=np.float64)
    c = np.ascontiguousarray(consts.consts, dtype=np.float64)
    val = np.zeros(75)
    jac = np.zeros((75, 127))
    if lib.adl_node_eval_host(_dptr(w), _dptr(th), _dptr(c), c.size, _dptr(val), _dptr(jac)) != AWE_OK:
        raise AwegpuError(_err(lib))
    return val, jac


class DualEvaluator:
    """HIP evaluator of the dual-kite direct-collocation NLP for ``batch`` (V, P) instances."""

    def __init__(self, consts: du.MultiConstants | None = None, batch: int = 1):
        self.consts = consts or du.build_constants()
        cfg = self.consts.cfg
        self.layout = du.layout_for(self.consts)
        self.batch = int(batch)
        self._lib = load_library()
        c = np.ascontiguousarray(self.consts.consts, dtype=np.float64)
        handle = ctypes.c_void_p()
        self._check(self._lib.adl_create(cfg.n_k, cfg.d, _dptr(c), c.size, self.batch, ctypes.byref(handle)))
        self._h = handle
        n_v, n_g, n_p, nnz = (ctypes.c_int() for _ in range(4))
        self._check(self._lib.adl_sizes(self._h, ctypes.byref(n_v), ctypes.byref(n_g), ctypes.byref(n_p),
                                        ctypes.byref(nnz)))
        self.n_v, self.n_g, self.n_p, self.nnz = n_v.value, n_g.value, n_p.value, nnz.value
        assert (self.n_v, self.n_g, self.n_p) == (self.layout.n_v, self.layout.n_g, self.layout.n_p)
        self._colind = np.zeros(self.n_v + 1, dtype=np.int32)
        self._row = np.zeros(self.nnz, dtype=np.int32)
        ip = ctypes.POINTER(ctypes.c_int)
        self._check(self._lib.adl_sparsity_jac(self._h, self._colind.ctypes.data_as(ip), self._row.ctypes.data_as(ip)))

    def _check(self, rc):
        if rc != AWE_OK:
            msg = _err(self._lib)
            if rc == AWE_ERR_NODEVICE:
                raise AwegpuUnavailable(msg)
            raise AwegpuError(f"awedual error {rc}: {msg}")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.adl_destroy(self._h)
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

    @property
    def generated_available(self) -> bool:
        """Whether the generated instance-minor path (adl_eval_nlp_im) serves these constants."""
        ok = ctypes.c_int()
        self._check(self._lib.adl_gen_status(self._h, ctypes.byref(ok)))
        return bool(ok.value)

    def eval_nlp_device(self, V, P, f, g, grad_f, jac, stream=None):
        """f, g, grad f, J_g for all instances; float64 CUDA tensors V [B, n_v], P [B, n_p], f [B],
        g [B, n_g] (contiguous) and grad_f [B, n_v], jac [B, nnz]: both contiguous (adl_eval_nlp, the
        colour kernel), or both instance-minor views ``x_t.t()`` of contiguous [n, ld] tensors with one
        ld >= B (adl_eval_nlp_im, the generated node code; ``alloc_grad`` / ``alloc_jac``)."""
        import torch
        for t, n in ((V, self.n_v), (P, self.n_p), (f, 1), (g, self.n_g)):
            if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous() or t.numel() != self.batch * n:
                raise ValueError("device tensors must be contiguous float64 CUDA tensors of the batch shape")
        for t, n in ((grad_f, self.n_v), (jac, self.nnz)):
            if t.dtype != torch.float64 or not t.is_cuda or tuple(t.shape) != (self.batch, n):
                raise ValueError("grad_f and jac must be float64 CUDA tensors [batch, n]")
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        im = lambda t: t.stride(0) == 1 and t.stride(1) >= self.batch   # noqa: E731
        if jac.is_contiguous() and grad_f.is_contiguous():
            self._check(self._lib.adl_eval_nlp(self._h, V.data_ptr(), P.data_ptr(), f.data_ptr(), g.data_ptr(),
                                               grad_f.data_ptr(), jac.data_ptr(), ctypes.c_void_p(s)))
        elif im(jac) and im(grad_f) and jac.stride(1) == grad_f.stride(1):
            self._check(self._lib.adl_eval_nlp_im(self._h, V.data_ptr(), P.data_ptr(), f.data_ptr(), g.data_ptr(),
                                                  grad_f.data_ptr(), jac.data_ptr(), int(jac.stride(1)),
                                                  ctypes.c_void_p(s)))
        else:
            raise ValueError("jac and grad_f must both be contiguous or both instance-minor views "
                             "(strides (1, ld), one ld)")

    def alloc_jac(self, device="cuda", instance_minor=False):
        """A J_g value tensor [B, nnz]: instance-minor (the transposed view of [nnz, B], written by the
        generated path with coalesced stores) when asked for, per instance otherwise."""
        import torch
        if instance_minor:
            return torch.zeros(self.nnz, self.batch, dtype=torch.float64, device=device).t()
        return torch.zeros(self.batch, self.nnz, dtype=torch.float64, device=device)

    def alloc_grad(self, device="cuda", instance_minor=False):
        """A grad f tensor [B, n_v] in the layout of ``alloc_jac``."""
        import torch
        if instance_minor:
            return torch.zeros(self.n_v, self.batch, dtype=torch.float64, device=device).t()
        return torch.zeros(self.batch, self.n_v, dtype=torch.float64, device=device)

    def last_kernel_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        self._check(self._lib.adl_last_kernel_ms(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def last_kernel_ms_im(self):
        """(input transposition, node kernel, interval kernel, finalize) of the last instance-minor
        evaluation, ms."""
        v = [ctypes.c_float() for _ in range(4)]
        self._check(self._lib.adl_last_kernel_ms_im(self._h, *(ctypes.byref(x) for x in v)))
        return tuple(x.value for x in v)

    def eval_nlp(self, V, P):
        V = np.ascontiguousarray(np.asarray(V, dtype=np.float64).reshape(self.batch, self.n_v))
        P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(self.batch, self.n_p))
        f = np.zeros(self.batch)
        g = np.zeros((self.batch, self.n_g))
        grad = np.zeros((self.batch, self.n_v))
        jac = np.zeros((self.batch, self.nnz))
        self._check(self._lib.adl_eval_nlp_host(self._h, _dptr(V), _dptr(P), _dptr(f), _dptr(g), _dptr(grad),
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

    # ---- Hessian of the Lagrangian (exact, dual_hess_kernel) ----------------------------
    @property
    def nnz_h(self):
        if not hasattr(self, "_hrow"):
            hn = ctypes.c_int()
            self._check(self._lib.adl_hess_nnz(self._h, ctypes.byref(hn)))
            self._hcolind = np.zeros(self.n_v + 1, dtype=np.int32)
            self._hrow = np.zeros(hn.value, dtype=np.int32)
            ip = ctypes.POINTER(ctypes.c_int)
            self._check(self._lib.adl_sparsity_hess(self._h, self._hcolind.ctypes.data_as(ip),
                                                    self._hrow.ctypes.data_as(ip)))
        return len(self._hrow)

    def sparsity_hess(self):
        """Upper-triangular CCS pattern of nlp_hess_l: (colind[n_v+1], row[nnz_h])."""
        self.nnz_h
        return self._hcolind.copy(), self._hrow.copy()

    def hess_csc(self, values, full=True):
        """scipy CSC of the Hessian values (full symmetric matrix unless ``full`` is False)."""
        import scipy.sparse as sp
        colind, row = self.sparsity_hess()
        U = sp.csc_matrix((np.asarray(values), row, colind), shape=(self.n_v, self.n_v))
        if not full:
            return U
        return (U + U.T - sp.diags(U.diagonal())).tocsc()

    def eval_hess_device(self, V, P, sigma, lam_g, H, stream=None):
        """Upper-triangular CCS values of sigma f + lam_g^T g for every instance: contiguous float64
        CUDA tensors V [B, n_v], P [B, n_p], sigma [B], lam_g [B, n_g], H [B, nnz_h]."""
        import torch
        for t, n in ((V, self.n_v), (P, self.n_p), (sigma, 1), (lam_g, self.n_g), (H, self.nnz_h)):
            if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous() or t.numel() != self.batch * n:
                raise ValueError("device tensors must be contiguous float64 CUDA tensors of the batch shape")
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._check(self._lib.adl_eval_hess(self._h, V.data_ptr(), P.data_ptr(), sigma.data_ptr(),
                                            lam_g.data_ptr(), H.data_ptr(), ctypes.c_void_p(s)))

    def eval_hess(self, V, P, sigma, lam_g):
        V = np.ascontiguousarray(np.asarray(V, dtype=np.float64).reshape(self.batch, self.n_v))
        P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(self.batch, self.n_p))
        sig = np.ascontiguousarray(np.broadcast_to(np.asarray(sigma, dtype=np.float64), (self.batch,)))
        lam = np.ascontiguousarray(np.asarray(lam_g, dtype=np.float64).reshape(self.batch, self.n_g))
        H = np.zeros((self.batch, self.nnz_h))
        self._check(self._lib.adl_eval_hess_host(self._h, _dptr(V), _dptr(P), _dptr(sig), _dptr(lam), _dptr(H)))
        return H

    def nlp_hess_l(self, x, p, lam_f, lam_g):
        """CasADi nlp_hess_l: Hessian of lam_f f + lam_g^T g (upper triangle, CCS values)."""
        if self.batch != 1:
            raise ValueError("the oracle-named entry points evaluate one instance (batch=1)")
        return self.eval_hess(np.asarray(x).reshape(1, -1), np.asarray(p).reshape(1, -1), lam_f,
                              np.asarray(lam_g).reshape(1, -1))[0]

    def last_hess_ms(self):
        a = ctypes.c_float()
        self._check(self._lib.adl_last_hess_ms(self._h, ctypes.byref(a)))
        return a.value
