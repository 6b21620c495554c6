"""Python side of the drop-in boundary: ctypes binding of ``libawegpu.so`` (include/awegpu.h).

``Ap2Evaluator`` exposes the NLP oracle surface IPOPT reaches through ``casadi.nlpsol`` in the
reference (awebox/opti/preparation.py:366-400): ``nlp_f``, ``nlp_g``, ``nlp_grad_f`` and
``nlp_jac_g`` with CasADi's argument meaning (x = V, p = P) and output convention (J_g in CCS,
column-major).  It also provides the batched device-pointer path used by the sweep / MPC drivers
and by ``bench.py``.

There is no CPU fallback: if the shared library is missing or no HIP device is visible, every
constructor raises ``AwegpuUnavailable``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import problem as pb

_LIB = None
_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libawegpu.so")

AWE_OK, AWE_ERR_ARG, AWE_ERR_HIP, AWE_ERR_NONFINITE, AWE_ERR_NODEVICE = 0, 1, 2, 3, 4

EXPORTED_SYMBOLS = ["awe_create", "awe_destroy", "awe_last_error", "awe_sizes", "awe_sparsity_jac",
                    "awe_sparsity_jac_static",
                    "awe_eval_nlp", "awe_eval_g", "awe_eval_f", "awe_eval_nlp_host", "awe_eval_f_host",
                    "awe_eval_g_host",
                    "awe_last_kernel_ms", "awe_device_count", "awe_hess_nnz", "awe_sparsity_hess",
                    "awe_sparsity_hess_static", "awe_eval_hess", "awe_eval_hess_host", "awe_last_hess_ms",
                    "awe_set_eval_path", "awe_get_eval_path", "awe_last_kernel_ms_gen", "awe_eval_nlp_im",
                    "awe_last_kernel_ms_soa", "awe_eval_hess_im", "awe_set_hess_path", "awe_get_hess_path",
                    "awe_eval_nlp_imv", "awe_instance_ld"]

PATH_COLOUR, PATH_GENERATED, PATH_SOA = 0, 1, 2


class AwegpuUnavailable(RuntimeError):
    """The HIP evaluator cannot run here (library not built or no MI355X visible)."""


class AwegpuError(RuntimeError):
    pass


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
    lib.awe_create.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(h)]
    lib.awe_destroy.argtypes = [h]
    lib.awe_last_error.restype = ctypes.c_char_p
    lib.awe_sizes.argtypes = [h, ip, ip, ip, ip]
    lib.awe_sparsity_jac.argtypes = [h, ip, ip]
    lib.awe_eval_nlp.argtypes = [h, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.awe_eval_nlp_im.argtypes = [h, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    lib.awe_last_kernel_ms_soa.argtypes = [h, ctypes.POINTER(ctypes.c_float)]
    lib.awe_eval_nlp_imv.argtypes = [h, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 4 + \
        [ctypes.c_int, ctypes.c_void_p]
    lib.awe_instance_ld.argtypes = [h, ip]
    lib.awe_eval_g.argtypes = [h, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.awe_eval_f.argtypes = [h, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.awe_eval_nlp_host.argtypes = [h, dp, dp, dp, dp, dp, dp]
    lib.awe_eval_f_host.argtypes = [h, dp, dp, dp]
    lib.awe_eval_g_host.argtypes = [h, dp, dp, dp]
    lib.awe_last_kernel_ms.argtypes = [h, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.awe_device_count.restype = ctypes.c_int
    lib.awe_sparsity_jac_static.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ip, ip, ip]
    lib.awe_sparsity_hess_static.argtypes = [ctypes.c_int, ctypes.c_int, dp, ctypes.c_int, ip, ip, ip]
    lib.awe_hess_nnz.argtypes = [h, ip]
    lib.awe_sparsity_hess.argtypes = [h, ip, ip]
    lib.awe_eval_hess.argtypes = [h] + [ctypes.c_void_p] * 6
    lib.awe_eval_hess_host.argtypes = [h, dp, dp, dp, dp, dp]
    lib.awe_last_hess_ms.argtypes = [h, ctypes.POINTER(ctypes.c_float)]
    lib.awe_set_eval_path.argtypes = [h, ctypes.c_int]
    lib.awe_get_eval_path.argtypes = [h, ip]
    lib.awe_last_kernel_ms_gen.argtypes = [h, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.awe_eval_hess_im.argtypes = [h] + [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_void_p]
    lib.awe_set_hess_path.argtypes = [h, ctypes.c_int]
    lib.awe_get_hess_path.argtypes = [h, ip]
    _LIB = lib
    return lib


def sparsity_jac_static(consts: pb.Ap2Constants):
    """CCS pattern (colind, row) of J_g derived on the CPU -- no device needed."""
    lib = load_library()
    cfg = consts.cfg
    c = np.ascontiguousarray(consts.consts, dtype=np.float64)
    nnz = ctypes.c_int()
    ip = ctypes.POINTER(ctypes.c_int)
    rc = lib.awe_sparsity_jac_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz), None, None)
    if rc != AWE_OK:
        raise AwegpuError(lib.awe_last_error().decode())
    lay = pb.NlpLayout(cfg.n_k, cfg.d)
    colind = np.zeros(lay.n_v + 1, dtype=np.int32)
    row = np.zeros(nnz.value, dtype=np.int32)
    rc = lib.awe_sparsity_jac_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz),
                                     colind.ctypes.data_as(ip), row.ctypes.data_as(ip))
    if rc != AWE_OK:
        raise AwegpuError(lib.awe_last_error().decode())
    return colind, row


def sparsity_hess_static(consts: pb.Ap2Constants):
    """Upper-triangular CCS pattern (colind, row) of nlp_hess_l derived on the CPU."""
    lib = load_library()
    cfg = consts.cfg
    c = np.ascontiguousarray(consts.consts, dtype=np.float64)
    nnz = ctypes.c_int()
    ip = ctypes.POINTER(ctypes.c_int)
    rc = lib.awe_sparsity_hess_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz), None, None)
    if rc != AWE_OK:
        raise AwegpuError(lib.awe_last_error().decode())
    lay = pb.NlpLayout(cfg.n_k, cfg.d)
    colind = np.zeros(lay.n_v + 1, dtype=np.int32)
    row = np.zeros(nnz.value, dtype=np.int32)
    rc = lib.awe_sparsity_hess_static(cfg.n_k, cfg.d, _dptr(c), c.size, ctypes.byref(nnz),
                                      colind.ctypes.data_as(ip), row.ctypes.data_as(ip))
    if rc != AWE_OK:
        raise AwegpuError(lib.awe_last_error().decode())
    return colind, row


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class Ap2Evaluator:
    """HIP evaluator of the AP2 direct-collocation NLP for ``batch`` (V, P) instances."""

    def __init__(self, consts: pb.Ap2Constants | None = None, batch: int = 1):
        self.consts = consts or pb.build_constants()
        cfg = self.consts.cfg
        self.layout = pb.NlpLayout(cfg.n_k, cfg.d)
        self.batch = int(batch)
        self._lib = load_library()
        if self._lib.awe_device_count() <= 0:
            raise AwegpuUnavailable("no HIP device visible: the evaluator has no CPU fallback")
        c = np.ascontiguousarray(self.consts.consts, dtype=np.float64)
        handle = ctypes.c_void_p()
        self._check(self._lib.awe_create(cfg.n_k, cfg.d, _dptr(c), c.size, self.batch, ctypes.byref(handle)))
        self._h = handle
        n_v, n_g, n_p, nnz = (ctypes.c_int() for _ in range(4))
        self._check(self._lib.awe_sizes(self._h, ctypes.byref(n_v), ctypes.byref(n_g), ctypes.byref(n_p),
                                        ctypes.byref(nnz)))
        self.n_v, self.n_g, self.n_p, self.nnz = n_v.value, n_g.value, n_p.value, nnz.value
        assert (self.n_v, self.n_g, self.n_p) == (self.layout.n_v, self.layout.n_g, self.layout.n_p)
        self._colind = np.zeros(self.n_v + 1, dtype=np.int32)
        self._row = np.zeros(self.nnz, dtype=np.int32)
        ip = ctypes.POINTER(ctypes.c_int)
        self._check(self._lib.awe_sparsity_jac(self._h, self._colind.ctypes.data_as(ip),
                                               self._row.ctypes.data_as(ip)))
        hn = ctypes.c_int()
        self._check(self._lib.awe_hess_nnz(self._h, ctypes.byref(hn)))
        self.nnz_h = hn.value
        self._hcolind = np.zeros(self.n_v + 1, dtype=np.int32)
        self._hrow = np.zeros(self.nnz_h, dtype=np.int32)
        self._check(self._lib.awe_sparsity_hess(self._h, self._hcolind.ctypes.data_as(ip),
                                                self._hrow.ctypes.data_as(ip)))

    # -------------------------------------------------------------------------------
    def _check(self, rc):
        if rc != AWE_OK:
            msg = self._lib.awe_last_error().decode()
            if rc == AWE_ERR_NODEVICE:
                raise AwegpuUnavailable(msg)
            raise AwegpuError(f"awegpu error {rc}: {msg}")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.awe_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sparsity_jac(self):
        """CCS pattern of J_g: (colind[n_v+1], row[nnz]) -- nlp_jac_g's output sparsity."""
        return self._colind.copy(), self._row.copy()

    # ---------------------------------------------- device path (torch CUDA tensors) ---
    def eval_nlp_device(self, V, P, f, g, grad_f, jac, stream=None):
        """f, g, grad f, J_g values for all batch members; fp64 CUDA tensors of shapes [B, n_v],
        [B, n_p], [B], [B, n_g] (contiguous), grad_f [B, n_v] and jac [B, nnz]: both contiguous
        (awe_eval_nlp), or both instance-minor views ``x_t.t()`` of contiguous [n, ld] tensors with
        one ld >= B (awe_eval_nlp_im, the layout the batched solver reads; ``alloc_grad`` /
        ``alloc_jac``)."""
        import torch
        ld_in = self.instance_ld
        vin_im = (self.batch > 1 and tuple(V.shape) == (self.batch, self.n_v) and V.stride() == (1, ld_in)
                  and tuple(P.shape) == (self.batch, self.n_p) and P.stride() == (1, ld_in))
        for t, n in ((V, self.n_v), (P, self.n_p), (g, self.n_g)):
            if t.dtype != torch.float64 or not t.is_cuda or t.numel() != self.batch * n or \
                    not (t.is_contiguous() or (vin_im and t is not g)):
                raise ValueError("device tensors must be contiguous float64 CUDA tensors of the batch shape "
                                 "(V and P may be instance-minor views from alloc_inputs)")
        if f.numel() != self.batch:
            raise ValueError("f must hold one value per batch member")
        for t, n, name in ((jac, self.nnz, "jac"), (grad_f, self.n_v, "grad_f")):
            if t.dtype != torch.float64 or not t.is_cuda or tuple(t.shape) != (self.batch, n):
                raise ValueError(f"{name} must be a float64 CUDA tensor of shape [batch, {n}]")
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        im = lambda t: t.stride(0) == 1 and t.stride(1) >= self.batch   # noqa: E731
        if vin_im:
            if not (im(jac) and im(grad_f) and jac.stride(1) == grad_f.stride(1)):
                raise ValueError("instance-minor V and P need instance-minor jac and grad_f")
            self._check(self._lib.awe_eval_nlp_imv(self._h, V.data_ptr(), P.data_ptr(), ld_in, f.data_ptr(),
                                                   g.data_ptr(), grad_f.data_ptr(), jac.data_ptr(),
                                                   int(jac.stride(1)), ctypes.c_void_p(s)))
        elif self.batch == 1 or (jac.is_contiguous() and grad_f.is_contiguous()):
            self._check(self._lib.awe_eval_nlp(self._h, V.data_ptr(), P.data_ptr(), f.data_ptr(), g.data_ptr(),
                                               grad_f.data_ptr(), jac.data_ptr(), ctypes.c_void_p(s)))
        elif im(jac) and im(grad_f) and jac.stride(1) == grad_f.stride(1):
            self._check(self._lib.awe_eval_nlp_im(self._h, V.data_ptr(), P.data_ptr(), f.data_ptr(),
                                                  g.data_ptr(), grad_f.data_ptr(), jac.data_ptr(),
                                                  int(jac.stride(1)), ctypes.c_void_p(s)))
        else:
            raise ValueError("jac and grad_f must both be contiguous or both instance-minor views "
                             "(strides (1, ld), one ld)")

    @property
    def instance_ld(self):
        """Leading dimension of the handle's instance-minor buffers (awe_instance_ld)."""
        v = ctypes.c_int()
        self._check(self._lib.awe_instance_ld(self._h, ctypes.byref(v)))
        return v.value

    def alloc_inputs(self, device="cuda"):
        """(V, P) value tensors [B, n_v], [B, n_p] stored instance-minor (the transposed views of
        contiguous [n, instance_ld] tensors): eval_nlp_device then runs awe_eval_nlp_imv, which reads
        them in place instead of transposing per-instance inputs (instance-minor path only)."""
        import torch
        ld = self.instance_ld
        return (torch.zeros(self.n_v, ld, dtype=torch.float64, device=device).t()[:self.batch],
                torch.zeros(self.n_p, ld, dtype=torch.float64, device=device).t()[:self.batch])

    def alloc_jac(self, device="cuda", instance_minor=True):
        """A J_g value tensor [B, nnz]; instance-minor (the transposed view of [nnz, B], which the
        instance-minor kernels write with coalesced stores) unless asked otherwise."""
        import torch
        if instance_minor:
            return torch.zeros(self.nnz, self.batch, dtype=torch.float64, device=device).t()
        return torch.zeros(self.batch, self.nnz, dtype=torch.float64, device=device)

    def alloc_grad(self, device="cuda", instance_minor=True):
        """A grad f tensor [B, n_v], instance-minor unless asked otherwise (pairs with alloc_jac)."""
        import torch
        if instance_minor:
            return torch.zeros(self.n_v, self.batch, dtype=torch.float64, device=device).t()
        return torch.zeros(self.batch, self.n_v, dtype=torch.float64, device=device)

    def last_kernel_ms_soa(self):
        """HIP-event times of the last instance-minor call: input transpose, node kernel, interval
        kernel, finalize, output transpose (ms)."""
        ms = (ctypes.c_float * 5)()
        self._check(self._lib.awe_last_kernel_ms_soa(self._h, ms))
        return [float(x) for x in ms]

    def eval_g_device(self, V, P, g, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._check(self._lib.awe_eval_g(self._h, V.data_ptr(), P.data_ptr(), g.data_ptr(), ctypes.c_void_p(s)))

    def eval_f_device(self, V, P, f, stream=None):
        import torch
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._check(self._lib.awe_eval_f(self._h, V.data_ptr(), P.data_ptr(), f.data_ptr(), ctypes.c_void_p(s)))

    def eval_hess_device(self, V, P, sigma, lam_g, H, stream=None):
        """Upper-triangular CCS values of the Hessian of sigma f + lam_g^T g for all batch
        members: sigma [B], lam_g [B, n_g], H [B, nnz_h] contiguous float64 CUDA tensors."""
        import torch
        for t, n in ((V, self.n_v), (P, self.n_p), (sigma, 1), (lam_g, self.n_g), (H, self.nnz_h)):
            if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous() or t.numel() != self.batch * n:
                raise ValueError("device tensors must be contiguous float64 CUDA tensors of the batch shape")
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._check(self._lib.awe_eval_hess(self._h, V.data_ptr(), P.data_ptr(), sigma.data_ptr(),
                                            lam_g.data_ptr(), H.data_ptr(), ctypes.c_void_p(s)))

    def eval_hess_device_im(self, V, P, sigma, lam_g, H, stream=None):
        """As eval_hess_device with H instance-minor: the transposed view ``x.t()`` of a contiguous
        [nnz_h, ld] tensor, ld >= B (awe_eval_hess_im; ``alloc_hess``)."""
        import torch
        for t, n in ((V, self.n_v), (P, self.n_p), (sigma, 1), (lam_g, self.n_g)):
            if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous() or t.numel() != self.batch * n:
                raise ValueError("device tensors must be contiguous float64 CUDA tensors of the batch shape")
        if H.dtype != torch.float64 or not H.is_cuda or tuple(H.shape) != (self.batch, self.nnz_h) or \
                H.stride(0) != 1 or H.stride(1) < self.batch:
            raise ValueError("H must be an instance-minor [batch, nnz_h] float64 view (strides (1, ld))")
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        self._check(self._lib.awe_eval_hess_im(self._h, V.data_ptr(), P.data_ptr(), sigma.data_ptr(),
                                               lam_g.data_ptr(), H.data_ptr(), int(H.stride(1)), ctypes.c_void_p(s)))

    def alloc_hess(self, device="cuda", instance_minor=True):
        """A Hessian value tensor [B, nnz_h], instance-minor unless asked otherwise."""
        import torch
        if instance_minor:
            return torch.zeros(self.nnz_h, self.batch, dtype=torch.float64, device=device).t()
        return torch.zeros(self.batch, self.nnz_h, dtype=torch.float64, device=device)

    HESS_PATHS = {"hyperdual": 0, "generated": 1, "follow": 2}

    @property
    def hess_path(self):
        """'generated' or 'hyperdual': the Hessian kernel the next call runs (include/awegpu.h)."""
        p = ctypes.c_int()
        self._check(self._lib.awe_get_hess_path(self._h, ctypes.byref(p)))
        return {0: "hyperdual", 1: "generated"}[p.value]

    @hess_path.setter
    def hess_path(self, name):
        self._check(self._lib.awe_set_hess_path(self._h, self.HESS_PATHS[name]))
        self._hess_mode = name

    @property
    def hess_mode(self):
        """The Hessian selection as set: 'follow' (the default: the kernel follows the evaluation
        path, resolved on every call), 'generated' or 'hyperdual'.  ``hess_path`` returns what the
        next call resolves to.  A solver that reads ``hess_path`` once to pick the H layout
        (ipm.DeviceNlp.h_im) only picks a layout: the C side dispatches the kernel on every call and
        both entry points (awe_eval_hess / awe_eval_hess_im) handle either kernel."""
        return getattr(self, "_hess_mode", "follow")

    def eval_hess(self, V, P, sigma, lam_g):
        """Host arrays in, host array out: H [B, nnz_h] (upper triangle, CCS)."""
        V = np.ascontiguousarray(np.asarray(V, dtype=np.float64).reshape(self.batch, self.n_v))
        P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(self.batch, self.n_p))
        sig = np.ascontiguousarray(np.broadcast_to(np.asarray(sigma, dtype=np.float64), (self.batch,)))
        lam = np.ascontiguousarray(np.asarray(lam_g, dtype=np.float64).reshape(self.batch, self.n_g))
        H = np.zeros((self.batch, self.nnz_h))
        self._check(self._lib.awe_eval_hess_host(self._h, _dptr(V), _dptr(P), _dptr(sig), _dptr(lam), _dptr(H)))
        return H

    def sparsity_hess(self):
        """Upper-triangular CCS pattern of nlp_hess_l: (colind[n_v+1], row[nnz_h])."""
        return self._hcolind.copy(), self._hrow.copy()

    def hess_csc(self, values, full=True):
        """scipy matrix from upper-triangular values; full=True adds the strict lower triangle."""
        import scipy.sparse as sp
        U = sp.csc_matrix((np.asarray(values), self._hrow, self._hcolind), shape=(self.n_v, self.n_v))
        return (U + sp.triu(U, 1).T).tocsc() if full else U

    def nlp_hess_l(self, x, p, lam_f, lam_g):
        """CasADi nlp_hess_l: Hessian of lam_f f + lam_g^T g (upper triangle, CCS values)."""
        if self.batch != 1:
            raise ValueError("the oracle-named entry points evaluate one instance (batch=1)")
        return self.eval_hess(np.asarray(x).reshape(1, -1), np.asarray(p).reshape(1, -1), lam_f,
                              np.asarray(lam_g).reshape(1, -1))[0]

    def last_hess_ms(self):
        a = ctypes.c_float()
        self._check(self._lib.awe_last_hess_ms(self._h, ctypes.byref(a)))
        return a.value

    def last_kernel_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        self._check(self._lib.awe_last_kernel_ms(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    # evaluation path of eval_nlp (include/awegpu.h): "soa" (the default: one lane per instance,
    # the build-time generated sparse-Jacobian code storing straight into J_g), "generated" (one
    # thread per collocation node, tangents gathered by a second kernel) or "colour" (compressed
    # forward mode)
    PATHS = {"colour": PATH_COLOUR, "generated": PATH_GENERATED, "soa": PATH_SOA}

    @property
    def path(self):
        p = ctypes.c_int()
        self._check(self._lib.awe_get_eval_path(self._h, ctypes.byref(p)))
        return {v: k for k, v in self.PATHS.items()}[p.value]

    @path.setter
    def path(self, name):
        self._check(self._lib.awe_set_eval_path(self._h, self.PATHS[name]))

    def last_kernel_ms_gen(self):
        """(node kernel ms, assembly kernel ms) of the last eval_nlp on the generated path."""
        a, b = ctypes.c_float(), ctypes.c_float()
        self._check(self._lib.awe_last_kernel_ms_gen(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    # ---------------------------------------------- host path (numpy) ----------------
    def eval_nlp(self, V, P):
        """Host arrays in, host arrays out: dict(f [B], g [B, n_g], grad_f [B, n_v], jac [B, nnz])."""
        V = np.ascontiguousarray(np.asarray(V, dtype=np.float64).reshape(self.batch, self.n_v))
        P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(self.batch, self.n_p))
        f = np.zeros(self.batch)
        g = np.zeros((self.batch, self.n_g))
        grad = np.zeros((self.batch, self.n_v))
        jac = np.zeros((self.batch, self.nnz))
        self._check(self._lib.awe_eval_nlp_host(self._h, _dptr(V), _dptr(P), _dptr(f), _dptr(g), _dptr(grad),
                                                _dptr(jac)))
        return {"f": f, "g": g, "grad_f": grad, "jac": jac}

    def jac_csc(self, values):
        import scipy.sparse as sp
        return sp.csc_matrix((np.asarray(values), self._row, self._colind), shape=(self.n_g, self.n_v))

    # ---- CasADi nlpsol oracle names (batch member 0) --------------------------------
    def _single(self, x, p):
        if self.batch != 1:
            raise ValueError("the oracle-named entry points evaluate one instance (batch=1)")
        return self.eval_nlp(np.asarray(x).reshape(1, -1), np.asarray(p).reshape(1, -1))

    def eval_f(self, V, P):
        """Host arrays in: f [B] from the value-only kernel (no derivatives)."""
        V = np.ascontiguousarray(np.asarray(V, dtype=np.float64).reshape(self.batch, self.n_v))
        P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(self.batch, self.n_p))
        f = np.zeros(self.batch)
        self._check(self._lib.awe_eval_f_host(self._h, _dptr(V), _dptr(P), _dptr(f)))
        return f

    def eval_g(self, V, P):
        """Host arrays in: g [B, n_g] from the value-only kernel (no derivatives)."""
        V = np.ascontiguousarray(np.asarray(V, dtype=np.float64).reshape(self.batch, self.n_v))
        P = np.ascontiguousarray(np.asarray(P, dtype=np.float64).reshape(self.batch, self.n_p))
        g = np.zeros((self.batch, self.n_g))
        self._check(self._lib.awe_eval_g_host(self._h, _dptr(V), _dptr(P), _dptr(g)))
        return g

    def nlp_f(self, x, p):
        if self.batch != 1:
            raise ValueError("the oracle-named entry points evaluate one instance (batch=1)")
        return float(self.eval_f(np.asarray(x).reshape(1, -1), np.asarray(p).reshape(1, -1))[0])

    def nlp_g(self, x, p):
        if self.batch != 1:
            raise ValueError("the oracle-named entry points evaluate one instance (batch=1)")
        return self.eval_g(np.asarray(x).reshape(1, -1), np.asarray(p).reshape(1, -1))[0]

    def nlp_grad_f(self, x, p):
        out = self._single(x, p)
        return float(out["f"][0]), out["grad_f"][0]

    def nlp_jac_g(self, x, p):
        out = self._single(x, p)
        return out["g"][0], self.jac_csc(out["jac"][0])
