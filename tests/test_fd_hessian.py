"""The coloured central-difference Hessian (awebox_amd/fd_hessian.py) against the exact AP2 Hessian
kernel (nlp_hess_l, parity-tested against the oracle in test_gpu_parity.py) on an MI355X.

Tolerance: central differences with h = 1e-5 (1 + |x|):
|H_fd - H| <= 1e-6 max|column of H| + 1e-9 max|H|.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from awebox_amd import problem as pb
from awebox_amd.initial_guess import batch_member, initial_guess

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.build import build
    build()
    return torch


@pytest.mark.parametrize("n_k,d", [(5, 3), (40, 4)])
def test_fd_hessian_matches_exact_kernel(gpu, n_k, d):
    torch = gpu
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.fd_hessian import FdHessian
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    V = batch_member(v0, lay, 3)
    P = pb.pack_p(lay, consts, v0)
    ev = Ap2Evaluator(consts, batch=1)
    fd = FdHessian(ev, lambda B: Ap2Evaluator(consts, batch=B), lay, device="cuda")
    lam = np.random.default_rng(7).standard_normal(lay.n_g)
    Vt = torch.tensor(V.reshape(1, -1), device="cuda")
    Pt = torch.tensor(P.reshape(1, -1), device="cuda")
    sig = torch.ones(1, dtype=torch.float64, device="cuda")
    lt = torch.tensor(lam.reshape(1, -1), device="cuda")
    He = torch.empty(1, ev.nnz_h, dtype=torch.float64, device="cuda")
    ev.eval_hess_device(Vt, Pt, sig, lt, He)
    Hf = torch.empty(1, fd.nnz_h, dtype=torch.float64, device="cuda")
    fd.eval_hess_device(Vt, Pt, sig, lt, Hf)
    torch.cuda.synchronize()
    ci, ri = ev.sparsity_hess()
    A = sp.csc_matrix((He.cpu().numpy()[0], ri, ci), shape=(lay.n_v, lay.n_v)).toarray()
    ci2, ri2 = fd.sparsity_hess()
    B = sp.csc_matrix((Hf.cpu().numpy()[0], ri2, ci2), shape=(lay.n_v, lay.n_v)).toarray()
    # the exact pattern lies inside the dense-per-interval FD pattern
    assert not np.any((A != 0) & (sp.csc_matrix((np.ones(len(ri2)), ri2, ci2), shape=A.shape).toarray() == 0))
    tol = 1e-6 * np.abs(A).max(axis=0) + 1e-9 * np.abs(A).max()
    excess = (np.abs(B - A) - tol[None, :]).max(axis=0)
    assert excess.max() <= 0, f"worst column {excess.argmax()}: {np.abs(B - A).max(axis=0)[excess.argmax()]:.2e}"
