"""Exact Hessian of the dual-kite Lagrangian (libawedual.so, dual_hess_kernel, nlp_hess_l) on an
MI355X.

* Parity with the CPU oracle (oracle/multikite_oracle.py, torch.func Hessians of the interval rows
  and of the whole objective) through the committed fixtures tests/golden/dual_hess_*.npz
  (tests/golden/make_dual_hess_golden.py): |a - b| <= 1e-9 |b| + 1e-11 max|H|, the fp64 tolerance
  of the AP2 Hessian parity test (test_gpu_parity.py).  psi is set strictly inside (0, 1) so the
  tracking and the period-coupled power cost both contribute.
* Config 3 at its full size (N=60, d=4): agreement with the coloured central differences of the
  exact HIP gradient (fd_hessian.py), |H_fd - H| <= 1e-6 max|column| + 1e-9 max|H|, which is the
  size-independent check available where the oracle is too slow; plus batch invariance and
  bitwise-repeatable launches.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from awebox_amd import dual as du
from awebox_amd import problem as pb

from test_gpu_parity import _close_hess  # noqa: E402  (tests/ is on sys.path)

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.build import LIB_DUAL, build_one
    build_one(LIB_DUAL)
    return torch


def _fixture(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    n_k, d = int(z["n_k"]), int(z["d"])
    mc = du.build_constants(du.MultiConfig(n_k=n_k, d=d))
    lay = du.layout_for(mc)
    U = sp.csc_matrix((z["H_data"], z["H_indices"], z["H_indptr"]), shape=(lay.n_v, lay.n_v))
    Ho = (U + sp.triu(U, 1).T).tocsc()
    return mc, lay, z, Ho


@pytest.mark.parametrize("name", ["dual_hess_n3_d2", "dual_hess_n4_d3"])
def test_dual_hessian_matches_oracle(gpu, name):
    from awebox_amd.dual_evaluator import DualEvaluator
    mc, lay, z, Ho = _fixture(name)
    ev = DualEvaluator(mc, batch=1)
    H = ev.eval_hess(z["V"], z["P"], float(z["sigma"]), z["lam"])
    _close_hess(ev.hess_csc(H[0]), Ho)
    # the oracle's nonzeros lie inside the kernel's structural pattern
    ci, ri = ev.sparsity_hess()
    pat = sp.csc_matrix((np.ones(len(ri)), ri, ci), shape=Ho.shape)
    pat = pat + sp.triu(pat, 1).T
    outside = abs(Ho) - abs(Ho).multiply(pat != 0)
    assert outside.max() <= 1e-12 * abs(Ho).max()


def test_dual_hessian_batch_and_repeatability(gpu):
    torch = gpu
    from awebox_amd.dual_evaluator import DualEvaluator
    mc, lay, z, Ho = _fixture("dual_hess_n3_d2")
    V0 = du.initial_guess(mc, lay)
    Vs = np.stack([z["V"], du.batch_member(V0, lay, 5), du.batch_member(V0, lay, 6)])
    Ps = np.stack([z["P"], du.pack_p(lay, mc, V0, "fictitious0", u_ref=6.0), du.pack_p(lay, mc, V0, "final0")])
    sig = np.array([float(z["sigma"]), 0.0, 2.5])
    lams = np.stack([z["lam"]] + [np.random.default_rng(s).standard_normal(lay.n_g) for s in (1, 2)])
    evb = DualEvaluator(mc, batch=3)
    Hb = evb.eval_hess(Vs, Ps, sig, lams)
    _close_hess(evb.hess_csc(Hb[0]), Ho, "H[0]")
    ev1 = DualEvaluator(mc, batch=1)
    for b in range(3):
        assert np.array_equal(ev1.eval_hess(Vs[b], Ps[b], sig[b], lams[b])[0], Hb[b]), f"batch member {b}"
    dev = lambda a: torch.tensor(np.ascontiguousarray(a), device="cuda")
    Hd = torch.zeros(3, evb.nnz_h, dtype=torch.float64, device="cuda")
    for _ in range(2):
        evb.eval_hess_device(dev(Vs), dev(Ps), dev(sig), dev(lams), Hd)
        torch.cuda.synchronize()
        assert np.array_equal(Hd.cpu().numpy(), Hb)
    assert evb.last_hess_ms() > 0


def test_dual_hessian_config3_against_differences(gpu):
    """N=60 d=4 (config 3): exact kernel vs the difference Hessian of the exact HIP gradient."""
    torch = gpu
    from awebox_amd.dual_evaluator import DualEvaluator
    from awebox_amd.fd_hessian import FdHessian
    mc = du.build_constants(du.MultiConfig(n_k=60, d=4))
    lay = du.layout_for(mc)
    V0 = du.initial_guess(mc, lay)
    V = du.batch_member(V0, lay, 3)
    V[lay.phi()[pb.PHI_NAMES.index("psi")]] = 0.5
    P = du.pack_p(lay, mc, V0, "power1")
    lam = np.random.default_rng(9).standard_normal(lay.n_g)
    ev = DualEvaluator(mc, batch=1)
    fd = FdHessian(ev, lambda B: DualEvaluator(mc, batch=B), lay, device="cuda")
    dev = lambda a: torch.tensor(np.ascontiguousarray(a).reshape(1, -1), device="cuda")
    sig = torch.ones(1, dtype=torch.float64, device="cuda")
    He = torch.empty(1, ev.nnz_h, dtype=torch.float64, device="cuda")
    ev.eval_hess_device(dev(V), dev(P), sig, dev(lam), He)
    Hf = torch.empty(1, fd.nnz_h, dtype=torch.float64, device="cuda")
    fd.eval_hess_device(dev(V), dev(P), sig, dev(lam), Hf)
    torch.cuda.synchronize()
    ci, ri = ev.sparsity_hess()
    A = sp.csc_matrix((He.cpu().numpy()[0], ri, ci), shape=(lay.n_v, lay.n_v))
    ci2, ri2 = fd.sparsity_hess()
    B = sp.csc_matrix((Hf.cpu().numpy()[0], ri2, ci2), shape=(lay.n_v, lay.n_v))
    assert np.isfinite(A.data).all()
    # the exact pattern lies inside the dense-per-interval difference pattern
    patB = sp.csc_matrix((np.ones(len(ri2)), ri2, ci2), shape=A.shape)
    assert (abs(A) - abs(A).multiply(patB != 0)).nnz == 0 or (abs(A) - abs(A).multiply(patB != 0)).max() == 0
    colmax = np.asarray(abs(A).max(axis=0).todense()).ravel()
    D = abs(B - A).tocsc()
    tol_col = 1e-6 * colmax + 1e-9 * abs(A).max()
    worst = np.asarray(D.max(axis=0).todense()).ravel() - tol_col
    assert worst.max() <= 0, f"worst column {worst.argmax()}: {np.asarray(D.max(axis=0).todense()).ravel()[worst.argmax()]:.2e}"
