"""Inertia of the structured KKT matrix (IPOPT's inertia correction, ipm.IpmOptions(inertia="exact")).

CPU: StructuredKKT.inertia (Haynsworth additivity over the interval blocks and the dense or
block-tridiagonal separator system) equals the eigenvalue counts of the assembled K.
GPU: the Bunch-Kaufman kernel (awelu_sym_inertia_batched) equals symmetric eigenvalue counts on
random indefinite and rank-deficient matrices, and the structured counts on the device equal the
host ones."""
import numpy as np
import pytest
import torch

from awebox_amd import homotopy as hm
from awebox_amd import problem as pb
from awebox_amd.initial_guess import initial_guess


def _case(device, evaluator, n_k=5, d=3, shift=0.0):
    from awebox_amd.ipm import DeviceNlp, StructuredKKT, _dense_A
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    st = hm.schedule(consts, lay, v0)[0]
    lbg, ubg = lay.g_bounds()
    nlp = DeviceNlp(evaluator(consts), pb.pack_p(lay, consts, v0, step=st.cost_step), st.lbx, st.ubx,
                    lbg, ubg, device)
    sk = StructuredKKT(nlp, lay, device, separators="btd")
    gen = torch.Generator().manual_seed(2)
    f64 = dict(dtype=torch.float64)
    hv = torch.randn(len(nlp.h_keep), generator=gen, **f64).to(device)
    jv = torch.randn(len(nlp.j_row), generator=gen, **f64).to(device)
    diag = (torch.rand(nlp.ny, generator=gen, **f64) + shift).to(device)
    N, ny = sk.N, nlp.ny
    K = torch.zeros(N, N, dtype=torch.float64, device=device)
    K[nlp.h_r, nlp.h_c] = hv
    K[nlp.h_c[nlp.h_offdiag], nlp.h_r[nlp.h_offdiag]] = hv[nlp.h_offdiag]
    i = torch.arange(ny, device=device)
    K[i, i] += diag
    _dense_A(nlp, jv, ny, K)
    return nlp, sk, hv, jv, diag, K


def _eig_counts(K):
    ev = torch.linalg.eigvalsh(K.cpu())
    tol = 1e-10 * ev.abs().max()
    return int((ev > tol).sum()), int((ev < -tol).sum()), int(((ev >= -tol) & (ev <= tol)).sum())


@pytest.mark.parametrize("btd,shift", [(False, 0.0), (True, 0.0), (False, 50.0), (True, 50.0)])
def test_structured_inertia_matches_eigenvalues(btd, shift):
    from oracle.cpu_device import CpuDeviceEvaluator
    nlp, sk, hv, jv, diag, K = _case("cpu", CpuDeviceEvaluator, shift=shift)
    sk.force_btd = btd
    sk.factor(hv, diag, jv, 0.0, nlp.mI)
    assert sk.use_btd == btd
    assert sk.inertia() == _eig_counts(K)


@pytest.mark.gpu
def test_bunch_kaufman_inertia_kernel():
    from awebox_amd.batched_lu import sym_inertia, sym_inertia_host
    gen = torch.Generator().manual_seed(3)
    for n, b in ((1, 3), (7, 5), (46, 41), (268, 8), (500, 2)):
        A = torch.randn(b, n, n, generator=gen, dtype=torch.float64)
        A = A + A.transpose(1, 2)
        if n > 2:                                   # rank-deficient members: zero eigenvalues
            U = torch.randn(n, n - 2, generator=gen, dtype=torch.float64)
            A[0] = U @ torch.diag(torch.linspace(-3, 2, n - 2, dtype=torch.float64)) @ U.T
        c = sym_inertia(A.cuda(), ztol=1e-11).cpu()
        ref = sym_inertia_host(A, ztol=1e-11)
        assert torch.equal(c, ref), (n, c, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("shift", [0.0, 50.0])
def test_structured_inertia_on_gpu(shift):
    from awebox_amd.evaluator import Ap2Evaluator
    nlp, sk, hv, jv, diag, K = _case("cuda", lambda c: Ap2Evaluator(c, batch=1), shift=shift)
    ref = _eig_counts(K)
    for sep in ("btd", "dense"):
        sk.btd_off = sep == "dense"
        sk.factor(hv, diag, jv, 0.0, nlp.mI)
        assert sk.inertia() == ref, sep
