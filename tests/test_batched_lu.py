"""The batched LU kernel (libawelu.so) against torch.linalg on an MI355X: P A = L U, and
torch.linalg.lu_solve on its output solves A x = b (relative residual <= 1e-12)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.build import LIB_LU, build_one
    build_one(LIB_LU)
    return torch


@pytest.mark.parametrize("batch,n", [(1, 1), (3, 17), (40, 268), (20, 640), (2, 1000)])
def test_lu_factor_matches_definition(gpu, batch, n):
    torch = gpu
    from awebox_amd.batched_lu import lu_factor
    g = torch.Generator(device="cuda").manual_seed(n)
    A = torch.randn(batch, n, n, dtype=torch.float64, device="cuda", generator=g)
    A[:, :, 0] *= 1e-3                                    # forces row interchanges
    LU, piv = lu_factor(A)
    P, L, U = torch.lu_unpack(LU, piv)
    assert torch.allclose(P @ L @ U, A, rtol=0, atol=1e-11 * A.abs().max().item() * n)
    rhs = torch.randn(batch, n, 3, dtype=torch.float64, device="cuda", generator=g)
    x = torch.linalg.lu_solve(LU, piv, rhs)
    res = (A @ x - rhs).abs().max() / (A.abs().max() * x.abs().max() + rhs.abs().max())
    assert res.item() < 1e-12
    # partial pivoting: every multiplier is bounded by 1 in magnitude (the pivot sequence itself may
    # differ from LAPACK's where rounding flips a near-tie; then all later choices differ too)
    assert L.abs().max().item() <= 1.0 + 1e-12
