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


@pytest.mark.parametrize("batch,n,nrhs", [(1, 1, 1), (5, 17, 3), (256, 60, 1), (64, 126, 22), (16, 463, 1),
                                          (3, 1000, 40)])
def test_lu_solve_matches_torch(gpu, batch, n, nrhs):
    """awelu_solve_batched (LDS-resident right-hand sides, chunked when n (16 + nrhs) doubles exceed
    the LDS budget, as for n = 1000, nrhs = 40) against torch.linalg.lu_solve on the same factors."""
    torch = gpu
    from awebox_amd.batched_lu import lu_factor, lu_solve
    g = torch.Generator(device="cuda").manual_seed(7 * n + nrhs)
    A = torch.randn(batch, n, n, dtype=torch.float64, device="cuda", generator=g)
    A[:, :, 0] *= 1e-3
    rhs = torch.randn(batch, n, nrhs, dtype=torch.float64, device="cuda", generator=g)
    LU, piv = lu_factor(A)
    x = lu_solve(LU, piv, rhs)
    x_ref = torch.linalg.lu_solve(LU, piv, rhs)
    assert (x - x_ref).abs().max().item() <= 1e-10 * x_ref.abs().max().item()
    res = (A @ x - rhs).abs().max() / (A.abs().max() * x.abs().max() + rhs.abs().max())
    assert res.item() < 1e-12


@pytest.mark.parametrize("batch,nb,m,nrhs", [(1, 1, 1, 1), (4, 5, 7, 2), (256, 21, 22, 1), (3, 9, 32, 8),
                                            (1, 81, 23, 30), (2, 41, 46, 70), (8, 41, 46, 1), (1, 7, 48, 3)])
def test_btd_solve_matches_dense(gpu, batch, nb, m, nrhs):
    """awelu_btd_factor_batched + awelu_btd_solve_batched (chunked beyond 64 right-hand sides, as
    for nrhs = 70) against a dense solve of the assembled block-tridiagonal matrix;
    KKT-like blocks (indefinite diagonal blocks with a zero-ish corner) exercise the in-block
    pivoting."""
    torch = gpu
    from awebox_amd.batched_lu import btd_dense, btd_factor, btd_solve
    g = torch.Generator(device="cuda").manual_seed(nb * m + nrhs)
    T = torch.randn(batch, nb, 3, m, m, dtype=torch.float64, device="cuda", generator=g)
    T[:, :, 1] += 4.0 * torch.eye(m, dtype=torch.float64, device="cuda")
    T[:, :, 1, : m // 2, : m // 2] *= 1e-6
    X = torch.randn(batch, nb, m, nrhs, dtype=torch.float64, device="cuda", generator=g)
    F, Dinv = btd_factor(T)
    x = btd_solve(F, Dinv, X)
    assert torch.equal(btd_solve(F, Dinv, X), x)          # the factors are reusable
    A = btd_dense(T).cpu()                               # host LAPACK as the independent reference
    b = X.reshape(batch, nb * m, nrhs).cpu()
    xs = x.reshape(batch, nb * m, nrhs).cpu()
    x_ref = torch.linalg.solve(A, b)
    scale = A.abs().amax(dim=(1, 2)) * xs.abs().amax(dim=(1, 2)) + b.abs().amax(dim=(1, 2))
    res = ((A @ xs - b).abs().amax(dim=(1, 2)) / scale).max().item()
    # backward error of the block sweep: explicit pivot-block inverses with one refinement step per
    # block solve, and no interchanges between block rows (1e-11 measured on the 256 random systems)
    assert res < 1e-10
    cond = torch.linalg.cond(A)                          # forward error: cond x eps x block growth
    fwd = ((xs - x_ref).abs().amax(dim=(1, 2)) / x_ref.abs().amax(dim=(1, 2)))
    assert bool((fwd <= 1e-13 * cond + 1e-10).all())
