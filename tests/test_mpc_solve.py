"""Converged tracking MPC (config 5 fidelity: Pmpc.step, pmpc.py:221-302) on the batched IPM.

CPU: the MPC variable bounds restate the model's system bounds and the MPC overrides; the
structured KKT elimination with the MPC's leading initial-condition rows (stage 0 of the separator
chain = [initial-condition multipliers, x[0]]) equals a dense solve, and its inertia the
eigenvalue counts; the coloured-difference Hessian covers the terminal-cost columns.
GPU: a converged solve of config 5's instances reaches the same KKT point as repeated real-time
iterations of the same instances (the bounds and path inequalities are inactive along the tracked
orbit), and the converged closed loop runs.
"""
import numpy as np
import pytest
import torch

from awebox_amd import kite3 as k3


def test_variable_bounds_restate_system_bounds():
    c = k3.build_constants(k3.Kite3Config(n_k=3, d=2))
    lay = k3.MpcLayout(3, 2)
    lb, ub = k3.variable_bounds(c, lay)
    s = c.scaling
    # x[0] released (pmpc.py:120-121); x[1..N] carry q_z >= 10, coeff, l_t, dl_t, ddl_t bounds
    assert np.all(np.isinf(lb[lay.x(0)])) and np.all(np.isinf(ub[lay.x(0)]))
    for k in (1, 3):
        x_lb, x_ub = lb[lay.x(k)] * s[:k3.NX], ub[lay.x(k)] * s[:k3.NX]
        np.testing.assert_allclose(x_lb[[2, 6, 7, 8, 9, 10]], [10.0, 0.0, -80 * np.pi / 180, 1e-2, -30.0, -100.0])
        np.testing.assert_allclose(x_ub[[6, 7, 8, 9, 10]], [2.0, 80 * np.pi / 180, 1e3, 30.0, 100.0])
        assert np.all(np.isinf(x_lb[[0, 1, 3, 4, 5]]))
    su = s[2 * k3.NX:2 * k3.NX + k3.NU]
    np.testing.assert_allclose(ub[lay.u(1)] * su, [0, 0, 0, 5.0, 80 * np.pi / 180, 100.0])
    np.testing.assert_allclose(lb[lay.u(1)] * su, [0, 0, 0, -5.0, -80 * np.pi / 180, -100.0])
    assert lb[lay.z(2)][0] == 0.0 and np.isinf(ub[lay.z(2)][0])
    fixed = lb >= ub
    assert fixed[:lay.v_intervals].all() and fixed[k3.fict_columns(lay)].all()
    assert fixed.sum() == lay.v_intervals + 3 * lay.n_k
    for j in range(lay.d):                                           # collocation variables free
        assert np.isinf(lb[lay.coll_x(1, j)]).all() and np.isinf(lb[lay.coll_z(1, j)]).all()


class _PatternEval:
    """The MPC NLP's sparsity (no values) for host-side KKT structure tests."""

    def __init__(self, c, lay):
        from awebox_amd.mpc import sparsity_jac_static
        self.colind, self.row = sparsity_jac_static(c)
        self.layout, self.n_v, self.n_g, self.n_p = lay, lay.n_v, lay.n_g, lay.n_p
        self.nnz, self.batch = len(self.row), 1

    def sparsity_jac(self):
        return self.colind.copy(), self.row.copy()


def _kkt_case(btd, n_k=3, d=2, shift=0.0):
    from awebox_amd.build import LIB_MPC, build_one
    from awebox_amd.fd_hessian import FdHessian
    from awebox_amd.ipm import DeviceNlp, StructuredKKT, _dense_A
    build_one(LIB_MPC)
    c = k3.build_constants(k3.Kite3Config(n_k=n_k, d=d))
    lay = k3.MpcLayout(n_k, d)
    ev = FdHessian(_PatternEval(c, lay), None, lay, device="cpu", tail=True)
    lb, ub = k3.variable_bounds(c, lay)
    lbg, ubg = lay.g_bounds()
    V, P = k3.batch_instance(c, lay, 0, 4)
    nlp = DeviceNlp(ev, P, lb, ub, lbg, ubg, "cpu")
    sk = StructuredKKT(nlp, lay, "cpu", separators="btd")
    sk.force_btd = btd
    gen = torch.Generator().manual_seed(5)
    f64 = dict(dtype=torch.float64)
    hv = torch.randn(len(nlp.h_keep), generator=gen, **f64)
    jv = torch.randn(len(nlp.j_row), generator=gen, **f64)
    diag = torch.rand(nlp.ny, generator=gen, **f64) + shift
    K = torch.zeros(sk.N, sk.N, **f64)
    K[nlp.h_r, nlp.h_c] = hv
    K[nlp.h_c[nlp.h_offdiag], nlp.h_r[nlp.h_offdiag]] = hv[nlp.h_offdiag]
    i = torch.arange(nlp.ny)
    K[i, i] += diag
    _dense_A(nlp, jv, nlp.ny, K)
    return lay, nlp, sk, hv, jv, diag, K


@pytest.mark.parametrize("btd", [False, True])
def test_structured_kkt_with_initial_rows_matches_dense(btd):
    lay, nlp, sk, hv, jv, diag, K = _kkt_case(btd)
    assert sk.btd is not None                        # stage 0 = [initial-condition rows, x[0]]
    sk.factor(hv, diag, jv, 0.0, nlp.mI)
    assert sk.use_btd == btd
    rhs = torch.randn(sk.N, generator=torch.Generator().manual_seed(6), dtype=torch.float64)
    x = sk.solve(rhs)
    ref = torch.linalg.solve(K, rhs)
    assert float((x - ref).abs().max()) <= 1e-9 * float(ref.abs().max())
    assert sk.n_dense == 0
    ev_ = torch.linalg.eigvalsh(K)
    tol = 1e-10 * ev_.abs().max()
    assert sk.inertia() == (int((ev_ > tol).sum()), int((ev_ < -tol).sum()), int((ev_.abs() <= tol).sum()))


def test_fd_hessian_covers_terminal_cost_columns():
    from awebox_amd.fd_hessian import FdHessian
    c = k3.build_constants(k3.Kite3Config(n_k=3, d=2))
    lay = k3.MpcLayout(3, 2)
    from awebox_amd.build import LIB_MPC, build_one
    build_one(LIB_MPC)
    pe = _PatternEval(c, lay)
    with_tail = FdHessian(pe, None, lay, device="cpu", tail=True)
    without = FdHessian(pe, None, lay, device="cpu")
    xN = lay.x(lay.n_k)
    colind, row = with_tail.sparsity_hess()
    for v in xN:                                     # the diagonal of every x[N] column
        assert v in row[colind[v]:colind[v + 1]]
    colind0, _ = without.sparsity_hess()
    assert np.all(np.diff(colind0)[xN] == 0)
    assert with_tail.nnz_h - without.nnz_h == sum(lay.v_intervals + p + 1 for p in range(k3.NX))


# ------------------------------------------------------------------ GPU -----------------------
@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from awebox_amd.build import build
    build()
    return torch.device("cuda:0")


@pytest.mark.gpu
def test_fd_hessian_matches_oracle_autograd(gpu):
    """The coloured-difference Lagrangian Hessian of the HIP MPC evaluator (terminal cost
    included) against the oracle's autograd Hessian, N=3 d=2."""
    from awebox_amd.fd_hessian import FdHessian
    from awebox_amd.mpc import MpcEvaluator
    from oracle.kite3_oracle import from_constants
    c = k3.build_constants(k3.Kite3Config(n_k=3, d=2))
    lay = k3.MpcLayout(3, 2)
    V, P = k3.batch_instance(c, lay, 1, 4)
    lam = np.random.default_rng(7).standard_normal(lay.n_g)
    ev = FdHessian(MpcEvaluator(c, 1), lambda b: MpcEvaluator(c, b), lay, device="cuda", tail=True)
    H = torch.zeros(1, ev.nnz_h, dtype=torch.float64, device="cuda")
    t = lambda a: torch.tensor(np.atleast_2d(a), dtype=torch.float64, device="cuda")  # noqa: E731
    ev.eval_hess_device(t(V), t(P), torch.ones(1, dtype=torch.float64, device="cuda"), t(lam), H)
    orc = from_constants(c, lay)
    lam_t = torch.tensor(lam)
    L = lambda v: orc.nlp_f(v, P, lay) + torch.dot(lam_t, torch.as_tensor(orc.nlp_g(v, P, lay)))  # noqa: E731
    Href = torch.func.hessian(L)(torch.tensor(V)).numpy()
    colind, row = ev.sparsity_hess()
    cols = np.repeat(np.arange(lay.n_v), np.diff(colind))
    got = np.zeros((lay.n_v, lay.n_v))
    got[row, cols] = H[0].cpu().numpy()
    up = np.triu(Href)
    scale = np.abs(up).max()
    assert np.abs(got - up).max() <= 1e-6 * scale
    mask = np.zeros_like(got, dtype=bool)
    mask[row, cols] = True
    assert np.abs(up[~mask]).max() <= 1e-12 * scale            # the pattern covers the Hessian
    xN = lay.x(lay.n_k)
    np.testing.assert_allclose(got[xN, xN], Href[xN, xN], rtol=1e-6)


@pytest.mark.gpu
def test_converged_mpc_reaches_rti_kkt_point(gpu):
    """Config 5 (N=20, d=4), four loops at four phases of the orbit, each tracking a dynamically
    feasible window (mpc_solve.simulated_reference) from x0 = the window's start + 0.01 N(0,1)
    on the invariant-free states (CL, roll, reel acceleration; mpc_solve.CONSISTENT_X0):
    the converged MPC solve with bounds, path inequalities and the exact Hessian (IPOPT tol 1e-6)
    and ten Gauss-Newton iterations on the equality rows (the RTI at fixed P) reach the same point,
    with every bound inactive -- one RTI trajectory is the converged MPC's to the solver's
    tolerance.  (Tracking the synthetic circle instead, the converged MPC saturates dCL/dt and
    the RTI's unconstrained step crosses lambda >= 0: only the bounded solve is faithful there.)"""
    from awebox_amd.mpc_solve import CONSISTENT_X0, BatchedPmpc, simulated_reference
    from awebox_amd.rti import BatchedRti
    c = k3.build_constants()
    B = 4
    pm = BatchedPmpc(c, B, device="cuda")
    pm.start()
    lay = pm.lay
    x_start = pm.P[:, lay.p_ref + lay.x(0)[0]:lay.p_ref + lay.x(0)[0] + k3.NX].clone()
    R = simulated_reference(pm, x_start)
    gen = torch.Generator().manual_seed(11)
    pm.P[:, lay.p_ref:lay.p_ref + lay.n_v] = R
    noise = torch.zeros(B, k3.NX, dtype=torch.float64)
    noise[:, list(CONSISTENT_X0)] = 0.01 * torch.randn(B, len(CONSISTENT_X0), generator=gen, dtype=torch.float64)
    pm.P[:, lay.p_x0:lay.p_x0 + k3.NX] = x_start + noise.cuda()
    pm.V.copy_(R)
    V_init = pm.V.clone()
    for _ in range(10):
        eq, _ = BatchedRti.iterate(pm)
    torch.cuda.synchronize()
    assert float(eq.max()) < 1e-9
    Vr = pm.V.cpu().numpy()
    pm.V.copy_(V_init)
    res = pm.solve()
    assert all(r.status == "solve_succeeded" for r in res), [r.status for r in res]
    Vp = pm.V.cpu().numpy()
    free = pm.free
    lb, ub = pm.lbx[free], pm.ubx[free]
    gap = np.minimum(Vp[:, free] - lb, ub - Vp[:, free])
    assert gap.min() > 1e-3                                   # no bound active at the solution
    diff = np.abs(Vp[:, free] - Vr[:, free]).max(axis=1)
    assert diff.max() <= 1e-4 * max(1.0, np.abs(Vr[:, free]).max()), diff
    np.testing.assert_allclose(Vp[:, lay.u(0)], Vr[:, lay.u(0)], atol=1e-4)


@pytest.mark.gpu
def test_converged_mpc_closed_loop(gpu):
    from awebox_amd.mpc_solve import BatchedPmpc
    c = k3.build_constants()
    pm = BatchedPmpc(c, 8, device="cuda")
    pm.start()
    for _ in range(3):
        out = pm.step()
        assert all(s == "solve_succeeded" for s in out["status"]), out["status"]
        assert float(out["plant_residual"].max()) < 1e-10
        assert torch.isfinite(out["x0"]).all()
    assert out["iterations"].max() < 60
