"""Parity of the HIP evaluator (through the C ABI) with the CPU oracle, on an MI355X.

Tolerances (fp64; the two implementations differ only in evaluation order -- the oracle
differentiates the Lagrangian automatically, the kernel evaluates hand-derived expressions):
  g, grad f : |a - b| <= 1e-9 |b| + 1e-11 * max|b|
  J_g       : |a - b| <= 1e-9 |b| + 1e-11 * max|column of b|  (values compared on the union pattern)
  f         : relative 1e-12
"""
import numpy as np
import pytest
import scipy.sparse as sp

from awebox_amd import problem as pb
from awebox_amd.initial_guess import batch_member, initial_guess

pytestmark = pytest.mark.gpu

RTOL, ATOL_REL = 1e-9, 1e-11


def _close(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    tol = RTOL * np.abs(b) + ATOL_REL * max(np.abs(b).max(), 1e-300)
    bad = np.abs(a - b) > tol
    assert not bad.any(), f"{what}: {bad.sum()} entries off, worst {np.abs(a - b)[bad].max():.3e} at {np.argmax(np.abs(a - b) - tol)}"


def _close_jac(Jk, Jo, what="J_g"):
    Jk, Jo = sp.csc_matrix(Jk), sp.csc_matrix(Jo)
    D = (Jk - Jo).tocsc()
    colmax = np.maximum(abs(Jo).max(axis=0).toarray().ravel(), 1e-300)
    D.data = np.abs(D.data)
    Jo_on_D = abs(Jo).tocsc()
    worst = 0.0
    for c in range(D.shape[1]):
        s, e = D.indptr[c], D.indptr[c + 1]
        if s == e:
            continue
        rows = D.indices[s:e]
        ref = np.asarray(Jo_on_D[rows, c].todense()).ravel()
        tol = RTOL * ref + ATOL_REL * colmax[c]
        excess = D.data[s:e] - tol
        worst = max(worst, excess.max())
        assert (excess <= 0).all(), f"{what}: column {c} rows {rows[excess > 0]} off by {D.data[s:e][excess > 0]}"


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.build import build
    build()
    return torch


def _setup(n_k=40, d=4):
    from oracle.ap2_oracle import from_problem
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    return consts, lay, v0, from_problem(consts, n_k=n_k, d=d)


def _oracle_all(orc, lay, V, P):
    g = orc.nlp_g(V, P, lay, pb.THETA0_OFF).numpy()
    f = float(orc.nlp_f(V, P, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES))
    grad = orc.nlp_grad_f(V, P, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES).numpy()
    J = orc.nlp_jac_g(V, P, lay, pb.THETA0_OFF)
    return f, g, grad, J


@pytest.mark.parametrize("n_k,d,member,path", [(40, 4, None, None), (40, 4, 0, None), (40, 4, 7, None),
                                                (5, 3, 1, None), (3, 2, 2, None), (40, 4, 7, "soa"),
                                                (5, 3, 1, "soa"), (3, 2, 2, "soa"), (40, 4, 7, "generated")])
def test_nlp_eval_matches_oracle(gpu, n_k, d, member, path):
    """One instance on the default path (the colour kernel at batch 1) and on the instance-minor and
    node + gather paths."""
    from awebox_amd.evaluator import Ap2Evaluator
    consts, lay, v0, orc = _setup(n_k, d)
    V = v0 if member is None else batch_member(v0, lay, member)
    P = pb.pack_p(lay, consts, v0)
    ev = Ap2Evaluator(consts, batch=1)
    if path is not None:
        ev.path = path
    out = ev.eval_nlp(V, P)
    f, g, grad, J = _oracle_all(orc, lay, V, P)
    _close(out["g"][0], g, "g")
    assert out["f"][0] == pytest.approx(f, rel=1e-12)
    _close(out["grad_f"][0], grad, "grad_f")
    _close_jac(ev.jac_csc(out["jac"][0]), J)


@pytest.mark.parametrize("B,path,members", [(8, None, (0, 3, 7)), (130, None, (0, 77, 129)),
                                             (8, "generated", (0, 7))])
def test_batched_sweep_members_match_oracle(gpu, B, path, members):
    """B instances per launch with different V and different u_ref (the sweep parameter): 8 on the
    default (colour) path and on the node + gather path, 130 on the default instance-minor path
    (two full blocks of 64 instances and a partial one)."""
    from awebox_amd.evaluator import Ap2Evaluator
    consts, lay, v0, orc = _setup()
    u_refs = np.linspace(5, 8, B)                      # dual_kites_power_curve sweep range
    Vs = np.stack([batch_member(v0, lay, b) for b in range(B)])
    Ps = np.stack([pb.pack_p(lay, consts, v0, u_ref=u) for u in u_refs])
    ev = Ap2Evaluator(consts, batch=B)
    assert ev.path == ("soa" if B >= 128 else "colour")
    if path is not None:
        ev.path = path
    out = ev.eval_nlp(Vs, Ps)
    for b in members:
        f, g, grad, J = _oracle_all(orc, lay, Vs[b], Ps[b])
        _close(out["g"][b], g, f"g[{b}]")
        assert out["f"][b] == pytest.approx(f, rel=1e-12)
        _close(out["grad_f"][b], grad, f"grad_f[{b}]")
        _close_jac(ev.jac_csc(out["jac"][b]), J, f"J[{b}]")


def test_device_path_value_kernels_and_determinism(gpu):
    torch = gpu
    from awebox_amd.evaluator import Ap2Evaluator
    consts, lay, v0, _ = _setup()
    B = 4
    ev = Ap2Evaluator(consts, batch=B)
    V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device="cuda")
    P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0)] * B), device="cuda")
    f = torch.zeros(B, dtype=torch.float64, device="cuda")
    g = torch.zeros(B, ev.n_g, dtype=torch.float64, device="cuda")
    gr = torch.zeros(B, ev.n_v, dtype=torch.float64, device="cuda")
    jac = torch.zeros(B, ev.nnz, dtype=torch.float64, device="cuda")
    ev.eval_nlp_device(V, P, f, g, gr, jac)
    f1, g1, gr1, j1 = f.clone(), g.clone(), gr.clone(), jac.clone()
    ev.eval_nlp_device(V, P, f, g, gr, jac)
    torch.cuda.synchronize()
    assert torch.equal(f, f1) and torch.equal(g, g1) and torch.equal(gr, gr1) and torch.equal(jac, j1)
    g2 = torch.zeros_like(g)
    f2 = torch.zeros_like(f)
    ev.eval_g_device(V, P, g2)
    ev.eval_f_device(V, P, f2)
    torch.cuda.synchronize()
    # the value-only kernel: the same model in plain double, objective summed in another order
    assert torch.allclose(g2, g1, rtol=1e-12, atol=1e-12 * float(g1.abs().max()))
    assert torch.allclose(f2, f1, rtol=1e-12, atol=0.0)
    g3 = torch.zeros_like(g)
    ev.eval_g_device(V, P, g3)
    torch.cuda.synchronize()
    assert torch.equal(g3, g2)                          # deterministic
    # host round trip (CasADi's nlp_f / nlp_g through the bridge)
    gh = ev.eval_g(V.cpu().numpy(), P.cpu().numpy())
    fh = ev.eval_f(V.cpu().numpy(), P.cpu().numpy())
    assert np.array_equal(gh, g2.cpu().numpy()) and np.array_equal(fh, f2.cpu().numpy())
    ms_main, ms_fin = ev.last_kernel_ms()
    assert ms_main > 0 and ms_fin > 0


def test_nonfinite_is_an_evaluation_error(gpu):
    from awebox_amd.evaluator import Ap2Evaluator, AwegpuError
    consts, lay, v0, _ = _setup()
    V = v0.copy()
    V[lay.x(3)[0:3]] = 0.0                              # |q| = 0 -> division by zero
    ev = Ap2Evaluator(consts, batch=1)
    with pytest.raises(AwegpuError, match="non-finite"):
        ev.eval_nlp(V, pb.pack_p(lay, consts, v0))


def _close_hess(Hk, Ho, what="H"):
    """Full symmetric matrices.  Entries outside the kernel pattern must be rounding-level zeros
    (t_f cancels analytically in the power cost; the oracle keeps 1e-16-level residues)."""
    Hk, Ho = sp.csc_matrix(Hk), sp.csc_matrix(Ho)
    scale = max(abs(Ho).max(), 1e-300)
    D = abs(Hk - Ho).tocoo()
    ref = np.asarray(abs(Ho)[D.row, D.col]).ravel()
    tol = RTOL * ref + ATOL_REL * scale
    bad = D.data > tol
    assert not bad.any(), f"{what}: {bad.sum()} entries off, worst {D.data[bad].max():.3e}"


@pytest.mark.parametrize("n_k,d,member,hess", [(40, 4, 3, "hyperdual"), (5, 3, 1, "hyperdual"),
                                                (3, 2, 2, "hyperdual"), (40, 4, 3, "generated"),
                                                (5, 3, 1, "generated"), (3, 2, 2, "generated"),
                                                (4, 5, 0, "generated")])
def test_hessian_matches_oracle(gpu, n_k, d, member, hess):
    """nlp_hess_l of one instance on both Hessian kernels: the hyper-dual colour-pair kernel and the
    generated forward-over-reverse node code + assembly kernel."""
    from awebox_amd.evaluator import Ap2Evaluator
    consts, lay, v0, orc = _setup(n_k, d)
    V = batch_member(v0, lay, member)
    P = pb.pack_p(lay, consts, v0, u_ref=7.0)
    lam = np.random.default_rng(7).standard_normal(lay.n_g)       # sigma 1, lam ~ N(0,1)
    ev = Ap2Evaluator(consts, batch=1)
    ev.hess_path = hess
    assert ev.hess_path == hess
    H = ev.hess_csc(ev.eval_hess(V, P, 1.0, lam)[0])
    Ho = orc.nlp_hess_l(V, P, 1.0, lam, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES)
    _close_hess(H, Ho)


def test_hessian_batch_sigma_lambda_and_determinism(gpu):
    torch = gpu
    from awebox_amd.evaluator import Ap2Evaluator
    consts, lay, v0, orc = _setup(5, 3)
    B = 3
    Vs = np.stack([batch_member(v0, lay, b) for b in range(B)])
    Ps = np.stack([pb.pack_p(lay, consts, v0, u_ref=u) for u in (5.0, 6.0, 8.0)])
    sig = np.array([1.0, 0.0, 2.5])
    lams = np.random.default_rng(11).standard_normal((B, lay.n_g))
    ev = Ap2Evaluator(consts, batch=B)
    Hh = ev.eval_hess(Vs, Ps, sig, lams)
    for b in range(B):
        Ho = orc.nlp_hess_l(Vs[b], Ps[b], sig[b], lams[b], lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES)
        _close_hess(ev.hess_csc(Hh[b]), Ho, f"H[{b}]")
    dev = lambda a: torch.tensor(a, device="cuda")
    Hd = torch.zeros(B, ev.nnz_h, dtype=torch.float64, device="cuda")
    ev.eval_hess_device(dev(Vs), dev(Ps), dev(sig), dev(lams), Hd)
    torch.cuda.synchronize()
    assert np.array_equal(Hd.cpu().numpy(), Hh)
    assert ev.last_hess_ms() > 0


def test_generated_hessian_batch_matches_hyperdual_and_oracle(gpu):
    """130 instances (two full blocks of 64 and a partial one) with different V, u_ref, sigma and
    multipliers: the generated Hessian against the hyper-dual kernel for every instance and the oracle
    for three; the instance-minor output (awe_eval_hess_im) equals the per-instance one bitwise, and
    repeats bitwise."""
    torch = gpu
    from awebox_amd.evaluator import Ap2Evaluator
    consts, lay, v0, orc = _setup()
    B = 130
    rng = np.random.default_rng(5)
    Vs = np.stack([batch_member(v0, lay, b) for b in range(B)])
    Ps = np.stack([pb.pack_p(lay, consts, v0, u_ref=u) for u in np.linspace(5, 8, B)])
    sig = rng.uniform(0.0, 2.0, B)
    lams = rng.standard_normal((B, lay.n_g))
    ev = Ap2Evaluator(consts, batch=B)
    assert ev.hess_path == "generated"                 # follows the instance-minor evaluation path
    Hg = ev.eval_hess(Vs, Ps, sig, lams)
    ev.hess_path = "hyperdual"
    Hh = ev.eval_hess(Vs, Ps, sig, lams)
    scale = np.abs(Hh).max(axis=1, keepdims=True)
    assert np.all(np.abs(Hg - Hh) <= RTOL * np.abs(Hh) + ATOL_REL * scale)
    for b in (0, 64, 129):
        Ho = orc.nlp_hess_l(Vs[b], Ps[b], sig[b], lams[b], lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES)
        _close_hess(ev.hess_csc(Hg[b]), Ho, f"H[{b}]")
    ev.hess_path = "generated"
    dev = lambda a: torch.tensor(a, device="cuda")
    Him = ev.alloc_hess()
    args = (dev(Vs), dev(Ps), dev(sig), dev(lams))
    ev.eval_hess_device_im(*args, Him)
    H1 = Him.clone()
    ev.eval_hess_device_im(*args, Him)
    torch.cuda.synchronize()
    assert torch.equal(Him, H1)
    assert np.array_equal(Him.cpu().numpy(), Hg)
    assert ev.last_hess_ms() > 0
