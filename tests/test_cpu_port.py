"""The evaluator's algorithm (colouring, gather list, objective pass), run on the CPU through the
CPU port, against the independent oracle.  Same tolerances as the GPU parity tests."""
import numpy as np
import pytest

from awebox_amd import problem as pb
from awebox_amd.initial_guess import batch_member, initial_guess

from test_gpu_parity import _close, _close_jac, _oracle_all


@pytest.mark.parametrize("n_k,d,member", [(5, 3, None), (5, 3, 1), (3, 2, 2), (4, 4, 3), (2, 5, 0), (3, 1, 4)])
def test_cpu_port_matches_oracle(n_k, d, member):
    from oracle.ap2_oracle import from_problem
    from oracle.cpu_port import CpuPort
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    V = v0 if member is None else batch_member(v0, lay, member)
    P = pb.pack_p(lay, consts, v0, u_ref=7.0 if member else None)
    port = CpuPort(consts)
    out = port.eval_nlp(V, P)
    f, g, grad, J = _oracle_all(from_problem(consts, n_k=n_k, d=d), lay, V, P)
    _close(out["g"][0], g, "g")
    assert out["f"][0] == pytest.approx(f, rel=1e-12)
    _close(out["grad_f"][0], grad, "grad_f")
    _close_jac(port.jac_csc(out["jac"][0]), J)


def test_cpu_port_batch_and_threads_deterministic():
    from oracle.cpu_port import CpuPort
    consts = pb.build_constants()
    lay = pb.NlpLayout()
    v0 = initial_guess(consts, lay)
    V = np.stack([batch_member(v0, lay, b) for b in range(3)])
    P = np.stack([pb.pack_p(lay, consts, v0, u_ref=u) for u in (5.0, 6.5, 8.0)])
    port = CpuPort(consts)
    a = port.eval_nlp(V, P, threads=1)
    b = port.eval_nlp(V, P, threads=4)
    one = port.eval_nlp(V[1], P[1])
    for key in ("f", "g", "grad_f", "jac"):
        assert np.array_equal(a[key], b[key])
        assert np.array_equal(a[key][1], one[key][0])
    assert np.isfinite(a["jac"]).all()


def _close_hess(Hk, Ho, what="H"):
    """Full symmetric matrices; entries outside the kernel pattern must be rounding-level zeros
    (t_f cancels analytically in the power cost; the oracle keeps 1e-16-level residues)."""
    import scipy.sparse as sp
    Hk, Ho = sp.csc_matrix(Hk), sp.csc_matrix(Ho)
    scale = max(abs(Ho).max(), 1e-300)
    D = abs(Hk - Ho).tocoo()
    ref = np.asarray(abs(Ho)[D.row, D.col]).ravel()
    tol = 1e-9 * ref + 1e-11 * scale
    bad = D.data > tol
    assert not bad.any(), f"{what}: {bad.sum()} entries off, worst {D.data[bad].max():.3e}"


@pytest.mark.parametrize("n_k,d,member", [(3, 2, 1), (5, 3, 2), (2, 5, 0), (3, 1, 3)])
def test_cpu_port_hessian_matches_oracle(n_k, d, member):
    from oracle.ap2_oracle import from_problem
    from oracle.cpu_port import CpuPort
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    V = batch_member(v0, lay, member)
    P = pb.pack_p(lay, consts, v0, u_ref=6.0)
    lam = np.random.default_rng(7).standard_normal(lay.n_g)
    sigma = 0.7
    port = CpuPort(consts)
    Hk = port.hess_csc(port.eval_hess(V, P, sigma, lam)[0])
    Ho = from_problem(consts, n_k=n_k, d=d).nlp_hess_l(V, P, sigma, lam, lay, pb.THETA0_OFF, pb.COST_NAMES,
                                                        pb.PHI_NAMES)
    _close_hess(Hk, Ho)
