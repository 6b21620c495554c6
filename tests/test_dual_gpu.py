"""Parity of the dual-kite HIP evaluator (libawedual.so, through the C ABI) with the CPU oracle
(oracle/multikite_oracle.py) on an MI355X -- config 3 (examples/dual_kites_power_curve.py).

Tolerances (fp64; the kernel evaluates hand-derived closed forms in compressed forward mode, the
oracle differentiates the Lagrangian automatically -- they differ only in evaluation order):
  g, grad f : |a - b| <= 1e-9 |b| + 1e-11 max|b|
  J_g       : |a - b| <= 1e-9 |b| + 1e-11 max|column of b|
  f         : relative 1e-12
"""
import numpy as np
import pytest

from awebox_amd import dual as du
from awebox_amd import problem as pb

from test_gpu_parity import _close, _close_jac  # noqa: E402  (tests/ is on sys.path)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.build import LIB_DUAL, build_one
    build_one(LIB_DUAL)
    return torch


def _setup(n_k, d):
    from oracle import multikite_oracle as mo
    mc = du.build_constants(du.MultiConfig(n_k=n_k, d=d))
    lay = du.layout_for(mc)
    V0 = du.initial_guess(mc, lay)
    return mc, lay, V0, mo.from_constants(mc, lay)


def _oracle_all(o, lay, V, P, sparse=False):
    from oracle import multikite_oracle as mo
    th = mo.theta0_dict(P[lay.p_theta0:])
    g = o.nlp_g(V, P, lay, th).numpy()
    f = float(o.nlp_f(V, P, lay, th, pb.COST_NAMES, pb.PHI_NAMES))
    grad = o.nlp_grad_f(V, P, lay, th, pb.COST_NAMES, pb.PHI_NAMES).numpy()
    J = o.nlp_jac_g_sparse(V, P, lay, th) if sparse else o.nlp_jac_g(V, P, lay, th)
    return f, g, grad, J


@pytest.mark.parametrize("n_k,d,member", [(5, 3, 0), (5, 3, 4), (4, 4, 1), (6, 2, 2), (7, 5, 3)])
def test_dual_eval_matches_oracle(gpu, n_k, d, member):
    from awebox_amd.dual_evaluator import DualEvaluator
    mc, lay, V0, o = _setup(n_k, d)
    V = du.batch_member(V0, lay, member)
    P = du.pack_p(lay, mc, V0, "power1")
    ev = DualEvaluator(mc, batch=1)
    out = ev.eval_nlp(V, P)
    f, g, grad, J = _oracle_all(o, lay, V, P)
    assert abs(out["f"][0] - f) <= 1e-12 * max(abs(f), 1e-300)
    _close(out["g"][0], g, "g")
    _close(out["grad_f"][0], grad, "grad_f")
    _close_jac(ev.jac_csc(out["jac"][0]), J)


def test_dual_batch_with_sweep_parameter(gpu):
    """B = 3 instances with different u_ref (the sweep axis) and homotopy steps in one launch."""
    from awebox_amd.dual_evaluator import DualEvaluator
    mc, lay, V0, o = _setup(5, 3)
    Vs = np.stack([du.batch_member(V0, lay, b) for b in range(3)])
    Ps = np.stack([du.pack_p(lay, mc, V0, step, u_ref=u) for step, u in
                   (("power1", 5.0), ("fictitious0", 6.5), ("final0", 8.0))])
    ev = DualEvaluator(mc, batch=3)
    out = ev.eval_nlp(Vs, Ps)
    for b in range(3):
        f, g, grad, J = _oracle_all(o, lay, Vs[b], Ps[b])
        assert abs(out["f"][b] - f) <= 1e-12 * max(abs(f), 1e-300)
        _close(out["g"][b], g, f"g[{b}]")
        _close(out["grad_f"][b], grad, f"grad_f[{b}]")
        _close_jac(ev.jac_csc(out["jac"][b]), J, f"J[{b}]")


def test_dual_full_size_config3(gpu):
    """Config 3 itself: N = 60, d = 4, single_reelout (n_V = 20104, n_g = 20092), one noisy member,
    every output against the oracle (J by per-interval forward-mode blocks)."""
    from awebox_amd.dual_evaluator import DualEvaluator
    mc, lay, V0, o = _setup(60, 4)
    V = du.batch_member(V0, lay, 5)
    P = du.pack_p(lay, mc, V0, "power1")
    ev = DualEvaluator(mc, batch=1)
    assert (ev.n_v, ev.n_g) == (20104, 20092)
    out = ev.eval_nlp(V, P)
    f, g, grad, J = _oracle_all(o, lay, V, P, sparse=True)
    assert abs(out["f"][0] - f) <= 1e-12 * max(abs(f), 1e-300)
    _close(out["g"][0], g, "g")
    _close(out["grad_f"][0], grad, "grad_f")
    _close_jac(ev.jac_csc(out["jac"][0]), J)


def test_dual_device_path_deterministic(gpu):
    torch = gpu
    from awebox_amd.dual_evaluator import DualEvaluator
    mc, lay, V0, _ = _setup(60, 4)
    B = 8
    ev = DualEvaluator(mc, batch=B)
    V = torch.tensor(np.stack([du.batch_member(V0, lay, b) for b in range(B)]), device="cuda")
    P = torch.tensor(np.stack([du.pack_p(lay, mc, V0) for _ in range(B)]), device="cuda")
    outs = []
    for _ in range(2):
        f = torch.empty(B, dtype=torch.float64, device="cuda")
        g = torch.empty(B, ev.n_g, dtype=torch.float64, device="cuda")
        gr = torch.empty(B, ev.n_v, dtype=torch.float64, device="cuda")
        jac = torch.empty(B, ev.nnz, dtype=torch.float64, device="cuda")
        ev.eval_nlp_device(V, P, f, g, gr, jac)
        torch.cuda.synchronize()
        outs.append([t.cpu().numpy() for t in (f, g, gr, jac)])
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
        assert np.isfinite(a).all()
    host = ev.eval_nlp(V.cpu().numpy(), P.cpu().numpy())
    assert np.array_equal(host["jac"], outs[0][3]) and np.array_equal(host["g"], outs[0][1])


def test_dual_nonfinite_is_an_error(gpu):
    from awebox_amd.dual_evaluator import DualEvaluator
    from awebox_amd.evaluator import AwegpuError
    mc, lay, V0, _ = _setup(5, 3)
    V = V0.copy()
    V[lay.x(2)[0]] = np.nan
    ev = DualEvaluator(mc, batch=1)
    with pytest.raises(AwegpuError):
        ev.eval_nlp(V, du.pack_p(lay, mc, V0))


@pytest.mark.parametrize("n_k,batch", [(60, 130), (20, 8), (5, 3)])
def test_dual_generated_path_matches_oracle_and_colour_kernel(gpu, n_k, batch):
    """adl_eval_nlp_im (generated node code, four wavefront roles per node, instance-minor J_g and
    grad f; ragged last instance block at B = 130) against the oracle for three instances and against
    the colour kernel for all, with different u_ref and homotopy steps across the batch."""
    torch = gpu
    from awebox_amd.dual_evaluator import DualEvaluator
    mc, lay, V0, o = _setup(n_k, 4)
    steps = ("power1", "fictitious0", "final0")
    Vs = np.stack([du.batch_member(V0, lay, b) for b in range(batch)])
    Ps = np.stack([du.pack_p(lay, mc, V0, steps[b % 3], u_ref=5.0 + 3.0 * b / max(batch - 1, 1))
                   for b in range(batch)])
    ev = DualEvaluator(mc, batch=batch)
    assert ev.generated_available
    Vt, Pt = torch.tensor(Vs, device="cuda"), torch.tensor(Ps, device="cuda")
    out = {}
    for im in (True, False):
        f = torch.full((batch,), float("nan"), dtype=torch.float64, device="cuda")
        g = torch.full((batch, ev.n_g), float("nan"), dtype=torch.float64, device="cuda")
        gr, jac = ev.alloc_grad("cuda", instance_minor=im), ev.alloc_jac("cuda", instance_minor=im)
        gr.fill_(float("nan"))
        jac.fill_(float("nan"))
        ev.eval_nlp_device(Vt, Pt, f, g, gr, jac)
        torch.cuda.synchronize()
        out[im] = [t.cpu().numpy() for t in (f, g, gr, jac)]
    fi, gi, gri, ji = out[True]
    assert np.isfinite(fi).all() and np.isfinite(gi).all() and np.isfinite(gri).all() and np.isfinite(ji).all()
    fc, gcol, grc, jc = out[False]
    assert np.allclose(fi, fc, rtol=1e-12, atol=0)
    for b in range(batch):
        _close(gi[b], gcol[b], f"g[{b}] vs colour")
        _close(gri[b], grc[b], f"grad_f[{b}] vs colour")
        _close(ji[b], jc[b], f"jac[{b}] vs colour")
    for b in sorted({0, batch // 2, batch - 1}):
        f, g, grad, J = _oracle_all(o, lay, Vs[b], Ps[b], sparse=n_k >= 10)
        assert abs(fi[b] - f) <= 1e-12 * max(abs(f), 1e-300)
        _close(gi[b], g, f"g[{b}]")
        _close(gri[b], grad, f"grad_f[{b}]")
        _close_jac(ev.jac_csc(ji[b]), J, f"J[{b}]")
    # deterministic: a second evaluation repeats every output bitwise
    f2 = torch.empty(batch, dtype=torch.float64, device="cuda")
    g2 = torch.empty(batch, ev.n_g, dtype=torch.float64, device="cuda")
    gr2, jac2 = ev.alloc_grad("cuda", instance_minor=True), ev.alloc_jac("cuda", instance_minor=True)
    ev.eval_nlp_device(Vt, Pt, f2, g2, gr2, jac2)
    torch.cuda.synchronize()
    for a, b in zip(out[True], (f2, g2, gr2, jac2)):
        assert np.array_equal(a, b.cpu().numpy())
