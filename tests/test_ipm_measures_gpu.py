"""The interior-point measures kernel (libawelu awelu_ipm_measures, ipm_measures.Measures) on MI355X:
bitwise the torch composition it replaces (ipm_measures.Measures.errors_torch / barrier_phi_torch,
the solver's CPU path), on random instances with infinite bounds, one-sided bounds, inequality rows,
a NaN and an infinity in the constraint values, without inequality rows and without constraints;
and batch-invariant (an instance alone gives the bits it gets inside the batch)."""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.build import LIB_LU, build_one
    build_one(LIB_LU)


def _case(seed, B, n, mI, m, nnz, poison=False):
    from awebox_amd.ipm import _GatherMv
    rng = np.random.default_rng(seed)
    ny = n + mI
    dev = torch.device("cuda")
    t = lambda a: torch.tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    yl0 = rng.normal(size=ny) * 3 - 5
    yu0 = yl0 + rng.uniform(0.5, 10, size=ny)
    kind = rng.integers(0, 4, size=ny)             # 0 both, 1 lower only, 2 upper only, 3 free
    yl0[kind >= 2] = -np.inf
    yu0[(kind == 1) | (kind == 3)] = np.inf
    ineq = np.sort(rng.choice(m, size=mI, replace=False)) if m else np.zeros(0, dtype=np.int64)
    yl, yu = np.tile(yl0, (B, 1)), np.tile(yu0, (B, 1))
    c_scale = rng.uniform(0.01, 1.0, size=(B, m))
    nlp = types.SimpleNamespace(
        yl=t(yl), yu=t(yu), yl0=yl0, yu0=yu0, ineq_t=torch.tensor(ineq, dtype=torch.int64, device=dev),
        c_scale=t(c_scale), obj_scale=t(rng.uniform(0.1, 1.0, size=B)))
    nlp.has_l = torch.isfinite(nlp.yl)
    nlp.has_u = torch.isfinite(nlp.yu)
    lo = np.where(np.isfinite(yl0), yl0, yu0 - 20.0)
    hi = np.where(np.isfinite(yu0), yu0, yl0 + 20.0)
    lo = np.where(np.isfinite(lo), lo, -10.0)
    hi = np.where(np.isfinite(hi), hi, 10.0)
    y = lo + rng.uniform(0.01, 0.99, size=(B, ny)) * (hi - lo)
    rows = rng.integers(0, n, size=nnz) if n else np.zeros(0, dtype=np.int64)
    cols = rng.integers(0, m, size=nnz) if m else np.zeros(0, dtype=np.int64)
    jt_op = _GatherMv(rows, cols, (ny, m), dev)
    spread = lambda shape: t(rng.normal(size=shape) * np.exp(rng.uniform(-8, 8, size=shape)))  # noqa: E731
    d = dict(grad=spread((B, n)), jv=spread((B, nnz)), c=spread((B, m)), y=t(y), lam=spread((B, m)),
             zl=t(np.abs(rng.normal(size=(B, ny)))) * nlp.has_l, zu=t(np.abs(rng.normal(size=(B, ny)))) * nlp.has_u,
             f=spread((B,)), mu=t(10.0 ** rng.uniform(-9, -1, size=B)))
    if poison and m > 1:
        d["c"][1, 3] = float("nan")
        d["c"][2, 0] = float("inf")
    opts = types.SimpleNamespace(mu_target=0.0, kappa_d=1e-5, s_max=100.0)
    return nlp, jt_op, d, opts


def _same(a, b):
    """Bitwise equal, NaN where the other is NaN."""
    a, b = a.cpu(), b.cpu()
    nan = torch.isnan(a)
    return torch.equal(nan, torch.isnan(b)) and torch.equal(a[~nan], b[~nan])


@pytest.mark.parametrize("B,n,mI,m,nnz,poison", [(5, 300, 40, 250, 2000, False), (4, 1000, 0, 600, 5000, True),
                                                 (3, 20, 0, 0, 0, False), (6, 2900, 120, 2600, 20000, True),
                                                 (2, 1, 1, 1, 3, False)])
def test_measures_kernel_is_the_torch_composition(B, n, mI, m, nnz, poison):
    _need_gpu()
    from awebox_amd.ipm_measures import Measures
    nlp, jt_op, d, opts = _case(B * 1000 + n, B, n, mI, m, nnz, poison)
    meas = Measures(nlp, opts, jt_op, torch.device("cuda"), n, mI, m, B)
    assert meas.fused
    args = (d["grad"], d["jv"], d["c"], d["y"], d["lam"], d["zl"], d["zu"], d["f"], d["mu"])
    got_head = meas.head(*args)
    got_merit = meas.merit(d["c"], d["f"], d["y"], d["mu"])
    meas.fused = False
    ref_head = meas.head(*args)
    ref_merit = meas.merit(d["c"], d["f"], d["y"], d["mu"])
    for r in range(ref_head.shape[0]):
        assert _same(got_head[r], ref_head[r]), (r, got_head[r], ref_head[r])
    assert _same(got_merit, ref_merit), (got_merit, ref_merit)
    # an instance alone: the same bits (one workgroup per instance, nothing depends on B)
    meas.fused = True
    b = B - 1
    nlp1 = types.SimpleNamespace(**{k: (v[b:b + 1] if torch.is_tensor(v) and v.dim() == 2 and v.shape[0] == B else v)
                                    for k, v in vars(nlp).items()})
    nlp1.obj_scale = nlp.obj_scale[b:b + 1]
    one = Measures(nlp1, opts, jt_op, torch.device("cuda"), n, mI, m, 1)
    h1 = one.head(*(a[b:b + 1] for a in args))
    assert _same(h1[:, 0], got_head[:, b])


@pytest.mark.parametrize("B,n,mI,m,nnz,poison", [(5, 300, 40, 250, 2000, False), (4, 1000, 0, 600, 5000, True),
                                                 (6, 2900, 120, 2600, 20000, True), (2, 1, 1, 1, 3, False)])
def test_newton_and_step_kernels_are_the_torch_composition(B, n, mI, m, nnz, poison):
    """awelu_ipm_newton (gaps, Sigma, grad phi, right-hand side) and awelu_ipm_step (accepted step,
    alpha_z, kappa_sigma safeguard; stepped and not stepped instances, no instance stepped) bitwise
    their torch compositions."""
    _need_gpu()
    from awebox_amd.ipm_measures import Measures
    nlp, jt_op, d, opts = _case(B * 7 + n, B, n, mI, m, nnz, poison)
    opts.kappa_sigma = 1e10
    dev = torch.device("cuda")
    meas = Measures(nlp, opts, jt_op, dev, n, mI, m, B)
    args = (d["grad"], d["jv"], d["c"], d["y"], d["lam"], d["zl"], d["zu"], d["mu"])
    got = meas.newton(*args)
    meas.fused = False
    ref = meas.newton(*args)
    for name, a, b in zip(("dl", "du", "sigma", "grad_phi", "rhs"), got, ref):
        assert _same(a, b), name
    dl, du = ref[0], ref[1]
    rng = np.random.default_rng(B + n)
    ny = n + mI
    t = lambda a: torch.tensor(a, dtype=torch.float64, device=dev)  # noqa: E731
    dy = t(rng.normal(size=(B, ny)) * 0.01)
    y_new = d["y"] + 0.5 * dy
    dlam = t(rng.normal(size=(B, m)))
    tau = t(np.full(B, 0.99))
    alpha = rng.uniform(0.1, 1.0, size=B)
    if poison:
        dlam[0, 0] = float("inf")          # an instance that does not step: lam + 0 * inf
    for acc in (np.arange(B) % 2 == 1, np.ones(B, dtype=bool), np.zeros(B, dtype=bool)):
        meas.fused = True
        g = meas.step(acc, d["y"], y_new, dy, d["lam"], dlam, d["zl"], d["zu"], dl, du, d["mu"], tau, alpha)
        meas.fused = False
        r = meas.step(acc, d["y"], y_new, dy, d["lam"], dlam, d["zl"], d["zu"], dl, du, d["mu"], tau, alpha)
        for name, a, b in zip(("y", "lam", "zl", "zu", "alpha_z"), g, r):
            assert _same(a, b), (name, acc)
