"""3-DOF tracking-MPC NLP.

CPU: layout sizes against the survey's derivation, option-derived constants, the C-ABI library's
exports and CPU-side sparsity (a superset of the oracle's non-zeros), restated geometric properties
of the 3-DOF force model (three_dof_kite.py:98-199) and of the tracking cost (pmpc.py:304-358).
GPU (MI355X, through the C ABI): f, g, grad f and J_g against the oracle.

Tolerances (fp64; the two sides differ only in evaluation order):
  g, grad f : |a - b| <= 1e-9 |b| + 1e-11 max|b|;  J_g per column likewise;  f relative 1e-12.
"""
import math
import os
import re
import subprocess

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from awebox_amd import kite3 as k3
from awebox_amd.build import LIB_MPC, build

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "awempc.h")
RTOL, ATOL_REL = 1e-9, 1e-11


def _setup(n_k=20, d=4):
    from oracle.kite3_oracle import from_constants
    c = k3.build_constants(k3.Kite3Config(n_k=n_k, d=d))
    lay = k3.MpcLayout(n_k, d)
    return c, lay, from_constants(c, lay)


def test_layout_sizes_match_survey():
    lay = k3.MpcLayout(20, 4)
    assert (lay.n_v, lay.n_g) == (1562, 1471)
    assert lay.n_p == 11 + lay.n_v + 1 + 11 + 6 + 11
    assert k3.NW == 31 and (k3.N_EQ, k3.N_INEQ) == (12, 2)
    assert len(k3.EQ_NAMES) == k3.N_EQ


def test_scaling_constants():
    c = k3.build_constants()
    s = dict(zip([f"{vt}.{n}.{i}" for vt, ents in k3.VAR_TYPES for n, sz in ents for i in range(sz)], c.scaling))
    assert math.isclose(s["x.q10.0"], 20.0 ** 2 / (12 * 9.81))          # centripetal radius
    assert s["x.dq10.1"] == 20.0 and s["x.l_t.0"] == 500.0
    assert s["x.ddl_t.0"] == 50.0 and s["u.dddl_t.0"] == 50.0 and s["xdot.dddl_t.0"] == 50.0
    assert s["xdot.ddq10.2"] == s["x.dq10.2"] and s["xdot.dcoeff10.1"] == s["x.coeff10.1"]
    assert math.isclose(s["x.coeff10.1"], 80 * math.pi / 180)
    assert math.isclose(s["z.lambda10.0"], (1.0 + 2000.0) / 2 / 500.0)
    # log wind at the estimated altitude l_t sin(40 deg)
    zz = 500 * math.sin(40 * math.pi / 180)
    u_alt = 5.0 * math.log10(math.sqrt(zz ** 2 + 1) / 0.1) / math.log10(10 / 0.1)
    assert math.isclose(s["x.dl_t.0"], u_alt / 3)


@pytest.fixture(scope="module")
def lib():
    build()
    from awebox_amd.mpc import load_library
    return load_library()


def test_exports_every_header_symbol(lib):
    from awebox_amd.mpc import EXPORTED_SYMBOLS
    declared = set(re.findall(r"^(?:int|const char\*)\s+(awempc_\w+)\(", open(HEADER).read(), re.M))
    assert declared == set(EXPORTED_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_MPC], capture_output=True, text=True, check=True).stdout
    assert declared <= set(re.findall(r"\bT (awempc_\w+)", out))


@pytest.mark.parametrize("n_k,d", [(20, 4), (3, 2), (5, 3)])
def test_static_sparsity_covers_oracle(lib, n_k, d):
    from awebox_amd.mpc import sparsity_jac_static
    c, lay, orc = _setup(n_k, d)
    colind, row = sparsity_jac_static(c)
    assert colind.size == lay.n_v + 1 and colind[-1] == row.size
    for col in range(lay.n_v):
        assert np.all(np.diff(row[colind[col]:colind[col + 1]]) > 0)
    V, p = k3.batch_instance(c, lay, 3, 16)
    J = orc.nlp_jac_g(V, p, lay)
    pat = sp.csc_matrix((np.ones(row.size), row, colind), shape=(lay.n_g, lay.n_v))
    nz = (J != 0).astype(float)
    assert (nz - nz.multiply(pat)).nnz == 0


def test_three_dof_force_geometry():
    """three_dof_kite.py:98-199: lift along the rolled normal of the (tether, apparent wind) plane,
    perpendicular to the apparent wind; drag along the apparent wind; CD = |CX0| + CL^2/(pi AR)."""
    from oracle.kite3_oracle import IDX
    c, lay, orc = _setup(3, 2)
    rng = np.random.default_rng(5)
    for psi in (0.0, 0.3, -0.7):
        w = torch.zeros(k3.NW)
        w[IDX[("x", "q10")]] = torch.tensor([300.0, 40.0, 250.0])
        w[IDX[("x", "dq10")]] = torch.as_tensor(rng.standard_normal(3) * 10)
        CL = 0.9
        w[IDX[("x", "coeff10")]] = torch.tensor([CL, psi])
        u_ref = 6.0
        F = orc.aero(w, u_ref)
        q, dq = w[IDX[("x", "q10")]], w[IDX[("x", "dq10")]]
        ua = orc.wind_velocity(q[2], u_ref) - dq
        rho = orc.density(q[2])
        CD = orc.c["cd0"] + CL ** 2 / (math.pi * orc.c["ar"])
        drag = CD * 0.5 * rho * torch.linalg.norm(ua) * orc.c["s_ref"] * ua
        lift = F - drag
        assert abs(float(torch.dot(lift, ua))) < 1e-9 * float(torch.linalg.norm(lift) * torch.linalg.norm(ua))
        assert math.isclose(float(torch.linalg.norm(lift)),
                            CL * 0.5 * float(rho) * float(torch.dot(ua, ua)) * orc.c["s_ref"], rel_tol=1e-12)
        # roll: the lift leaves the (tether, wind) plane by psi, towards -(q x u)
        nplane = torch.linalg.cross(q, ua)
        sin_roll = float(torch.dot(lift, nplane) / (torch.linalg.norm(lift) * torch.linalg.norm(nplane)))
        assert math.isclose(sin_roll, -math.sin(psi), abs_tol=1e-12)


def test_tracking_cost_gradient_closed_form():
    c, lay, orc = _setup(3, 2)
    V, p = k3.batch_instance(c, lay, 1, 4)
    rng = np.random.default_rng(3)
    p[lay.p_Q:lay.p_Q + k3.NX] = rng.uniform(0.5, 2, k3.NX)
    p[lay.p_R:lay.p_R + k3.NU] = rng.uniform(0.5, 2, k3.NU)
    p[lay.p_P:lay.p_P + k3.NX] = rng.uniform(0.5, 2, k3.NX)
    g = orc.nlp_grad_f(V, p, lay).numpy()
    ref = p[lay.p_ref:lay.p_ref + lay.n_v]
    w = orc.w
    exp = np.zeros(lay.n_v)
    Q, R, P = p[lay.p_Q:lay.p_Q + 11], p[lay.p_R:lay.p_R + 6], p[lay.p_P:lay.p_P + 11]
    for k in range(lay.n_k):
        for j in range(lay.d):
            exp[lay.coll_x(k, j)] = 2 * w[j] * Q * (V[lay.coll_x(k, j)] - ref[lay.coll_x(k, j)]) / lay.n_k
            exp[lay.coll_z(k, j)] = 2 * w[j] * (V[lay.coll_z(k, j)] - ref[lay.coll_z(k, j)]) / lay.n_k
        exp[lay.u(k)] = 2 * w.sum() * R * (V[lay.u(k)] - ref[lay.u(k)]) / lay.n_k
    exp[lay.x(lay.n_k)] = 2 * P * (V[lay.x(lay.n_k)] - ref[lay.x(lay.n_k)])
    assert np.allclose(g, exp, rtol=1e-13, atol=1e-15)


def test_initial_rows_are_exact():
    c, lay, orc = _setup(3, 2)
    V, p = k3.batch_instance(c, lay, 0, 4)
    g = orc.nlp_g(V, p, lay).numpy()
    assert np.array_equal(g[lay.g_init()], V[lay.x(0)] - p[lay.p_x0:lay.p_x0 + 11])
    p2 = p.copy()
    p2[lay.p_x0:lay.p_x0 + 11] = V[lay.x(0)]
    assert np.all(orc.nlp_g(V, p2, lay).numpy()[lay.g_init()] == 0)


# ------------------------------------------------------------------------------------ GPU
def _close(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    tol = RTOL * np.abs(b) + ATOL_REL * max(np.abs(b).max(), 1e-300)
    bad = np.abs(a - b) > tol
    assert not bad.any(), f"{what}: {bad.sum()} off, worst {np.abs(a - b)[bad].max():.3e}"


def _close_jac(Jk, Jo):
    D = (sp.csc_matrix(Jk) - sp.csc_matrix(Jo)).tocsc()
    colmax = np.maximum(abs(Jo).max(axis=0).toarray().ravel(), 1e-300)
    Jo = abs(sp.csc_matrix(Jo)).tocsc()
    for col in range(D.shape[1]):
        s, e = D.indptr[col], D.indptr[col + 1]
        if s == e:
            continue
        rows = D.indices[s:e]
        ref = np.asarray(Jo[rows, col].todense()).ravel()
        excess = np.abs(D.data[s:e]) - (RTOL * ref + ATOL_REL * colmax[col])
        assert (excess <= 0).all(), f"J_g column {col}: rows {rows[excess > 0]}"


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    build()
    return torch


@pytest.mark.gpu
@pytest.mark.parametrize("n_k,d,batch", [(20, 4, 8), (3, 2, 3), (5, 3, 4)])
def test_mpc_eval_matches_oracle(gpu, n_k, d, batch):
    from awebox_amd.mpc import MpcEvaluator
    c, lay, orc = _setup(n_k, d)
    inst = [k3.batch_instance(c, lay, i * 37, 256) for i in range(batch)]
    V = np.stack([v for v, _ in inst])
    P = np.stack([p for _, p in inst])
    P[:, lay.p_u_ref] = np.linspace(4.0, 8.0, batch)           # sweep axis
    rng = np.random.default_rng(11)
    P[:, lay.p_Q:lay.p_Q + 11] = rng.uniform(0.5, 2.0, (batch, 11))
    ev = MpcEvaluator(c, batch=batch)
    out = ev.eval_nlp(V, P)
    for b in range(batch):
        _close(out["g"][b], orc.nlp_g(V[b], P[b], lay).numpy(), f"g[{b}]")
        f = float(orc.nlp_f(V[b], P[b], lay))
        assert abs(out["f"][b] - f) <= 1e-12 * abs(f)
        _close(out["grad_f"][b], orc.nlp_grad_f(V[b], P[b], lay).numpy(), f"grad_f[{b}]")
        _close_jac(ev.jac_csc(out["jac"][b]), orc.nlp_jac_g(V[b], P[b], lay))


@pytest.mark.gpu
def test_mpc_batch256_device_path_deterministic(gpu):
    from awebox_amd.mpc import MpcEvaluator
    c, lay, orc = _setup(20, 4)
    B = 256
    inst = [k3.batch_instance(c, lay, i, B) for i in range(B)]
    dev = torch.device("cuda", 0)
    V = torch.tensor(np.stack([v for v, _ in inst]), device=dev)
    P = torch.tensor(np.stack([p for _, p in inst]), device=dev)
    ev = MpcEvaluator(c, batch=B)
    outs = []
    for _ in range(2):
        f = torch.empty(B, dtype=torch.float64, device=dev)
        g = torch.empty(B, ev.n_g, dtype=torch.float64, device=dev)
        gr = torch.empty(B, ev.n_v, dtype=torch.float64, device=dev)
        jac = torch.empty(B, ev.nnz, dtype=torch.float64, device=dev)
        ev.eval_nlp_device(V, P, f, g, gr, jac)
        torch.cuda.synchronize()
        outs.append([t.cpu().numpy() for t in (f, g, gr, jac)])
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    f, g, gr, jac = outs[0]
    assert np.isfinite(jac).all() and np.isfinite(g).all()
    b = 201
    _close(g[b], orc.nlp_g(inst[b][0], inst[b][1], lay).numpy(), "g[201]")
    _close_jac(ev.jac_csc(jac[b]), orc.nlp_jac_g(inst[b][0], inst[b][1], lay))


@pytest.mark.gpu
@pytest.mark.parametrize("n_k,d,batch", [(20, 4, 130), (3, 2, 70), (5, 3, 65), (4, 5, 3)])
def test_mpc_generated_path_matches_oracle_and_dual_kernel(gpu, n_k, d, batch):
    """awempc_eval_nlp_im (generated node code, instance-minor J_g and grad f; ragged last instance
    block) against the oracle for three instances and against the dual-number kernel for all."""
    from awebox_amd.mpc import MpcEvaluator
    c, lay, orc = _setup(n_k, d)
    inst = [k3.batch_instance(c, lay, i * 13, 64) for i in range(batch)]
    V = np.stack([v for v, _ in inst])
    P = np.stack([p for _, p in inst])
    P[:, lay.p_u_ref] = np.linspace(4.0, 8.0, batch)
    rng = np.random.default_rng(5)
    P[:, lay.p_Q:lay.p_Q + 11] = rng.uniform(0.5, 2.0, (batch, 11))
    ev = MpcEvaluator(c, batch=batch)
    assert ev.generated_available
    dev = torch.device("cuda", 0)
    Vt, Pt = torch.tensor(V, device=dev), torch.tensor(P, device=dev)
    out = {}
    for im in (True, False):
        f = torch.empty(batch, dtype=torch.float64, device=dev)
        g = torch.full((batch, ev.n_g), float("nan"), dtype=torch.float64, device=dev)
        gr, jac = ev.alloc_grad(dev, instance_minor=im), ev.alloc_jac(dev, instance_minor=im)
        gr.fill_(float("nan"))
        jac.fill_(float("nan"))
        ev.eval_nlp_device(Vt, Pt, f, g, gr, jac)
        torch.cuda.synchronize()
        out[im] = [t.cpu().numpy() for t in (f, g, gr, jac)]
    fi, gi, gri, ji = out[True]
    assert np.isfinite(gi).all() and np.isfinite(gri).all() and np.isfinite(ji).all()
    fd, gd, grd, jd = out[False]
    assert np.allclose(fi, fd, rtol=1e-13, atol=0)
    for b in range(batch):
        _close(gi[b], gd[b], f"g[{b}] vs dual")
        _close(gri[b], grd[b], f"grad_f[{b}] vs dual")
        _close(ji[b], jd[b], f"jac[{b}] vs dual")
    for b in sorted({0, batch // 2, batch - 1}):
        _close(gi[b], orc.nlp_g(V[b], P[b], lay).numpy(), f"g[{b}]")
        fo = float(orc.nlp_f(V[b], P[b], lay))
        assert abs(fi[b] - fo) <= 1e-12 * abs(fo)
        _close(gri[b], orc.nlp_grad_f(V[b], P[b], lay).numpy(), f"grad_f[{b}]")
        _close_jac(ev.jac_csc(ji[b]), orc.nlp_jac_g(V[b], P[b], lay))


@pytest.mark.gpu
def test_mpc_nonfinite_is_an_error(gpu):
    from awebox_amd.evaluator import AwegpuError
    from awebox_amd.mpc import MpcEvaluator
    c, lay, _ = _setup(3, 2)
    V, p = k3.batch_instance(c, lay, 0, 4)
    V[lay.x(1)[0]] = np.nan
    ev = MpcEvaluator(c, batch=1)
    with pytest.raises(AwegpuError):
        ev.eval_nlp(V, p)


def test_mpc_p_from_reference_and_p_fun():
    """The MPC boundary: Pmpc's parameter struct read by name (pmpc.py:166-186) packs to the flat p;
    and the constraints depend on p only through the restated P_fun (pmpc.py:641-689): changing
    the tracking reference (except x[N]), Q, R and P leaves g unchanged, the initial-condition rows
    are x[0] - P_fun(p).p.ref.x[0], and u_ref enters through theta0.wind.u_ref."""
    c, lay, orc = _setup(n_k=3, d=2)
    V, p = k3.batch_instance(c, lay, 1, 4)
    named = {("x0",): p[lay.p_x0:lay.p_x0 + k3.NX], ("ref",): p[lay.p_ref:lay.p_ref + lay.n_v],
             ("u_ref",): p[lay.p_u_ref:lay.p_u_ref + 1], ("Q",): p[lay.p_Q:lay.p_Q + k3.NX],
             ("R",): p[lay.p_R:lay.p_R + k3.NU], ("P",): p[lay.p_P:lay.p_P + k3.NX]}
    assert np.array_equal(k3.pack_p_from_reference(named.__getitem__, lay), p)
    with pytest.raises(KeyError):
        k3.pack_p_from_reference({k: v for k, v in named.items() if k != ("Q",)}.__getitem__, lay)
    Pf = k3.p_fun(p, lay)
    assert np.array_equal(Pf[("p", "ref")][lay.x(0)], p[lay.p_x0:lay.p_x0 + k3.NX])
    assert np.count_nonzero(Pf[("p", "ref")]) <= 2 * k3.NX
    g = orc.nlp_g(V, p, lay).numpy()
    np.testing.assert_array_equal(g[lay.g_init()], V[lay.x(0)] - Pf[("p", "ref")][lay.x(0)])
    p2 = p.copy()
    rng = np.random.default_rng(5)
    keep = np.zeros(lay.n_v, dtype=bool)
    keep[lay.x(lay.n_k)] = True
    p2[lay.p_ref:lay.p_ref + lay.n_v] = np.where(keep, p2[lay.p_ref:lay.p_ref + lay.n_v], rng.standard_normal(lay.n_v))
    p2[lay.p_Q:] = rng.uniform(0.5, 2.0, lay.n_p - lay.p_Q)
    for key in Pf:
        np.testing.assert_array_equal(k3.p_fun(p2, lay)[key], Pf[key])
    np.testing.assert_array_equal(orc.nlp_g(V, p2, lay).numpy(), g)
    p3 = p.copy()
    p3[lay.p_u_ref] += 1.0
    assert k3.p_fun(p3, lay)[("theta0", "wind", "u_ref")][0] == p[lay.p_u_ref] + 1.0
    assert not np.allclose(orc.nlp_g(V, p3, lay).numpy(), g)


# ---- nlp_hess_l (exact Hessian of the MPC NLP, pmpc.py:193-217 with IPOPT's default) ------------
def _hess_inputs(c, lay, B=1, seed=3):
    rng = np.random.default_rng(seed)
    Vs, ps = zip(*(k3.batch_instance(c, lay, i, max(B, 4)) for i in range(B)))
    lam = rng.standard_normal((B, lay.n_g))
    sig = 1.0 + rng.random(B)
    return np.stack(Vs), np.stack(ps), sig, lam


def test_hessian_pattern_covers_oracle():
    """The host-derived nlp_hess_l pattern (second-order dependency analysis of kite3_node) is a
    superset of the oracle's structural non-zeros at a generic point (N=3 d=2 and N=4 d=4)."""
    from awebox_amd.mpc import sparsity_hess_static
    for n_k, d in ((3, 2), (4, 4)):
        c, lay, orc = _setup(n_k=n_k, d=d)
        V, p, sig, lam = _hess_inputs(c, lay)
        Ho = orc.nlp_hess_l(V[0], p[0], sig[0], lam[0], lay)
        colind, row = sparsity_hess_static(c)
        pat = sp.csc_matrix((np.ones(len(row)), row, colind), shape=(lay.n_v, lay.n_v)).toarray() > 0
        upper = np.triu(np.abs(Ho) > 0)
        missing = upper & ~pat
        assert not missing.any(), np.argwhere(missing)[:10]
        assert np.all(np.diff(colind) >= 0) and np.all(row <= np.repeat(np.arange(lay.n_v), np.diff(colind)))


@pytest.mark.gpu
@pytest.mark.parametrize("n_k,d,B", [(3, 2, 2), (20, 4, 3)])
def test_hessian_matches_oracle_gpu(n_k, d, B):
    """HIP nlp_hess_l (hyper-dual direction-pair kernel) against the oracle's automatic Hessian:
    per column |a - b| <= 1e-9 |b| + 1e-11 max|b| (fp64, evaluation order only), for B instances
    with different sigma and lambda; bitwise repeatable."""
    from awebox_amd.mpc import MpcEvaluator
    c, lay, orc = _setup(n_k=n_k, d=d)
    V, p, sig, lam = _hess_inputs(c, lay, B=B)
    ev = MpcEvaluator(c, batch=B)
    H = ev.eval_hess(V, p, sig, lam)
    assert np.array_equal(H, ev.eval_hess(V, p, sig, lam))
    for b in range(B):
        Ho = np.triu(orc.nlp_hess_l(V[b], p[b], sig[b], lam[b], lay))
        Hk = ev.hess_csc(H[b], full=False).toarray()
        scale = np.abs(Ho).max()
        err = np.abs(Hk - Ho)
        assert np.all(err <= RTOL * np.abs(Ho) + ATOL_REL * scale), (err.max(), np.unravel_index(err.argmax(), err.shape))
