"""The interior-point measures of ipm_measures.Measures on host tensors (the CPU harness's path and
the restatement the fused kernels are checked against on the GPU, tests/test_ipm_measures_gpu.py)
against IPOPT's definitions written independently in numpy: the scaled optimality error
(IpIpoptCalculatedQuantities curr_nlp_error: dual infeasibility and complementarity scaled by s_d,
s_c with s_max = 100), the barrier function with kappa_d damping, the Newton right-hand side, the
bound multipliers' step with its fraction-to-the-boundary length and the kappa_sigma safeguard."""
import types

import numpy as np
import torch


def _case(seed=3, B=3, n=40, mI=6, m=30, nnz=150):
    from awebox_amd.ipm import _GatherMv
    rng = np.random.default_rng(seed)
    ny = n + mI
    yl0 = rng.normal(size=ny) - 3
    yu0 = yl0 + rng.uniform(1, 5, size=ny)
    kind = rng.integers(0, 4, size=ny)
    yl0[kind >= 2] = -np.inf
    yu0[(kind == 1) | (kind == 3)] = np.inf
    ineq = np.sort(rng.choice(m, size=mI, replace=False))
    t = lambda a: torch.tensor(a, dtype=torch.float64)  # noqa: E731
    nlp = types.SimpleNamespace(yl=t(np.tile(yl0, (B, 1))), yu=t(np.tile(yu0, (B, 1))), yl0=yl0, yu0=yu0,
                                ineq_t=torch.tensor(ineq), c_scale=t(rng.uniform(0.1, 1, size=(B, m))),
                                obj_scale=t(rng.uniform(0.2, 1, size=B)))
    nlp.has_l = torch.isfinite(nlp.yl)
    nlp.has_u = torch.isfinite(nlp.yu)
    lo = np.where(np.isfinite(yl0), yl0, np.where(np.isfinite(yu0), yu0 - 10, -5))
    hi = np.where(np.isfinite(yu0), yu0, lo + 10)
    y = lo + rng.uniform(0.05, 0.95, size=(B, ny)) * (hi - lo)
    rows, cols = rng.integers(0, n, size=nnz), rng.integers(0, m, size=nnz)
    jt_op = _GatherMv(rows, cols, (ny, m), "cpu")
    d = dict(grad=t(rng.normal(size=(B, n))), jv=t(rng.normal(size=(B, nnz))), c=t(rng.normal(size=(B, m))), y=t(y),
             lam=t(rng.normal(size=(B, m))), zl=t(rng.uniform(0.1, 2, size=(B, ny))) * nlp.has_l,
             zu=t(rng.uniform(0.1, 2, size=(B, ny))) * nlp.has_u, f=t(rng.normal(size=B)),
             mu=t(10.0 ** rng.uniform(-6, -1, size=B)))
    opts = types.SimpleNamespace(mu_target=0.0, kappa_d=1e-5, s_max=100.0, kappa_sigma=1e10)
    return nlp, jt_op, d, opts, (rows, cols, ineq, yl0, yu0)


def test_measures_host_path_matches_ipopt_definitions():
    from awebox_amd.ipm_measures import Measures
    B, n, mI, m = 3, 40, 6, 30
    nlp, jt_op, d, opts, (rows, cols, ineq, yl0, yu0) = _case(B=B, n=n, mI=mI, m=m)
    meas = Measures(nlp, opts, jt_op, torch.device("cpu"), n, mI, m, B)
    assert not meas.fused
    head = meas.head(d["grad"], d["jv"], d["c"], d["y"], d["lam"], d["zl"], d["zu"], d["f"], d["mu"]).numpy()
    merit = meas.merit(d["c"], d["f"], d["y"], d["mu"]).numpy()
    g = {k: v.numpy() for k, v in d.items()}
    hl, hu = np.isfinite(yl0), np.isfinite(yu0)
    nb = hl.sum() + hu.sum()
    for b in range(B):
        y, zl, zu, lam, c, mu = g["y"][b], g["zl"][b], g["zu"][b], g["lam"][b], g["c"][b], g["mu"][b]
        AtL = np.zeros(n + mI)
        np.add.at(AtL, rows, g["jv"][b] * lam[cols])
        AtL[n:] -= lam[ineq]
        dual = np.concatenate([g["grad"][b], np.zeros(mI)]) + AtL - zl + zu
        dl = np.where(hl, y - nlp.yl[b].numpy(), 1.0)
        du = np.where(hu, nlp.yu[b].numpy() - y, 1.0)
        s_d = max(100.0, (np.abs(lam).sum() + np.abs(zl).sum() + np.abs(zu).sum()) / (m + nb)) / 100.0
        s_c = max(100.0, (np.abs(zl).sum() + np.abs(zu).sum()) / nb) / 100.0
        compl0 = max(np.abs(np.where(hl, dl * zl, 0)).max(), np.abs(np.where(hu, du * zu, 0)).max())
        e_d, e_p, e_c = np.abs(dual).max() / s_d, np.abs(c).max(), compl0 / s_c
        damp = (hl & ~hu).astype(float) - (hu & ~hl).astype(float)
        e_mu = max(np.abs(dual + opts.kappa_d * mu * damp).max() / s_d, e_p,
                   max(np.abs(np.where(hl, dl * zl - mu, 0)).max(), np.abs(np.where(hu, du * zu - mu, 0)).max()) / s_c)
        phi = g["f"][b] - mu * (np.log(dl[hl]).sum() + np.log(du[hu]).sum()) + \
            opts.kappa_d * mu * (((hl & ~hu) * dl).sum() + ((hu & ~hl) * du).sum())
        want = [max(e_d, e_p, e_c), e_d, e_p, e_c]
        np.testing.assert_allclose(head[:4, b], want, rtol=1e-12)
        np.testing.assert_allclose(head[7, b], e_mu, rtol=1e-12)
        np.testing.assert_allclose(head[8, b], np.abs(c).sum(), rtol=1e-12)
        np.testing.assert_allclose([head[9, b], merit[1, b]], [phi, phi], rtol=1e-12)
        # the Newton right-hand side and the step update
        dl_t, du_t, sig, gp, rhs = (x[b].numpy() for x in meas.newton(d["grad"], d["jv"], d["c"], d["y"], d["lam"],
                                                                      d["zl"], d["zu"], d["mu"]))
        gp_ref = np.concatenate([g["grad"][b], np.zeros(mI)]) - np.where(hl, mu / dl, 0) + np.where(hu, mu / du, 0) + \
            opts.kappa_d * mu * damp
        np.testing.assert_allclose(sig, np.where(hl, zl / dl, 0) + np.where(hu, zu / du, 0), rtol=1e-13)
        np.testing.assert_allclose(gp, gp_ref, rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(rhs, np.concatenate([-(gp_ref + AtL), -c]), rtol=1e-11, atol=1e-14)
    rng = np.random.default_rng(9)
    dy = torch.tensor(rng.normal(size=(B, n + mI)) * 0.01)
    y_new = d["y"] + 0.7 * dy
    dlam = torch.tensor(rng.normal(size=(B, m)))
    acc = np.array([True, False, True])
    alpha = np.array([0.7, 0.3, 0.7])
    dl_all, du_all = meas.gaps(d["y"])
    y2, lam2, zl2, zu2, az = meas.step(acc, d["y"], y_new, dy, d["lam"], dlam, d["zl"], d["zu"], dl_all, du_all, d["mu"],
                                       torch.full((B,), 0.99, dtype=torch.float64), alpha)
    for b in range(B):
        zl, zu, mu = g["zl"][b], g["zu"][b], g["mu"][b]
        dl, du = dl_all[b].numpy(), du_all[b].numpy()
        dzl = np.where(hl, mu / dl - zl - zl / dl * dy[b].numpy(), 0)
        dzu = np.where(hu, mu / du - zu + zu / du * dy[b].numpy(), 0)
        ratio = np.concatenate([np.where(hl & (dzl < 0), -0.99 * zl / np.where(dzl < 0, dzl, -1), np.inf),
                                np.where(hu & (dzu < 0), -0.99 * zu / np.where(dzu < 0, dzu, -1), np.inf)])
        a_z = min(1.0, ratio.min())
        np.testing.assert_allclose(az[b].item(), a_z, rtol=1e-13)
        yb = y_new[b].numpy() if acc[b] else g["y"][b]
        np.testing.assert_array_equal(y2[b].numpy(), yb)
        zl_new = zl + (a_z if acc[b] else 0.0) * dzl
        dl_n = np.where(hl, yb - nlp.yl[b].numpy(), 1.0)
        zl_new = np.where(hl, np.clip(zl_new, mu / (1e10 * dl_n), 1e10 * mu / dl_n), zl_new)
        np.testing.assert_allclose(zl2[b].numpy(), zl_new, rtol=1e-13)
        np.testing.assert_allclose(lam2[b].numpy(), g["lam"][b] + (alpha[b] if acc[b] else 0.0) * dlam[b].numpy(),
                                   rtol=1e-14)
