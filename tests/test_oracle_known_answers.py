"""Restated known-answer tests of the reference, applied to the CPU oracle.

* Lagrangian residual of a pendulum / pseudo-Atwood machine is ~0 for consistent inputs and large
  for inconsistent ones (``test/units/test_model.py:438-787``): m=17 kg, g=11 m/s^2, L=37 m, rod
  d=0.02 m (massless or 41 kg), angle 0.35*pi, frictionless (rho_ref = 0, u_ref = 1e-15).
  The reference builds a 3-DOF kite for these; the translational/holonomic Lagrangian code path
  (``lagr_dyn.py:20-204``) is identical for the 6-DOF AP2 model used here, whose extra rows are
  made consistent with R = I, omega = 0.
* time derivative under non-trivial scaling (``test_model.py:789-832``).
* Radau constants against an independent computation.
"""
import math

import numpy as np
import pytest
import torch

from awebox_amd import problem as pb
from oracle.ap2_oracle import IDX, Ap2Oracle, from_problem


def _system(rod_has_mass, kind):
    mass, g, length = 17., 11., 37.
    angle = np.pi / 2. * 0.7 if kind == "pendulum" else 0.
    rod_mass = 41. if rod_has_mass else 0.
    diam = 0.02
    vol = np.pi * (diam / 2.) ** 2. * length
    return dict(mass=mass, g=g, length=length, length_full=5 * length, angle=angle, rod_mass=rod_mass,
                diam=diam, rho=rod_mass / vol)


def _consistent(sp, kind):
    xhat, zhat = np.array([1., 0, 0]), np.array([0, 0, 1.])
    if kind == "pendulum":
        th = sp["angle"]
        num = sp["rod_mass"] / 2. + sp["mass"]
        den = sp["rod_mass"] / 3. + sp["mass"]
        ddth = -(sp["g"] / sp["length"]) * (num / den) * np.sin(th)
        q = sp["length"] * (-np.sin(th) * xhat - np.cos(th) * zhat)
        dq = np.zeros(3)
        ddq = sp["length"] * (-np.cos(th) * xhat + np.sin(th) * zhat) * ddth
        total = sp["mass"] + sp["rod_mass"]
        tension = -total * sp["g"] * np.dot(zhat, q / sp["length"])
        return dict(q10=q, dq10=dq, ddq10=ddq, l_t=sp["length"], dl_t=0., ddl_t=0.,
                    lambda10=tension / sp["length"], diam_t=sp["diam"], t_f=1.0)
    area = np.pi * (sp["diam"] / 2.) ** 2.
    m_unw = sp["length"] * area * sp["rho"]
    m_full = sp["length_full"] * area * sp["rho"]
    ddl = sp["g"] * (m_unw + sp["mass"]) / (m_full + sp["mass"])
    tension = (sp["mass"] + m_unw) * (sp["g"] - ddl)
    return dict(q10=-sp["length"] * zhat, dq10=-2. * zhat, ddq10=-ddl * zhat, l_t=sp["length"], dl_t=2.,
                ddl_t=ddl, lambda10=tension / sp["length"], diam_t=sp["diam"], t_f=1.0)


def _eval(kind, rod_has_mass, consistent):
    consts = pb.build_constants()
    orc = from_problem(consts)
    sp = _system(rod_has_mass, kind)
    init = _consistent(sp, kind)
    if not consistent:
        init["q10"] = 80 * np.array([1., 0, 0])
        init["dq10"] = 50. + init["q10"]
        init["lambda10"] = 4.
    w_si = np.zeros(pb.NW)
    for (vt, name), sl in IDX.items():
        if name in init:
            w_si[sl] = init[name]
    w_si[IDX[("x", "r10")]] = np.eye(3).reshape(-1, order="F")
    w_sc = torch.as_tensor(w_si / consts.scaling)
    th = orc.unpack_theta0(torch.as_tensor(consts.theta0), pb.THETA0_OFF)
    th = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in th.items()}
    th["atmosphere.rho_ref"] = torch.tensor(0.)
    th["atmosphere.g"] = torch.tensor(sp["g"])
    th["geometry.m_k"] = torch.tensor(sp["mass"])
    th["wind.u_ref"] = torch.tensor(1e-15)
    th["tether.rho"] = torch.tensor(sp["rho"])
    eq, ineq, power, beta = orc.node(w_sc, torch.tensor(1.0), th)
    return eq


@pytest.mark.parametrize("kind,rod,eps", [("pendulum", False, 1e-5), ("pendulum", True, 1e-5),
                                          ("pseudo_atwood", False, 1e-5), ("pseudo_atwood", True, 1e-2)])
def test_lagrangian_residual_zero_for_consistent_inputs(kind, rod, eps):
    eq = _eval(kind, rod, True)
    assert float(eq @ eq) < eps ** 2, eq


@pytest.mark.parametrize("kind", ["pendulum", "pseudo_atwood"])
def test_lagrangian_residual_nonzero_for_inconsistent_inputs(kind):
    eq = _eval(kind, False, False)
    assert float(eq @ eq) > (1e-2) ** 2


def test_time_derivative_under_scaling():
    # test_model.py:789-832: d/dt(q_si) == x.dq_si and == xdot.dq_si for consistent values
    consts = pb.build_constants()
    orc = from_problem(consts)
    assert not np.allclose(consts.scaling[IDX[("x", "q10")]], consts.scaling[IDX[("x", "dq10")]])
    rng = np.random.default_rng(0)
    w_sc = torch.as_tensor(rng.standard_normal(pb.NW))
    w_sc[IDX[("x", "r10")]] = torch.as_tensor(np.eye(3).reshape(-1))
    for name, dname in (("q10", "dq10"), ("l_t", "dl_t")):
        f = lambda w: orc.si(w)[IDX[("x", name)]]  # noqa: E731
        dot = orc.time_derivative(f)(w_sc)
        ref = orc.si(w_sc)[IDX[("x", dname)]]
        assert torch.allclose(dot, ref, rtol=1e-13, atol=1e-13)


def test_radau_constants_independent():
    # collocation.py:67-200 restated two ways: awebox_amd.collocation (product rule on the exact
    # roots) vs the oracle (numpy Legendre roots + monomial derivative)
    from awebox_amd.collocation import coefficients
    tau, C, D, w = coefficients(4)
    o_tau, o_C, o_D, o_w = Ap2Oracle._radau(4)
    np.testing.assert_allclose(tau, o_tau, rtol=0, atol=2e-15)
    np.testing.assert_allclose(C, o_C, rtol=0, atol=1e-12)
    np.testing.assert_array_equal(D, o_D)
    np.testing.assert_allclose(w, o_w, rtol=0, atol=1e-14)
    # published Radau IIA (s=4) nodes and weights
    np.testing.assert_allclose(tau[1:], [0.088587959512704, 0.409466864440735, 0.787659461760847, 1.0], atol=1e-14)
    np.testing.assert_allclose(w, [0.2204622112, 0.3881934688, 0.3288443200, 0.0625], atol=1e-10)
    assert abs(w.sum() - 1.0) < 1e-14
    assert D[-1] == 1.0 and np.all(D[:-1] == 0.0)
