"""Energy conservation of the shared node model (known-answer test).

Restates ``test/units/test_model.py:862-1168``: a frictionless pendulum (massless or massive rod)
and a pseudo-Atwood machine with a massless cable conserve the total energy of the model's own
Lagrangian over an integration of its DAE, the pseudo-Atwood machine with a massive cable does
not (the reeled-out mass enters with the momentum correction of ``lagr_dyn.py:174-204``).

The DAE is the product's node model (``awebox_amd/csrc/ap2_model.hpp``) reached through the CPU
port's ``ap2cpu_node`` export: the 24 model equalities are affine in (xdot, z), so each RK4 stage
solves them for the state derivative and the tether multiplier with one Newton step on the
Jacobian the port returns.  The reference integrates with IDAS at 100 (pendulum) / 1000
(pseudo-Atwood) steps per second; here fixed-step RK4 at the same steps.  System constants are the
ones of ``tests/test_oracle_known_answers.py`` (m=17 kg, g=11, L=37 m, rod d=0.02 m).  The
pseudo-Atwood free fall also checks the final kite position (``test_model.py:1052-1080``).
"""
import math

import numpy as np
import pytest

from awebox_amd import problem as pb
from oracle.cpu_port import CpuPort

from test_oracle_known_answers import _consistent, _system

XD = np.arange(pb.W_XDOT0, pb.W_XDOT0 + pb.NX)
UNK = np.concatenate([XD, [pb.W_Z0]])


def _setup(kind, rod_has_mass):
    consts = pb.build_constants(pb.Ap2Config(n_k=2, d=1))
    port = CpuPort(consts)
    sp = _system(rod_has_mass, kind)
    init = _consistent(sp, kind)
    th = np.array(consts.theta0, dtype=float)

    def put(name, v):
        th[pb.THETA0_OFF[name][0]] = v
    put("atmosphere.rho_ref", 0.0)
    put("atmosphere.g", sp["g"])
    put("geometry.m_k", sp["mass"])
    put("wind.u_ref", 1e-15)
    put("tether.rho", sp["rho"])
    w_si = np.zeros(pb.NW)
    for (vt, name), (o, n) in pb.W_OFF.items():
        if name in init and vt in ("x", "u", "z", "theta"):
            w_si[o:o + n] = init[name]
    o, _ = pb.W_OFF[("x", "r10")]
    w_si[o:o + 9] = np.eye(3).reshape(-1, order="F")
    return consts, port, sp, th, w_si


def _energy(w_si, sp, th):
    q = w_si[pb.W_OFF[("x", "q10")][0]:][:3]
    dq = w_si[pb.W_OFF[("x", "dq10")][0]:][:3]
    om = w_si[pb.W_OFF[("x", "omega10")][0]:][:3]
    m_t = sp["rho"] * math.pi * sp["diam"] ** 2 / 4 * np.linalg.norm(q)
    ehat = q / np.linalg.norm(q)
    dq_p = (dq @ ehat) * ehat
    ke_t = 0.5 * m_t / 3 * (dq @ dq + dq_p @ dq_p + dq @ dq_p)
    o = pb.THETA0_OFF["geometry.j"][0]
    J = th[o:o + 9].reshape(3, 3, order="F")
    ke = ke_t + 0.5 * sp["mass"] * dq @ dq + 0.5 * om @ J @ om
    pe = sp["g"] * m_t * q[2] / 2 + sp["g"] * sp["mass"] * q[2]
    return ke + pe


def _integrate(port, consts, th, w_si, t_end, steps_per_s):
    s = consts.scaling
    dt = 1.0 / steps_per_s
    xs = slice(0, pb.NX)

    def deriv(x_si):
        w = w_si.copy()
        w[xs] = x_si
        w_sc = w / s
        for _ in range(2):                          # the rows are affine in (xdot, z)
            rows, jac = port.node(w_sc, th)
            w_sc[UNK] -= np.linalg.solve(jac[:pb.N_EQ][:, UNK], rows[:pb.N_EQ])
        return (w_sc * s)[XD]

    x = w_si[xs].copy()
    for _ in range(int(round(t_end * steps_per_s))):
        k1 = deriv(x)
        k2 = deriv(x + 0.5 * dt * k1)
        k3 = deriv(x + 0.5 * dt * k2)
        k4 = deriv(x + dt * k3)
        x = x + dt / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    out = w_si.copy()
    out[xs] = x
    return out


@pytest.mark.parametrize("kind,rod,conserved,eps", [
    ("pendulum", False, True, 1e-2),
    ("pendulum", True, True, 1e-2),
    ("pseudo_atwood", False, True, 1e-2),
    ("pseudo_atwood", True, False, 1e-4),
])
def test_energy_conservation(kind, rod, conserved, eps):
    consts, port, sp, th, w0 = _setup(kind, rod)
    t_end, rate = (30.0, 100) if kind == "pendulum" else (4.0, 1000)
    w1 = _integrate(port, consts, th, w0, t_end, rate)
    e0, e1 = _energy(w0, sp, th), _energy(w1, sp, th)
    err = (e1 - e0) / e0
    assert (err ** 2 < eps ** 2) == conserved, (e0, e1, err)
    if kind == "pendulum":                         # the rod length is held by the constraint
        q = w1[pb.W_OFF[("x", "q10")][0]:][:3]
        assert abs(np.linalg.norm(q) - sp["length"]) < 1e-3 * sp["length"]
        assert q[0] > 0.5 * sp["length"]            # swung through to the other side
    elif not rod:
        # free fall of the kite on a massless cable (test_model.py:1052-1080, epsilon 2 m)
        q = w1[pb.W_OFF[("x", "q10")][0]:][:3]
        z_exp = -sp["length"] - 2.0 * t_end - 0.5 * sp["g"] * t_end ** 2
        assert np.linalg.norm(q - np.array([0.0, 0.0, z_exp])) < 2.0
