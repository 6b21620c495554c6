"""Known answers the reference holds for the objective and the integral outputs (rows a32/a33),
restated for the AP2 collocation NLP and checked on the evaluator's own f / grad f / Hessian:

* test/units/test_objective.py:63-143 (generalized regularization mechanism): with zoh controls
  the regularization of a state (x.l_t) enters the tracking cost at every collocation node and
  NOT at the shooting nodes (``we_expect_shooting_nodes_to_also_be_weighted``: direct
  collocation + zoh -> False); it does not enter the u-regularisation cost.  The reference
  checks the cost's Jacobian at V = 2 against 1e-4.
* test/units/test_objective.py:168-223: multiplying ``solver.weights.l_t`` by 17.3 multiplies the
  objective Hessian's diagonal at every regularized l_t instance by 17.3 (to 1e-4), with the
  tracking cost of the initial homotopy step set to 1; evaluated at V = 2.
* test/reg/test_quadrature_integration.py:47-69: the integral output of a constant 1 over the
  trajectory equals the time period (to 1e-3).  Here through the power integral of the
  objective: with the integrand p = lambda l_t dl_t set to 1 at every collocation node, the
  power term of f is -c_power (integral of p dt) / (t_f E_scale) (objective.py:279-298 with
  collocation.py:272-316), so the integral recovered from f equals t_f.

CPU: the C++ CPU port (the kernel's algorithm on the host, test infrastructure).  GPU: the HIP
evaluator through the C ABI (first-order kernel and the Hessian kernel).  Tolerances are the
reference's (1e-4 absolute; 1e-3 for the integral)."""
import numpy as np
import pytest

from awebox_amd import problem as pb
from awebox_amd.initial_guess import initial_guess

N_K, D = 5, 4
EPS = 1e-4


def _setup():
    consts = pb.build_constants(pb.Ap2Config(n_k=N_K, d=D))
    lay = pb.NlpLayout(N_K, D)
    return consts, lay, initial_guess(consts, lay)


def _cost(only: dict):
    c = np.zeros(pb.NCOST)
    for k, v in only.items():
        c[pb.COST_NAMES.index(k)] = v
    return c


def _P(consts, lay, v0, cost, w_lt=None, ones=False):
    """P of the initial homotopy step with the given cost vector; ``ones``: p.ref and p.weights
    set to 1 as in the reference's ``trial.nlp.P(1.)`` (test_objective.py:102), theta0 kept."""
    P = pb.pack_p(lay, consts, v0, step="initial0")
    if ones:
        P[lay.p_ref:lay.p_cost] = 1.0
    P[lay.p_cost:lay.p_cost + pb.NCOST] = cost
    if w_lt is not None:
        P[lay.p_weights + pb.W_OFF[("x", "l_t")][0]] = w_lt
    return P


def _lt_indices(lay):
    o = pb.W_OFF[("x", "l_t")][0]
    coll = np.array([lay.coll_x(k, j)[o] for k in range(lay.n_k) for j in range(lay.d)])
    shoot = np.array([lay.x(k)[o] for k in range(lay.n_k + 1)])
    return coll, shoot


def check_regularization_placement(grad_f):
    """grad_f(V, P) -> gradient of f.  test_objective.py:63-143 at V = 2."""
    consts, lay, v0 = _setup()
    V = np.full(lay.n_v, 2.0)
    coll, shoot = _lt_indices(lay)
    g_track = grad_f(V, _P(consts, lay, v0, _cost({"tracking": 1.0}), ones=True))
    assert np.all(g_track[coll] ** 2 >= EPS ** 2), g_track[coll]          # every collocation node
    assert np.all(g_track[shoot] ** 2 < EPS ** 2), g_track[shoot]         # no shooting node (zoh)
    g_ureg = grad_f(V, _P(consts, lay, v0, _cost({"u_regularisation": 1.0}), ones=True))
    assert np.all(g_ureg[np.concatenate([coll, shoot])] ** 2 < EPS ** 2)


def check_weight_scales_hessian(hess_f, factor=17.3):
    """hess_f(V, P) -> dense symmetric Hessian of f.  test_objective.py:168-223 at V = 2."""
    consts, lay, v0 = _setup()
    V = np.full(lay.n_v, 2.0)
    coll, shoot = _lt_indices(lay)
    cost = consts.cost_steps["initial0"].copy()
    cost[pb.COST_NAMES.index("tracking")] = 1.0                # solver.cost.tracking.0 = 1
    H1 = hess_f(V, _P(consts, lay, v0, cost, w_lt=1.0))
    H2 = hess_f(V, _P(consts, lay, v0, cost, w_lt=factor))
    d1, d2 = np.diag(H1)[coll], np.diag(H2)[coll]
    assert np.all(d1 ** 2 >= EPS ** 2), d1
    assert np.all((d2 - factor * d1) ** 2 <= EPS ** 2), (d1, d2)
    # the expected value itself: d^2/dl^2 of w_j psi (c_track W / norm) (l - ref)^2, psi = 2; the
    # xdot regularisation (cost 1e-8 in the initial step) adds ~1e-9 relative through the
    # collocation polynomial (dl_t's xdot depends on the collocation l_t)
    w = pb.collocation(D)[3]
    norm = consts.consts[pb.CONST_IDX["norm_tracking"]]
    expect = np.array([2.0 * w[j] * 2.0 * 1.0 / norm for k in range(N_K) for j in range(D)])
    np.testing.assert_allclose(d1, expect, rtol=1e-7)


def check_integral_of_one_is_period(f_of):
    """f_of(V, P) -> f.  test_quadrature_integration.py:47-69 through the power integral."""
    consts, lay, v0 = _setup()
    s = consts.scaling
    V = v0.copy()
    o_l, _ = pb.W_OFF[("x", "l_t")]
    o_dl, _ = pb.W_OFF[("x", "dl_t")]
    o_lam, _ = pb.W_OFF[("z", "lambda10")]
    for k in range(N_K):
        for j in range(D):
            cx = lay.coll_x(k, j)
            V[cx[o_l]] = 1.0 / s[o_l]                  # l_t = 1 m
            V[cx[o_dl]] = 1.0 / s[o_dl]                # dl_t = 1 m/s
            V[lay.coll_z(k, j)[0]] = 1.0 / s[o_lam]    # lambda = 1 N/m  -> p = 1 W at every node
    V[lay.phi("psi")] = 0.0                            # the power problem's share (1 - psi) = 1
    c_p = 3.0
    P = _P(consts, lay, v0, _cost({"power": c_p}))
    tf = V[lay.theta()[1]] * s[pb.W_TH0 + 1]
    E_s = consts.consts[pb.CONST_IDX["energy_scaling"]]
    integral = -f_of(V, P) * tf * E_s / c_p
    assert abs(integral - tf) < 1e-3, (integral, tf)
    assert abs(integral - tf) <= 1e-12 * tf


# ---- CPU port (test infrastructure) ---------------------------------------------------------
def _port():
    from oracle.cpu_port import CpuPort
    return CpuPort(_setup()[0])


def test_regularization_placement_cpu_port():
    port = _port()
    check_regularization_placement(lambda V, P: port.eval_nlp(V, P)["grad_f"][0])


def test_weight_scales_hessian_cpu_port():
    port = _port()
    lay = pb.NlpLayout(N_K, D)
    check_weight_scales_hessian(
        lambda V, P: port.hess_csc(port.eval_hess(V, P, 1.0, np.zeros(lay.n_g))[0]).toarray())


def test_integral_of_one_is_period_cpu_port():
    port = _port()
    check_integral_of_one_is_period(lambda V, P: float(port.eval_nlp(V, P)["f"][0]))


# ---- HIP evaluator --------------------------------------------------------------------------
@pytest.fixture(scope="module")
def hip_ev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.evaluator import Ap2Evaluator
    return Ap2Evaluator(_setup()[0], batch=1)


@pytest.mark.gpu
def test_regularization_placement_hip(hip_ev):
    check_regularization_placement(lambda V, P: hip_ev.eval_nlp(V, P)["grad_f"][0])


@pytest.mark.gpu
def test_weight_scales_hessian_hip(hip_ev):
    lay = pb.NlpLayout(N_K, D)
    check_weight_scales_hessian(
        lambda V, P: hip_ev.hess_csc(hip_ev.eval_hess(V, P, 1.0, np.zeros((1, lay.n_g)))[0]).toarray())


@pytest.mark.gpu
def test_integral_of_one_is_period_hip(hip_ev):
    check_integral_of_one_is_period(lambda V, P: float(hip_ev.eval_nlp(V, P)["f"][0]))
