"""The oracle's Hessian of the Lagrangian (per-interval blocks) against torch.func.hessian of
sigma f + lam^T g over the whole decision vector, and its per-interval objective against nlp_f."""
import numpy as np
import pytest
import torch

from awebox_amd import problem as pb
from awebox_amd.initial_guess import batch_member, initial_guess


@pytest.mark.parametrize("n_k,d", [(3, 2), (40, 4)])
def test_interval_objective_sums_to_nlp_f(n_k, d):
    from oracle.ap2_oracle import from_problem
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    orc = from_problem(consts, n_k=n_k, d=d)
    V, P = batch_member(v0, lay, 1), pb.pack_p(lay, consts, v0, u_ref=6.5)
    args = (lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES)
    assert float(orc.nlp_f_by_interval(V, P, *args)) == pytest.approx(float(orc.nlp_f(V, P, *args)), rel=1e-13)


def test_hessian_blocks_match_full_hessian():
    from torch.func import hessian

    from oracle.ap2_oracle import from_problem
    n_k, d = 3, 2
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    orc = from_problem(consts, n_k=n_k, d=d)
    V, P = batch_member(v0, lay, 2), pb.pack_p(lay, consts, v0)
    lam = np.random.default_rng(7).standard_normal(lay.n_g)
    sigma = 1.3
    H = orc.nlp_hess_l(V, P, sigma, lam, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES).toarray()
    lt = torch.as_tensor(lam)

    def lag(v):
        return (sigma * orc.nlp_f(v, P, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES)
                + lt @ orc.nlp_g(v, P, lay, pb.THETA0_OFF))

    Hf = hessian(lag)(torch.as_tensor(V)).numpy()
    assert np.abs(H - Hf).max() <= 1e-12 * np.abs(Hf).max()
