"""Generate the golden NLP vectors in tests/golden/ from the CPU oracle (oracle/ap2_oracle.py).

The reference's own CasADi path cannot run in this container, so these
fixtures pin the *oracle*: the f / g / grad f / J_g / H_L values of the AP2 collocation NLP at
small seeded configurations, stored as plain npz arrays (no pickles).  tests/test_golden.py checks
that the oracle, the CPU port and (on a GPU) the HIP evaluator reproduce them.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from awebox_amd import problem as pb  # noqa: E402
from awebox_amd.initial_guess import batch_member, initial_guess  # noqa: E402
from oracle.ap2_oracle import from_problem  # noqa: E402

# (name, n_k, d, batch member or None, u_ref or None, cost step)
CASES = [("ap2_n3_d2_m2", 3, 2, 2, 7.0, "power1"),
         ("ap2_n2_d4_m0", 2, 4, 0, None, "initial0"),
         ("ap2_n2_d3_v0", 2, 3, None, 9.0, "final0")]


def make(name, n_k, d, member, u_ref, step):
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    V = v0 if member is None else batch_member(v0, lay, member)
    P = pb.pack_p(lay, consts, v0, step=step, u_ref=u_ref)
    orc = from_problem(consts, n_k=n_k, d=d)
    g = orc.nlp_g(V, P, lay, pb.THETA0_OFF).numpy()
    f = float(orc.nlp_f(V, P, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES))
    grad = orc.nlp_grad_f(V, P, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES).numpy()
    J = orc.nlp_jac_g(V, P, lay, pb.THETA0_OFF).tocsc()
    rng = np.random.default_rng(7)
    lam = rng.standard_normal(lay.n_g)
    sigma = 1.0
    H = orc.nlp_hess_l(V, P, sigma, lam, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES)
    import scipy.sparse as sp
    Hu = sp.triu(sp.csc_matrix(H)).tocsc()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), n_k=n_k, d=d, consts=consts.consts, V=V, P=P,
                        f=f, g=g, grad_f=grad, J_data=J.data, J_indices=J.indices, J_indptr=J.indptr,
                        sigma=sigma, lam=lam, H_data=Hu.data, H_indices=Hu.indices, H_indptr=Hu.indptr)
    print(name, "n_v", lay.n_v, "n_g", lay.n_g, "J nnz", J.nnz, "H upper nnz", Hu.nnz)


if __name__ == "__main__":
    for c in CASES:
        make(*c)
