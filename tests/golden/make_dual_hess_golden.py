"""Generate the dual-kite Hessian fixtures in tests/golden/ from the CPU oracle
(oracle/multikite_oracle.py, nlp_hess_l).

The oracle's dense objective Hessian takes about a minute per case on the CPU, too slow to run in
every GPU session, so its output is stored here (plain npz, no pickles) and
tests/test_dual_hess_gpu.py compares the HIP kernel (libawedual.so, dual_hess_kernel) with it.
Inputs are stored too: V is a seeded perturbation of the standard multi-kite guess with the
homotopy parameter psi set strictly between 0 and 1, so both the tracking and the power cost
(with its phase-fixed period, ocp_outputs.py:118-140) carry second-order terms.

    python tests/golden/make_dual_hess_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from awebox_amd import dual as du  # noqa: E402
from awebox_amd import problem as pb  # noqa: E402
from oracle import multikite_oracle as mo  # noqa: E402

# (name, n_k, d, batch member, u_ref, cost step, psi, sigma)
CASES = [("dual_hess_n3_d2", 3, 2, 1, 7.0, "power1", 0.4, 1.0),
         ("dual_hess_n4_d3", 4, 3, 2, 9.0, "final0", 0.7, 0.6)]


def make(name, n_k, d, member, u_ref, step, psi, sigma):
    import scipy.sparse as sp
    mc = du.build_constants(du.MultiConfig(n_k=n_k, d=d))
    lay = du.layout_for(mc)
    V0 = du.initial_guess(mc, lay)
    V = du.batch_member(V0, lay, member)
    V[lay.phi()[pb.PHI_NAMES.index("psi")]] = psi
    P = du.pack_p(lay, mc, V0, step, u_ref=u_ref)
    o = mo.from_constants(mc, lay)
    th = mo.theta0_dict(P[lay.p_theta0:])
    lam = np.random.default_rng(17).standard_normal(lay.n_g)
    H = o.nlp_hess_l(V, P, sigma, lam, lay, th, pb.COST_NAMES, pb.PHI_NAMES)
    Hu = sp.triu(sp.csc_matrix(H)).tocsc()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), n_k=n_k, d=d, V=V, P=P, sigma=sigma, lam=lam,
                        H_data=Hu.data, H_indices=Hu.indices, H_indptr=Hu.indptr)
    print(name, "n_v", lay.n_v, "H upper nnz", Hu.nnz)


if __name__ == "__main__":
    for case in CASES:
        make(*case)
