"""Golden NLP vectors (tests/golden/*.npz, made by tests/golden/make_golden.py from the oracle).

* the oracle still reproduces them (guards the checker itself against drift);
* the CPU port (the evaluator's algorithm on the host) matches them;
* on a GPU, the HIP evaluator's f / g / grad f / J_g and H_L match them.
Tolerances as in test_gpu_parity.py (fp64, rtol 1e-10 on each entry plus 1e-12 of the largest)."""
import glob
import os

import numpy as np
import pytest
import scipy.sparse as sp

from awebox_amd import problem as pb

from test_cpu_port import _close_hess
from test_gpu_parity import _close, _close_jac

# the AP2 evaluator fixtures (the dual-kite Hessian fixtures, dual_hess_*.npz, belong to test_dual_hess_gpu.py)
FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "ap2_*.npz")))
IDS = [os.path.basename(f)[:-4] for f in FILES]


def _load(path):
    z = np.load(path)              # allow_pickle=False (default): plain arrays only
    n_k, d = int(z["n_k"]), int(z["d"])
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    assert np.array_equal(consts.consts, z["consts"]), "model constants changed since the fixture"
    lay = pb.NlpLayout(n_k, d)
    J = sp.csc_matrix((z["J_data"], z["J_indices"], z["J_indptr"]), shape=(lay.n_g, lay.n_v))
    U = sp.csc_matrix((z["H_data"], z["H_indices"], z["H_indptr"]), shape=(lay.n_v, lay.n_v))
    H = (U + sp.triu(U, 1).T).tocsc()
    return consts, lay, z, J, H


def test_golden_fixtures_present():
    assert len(FILES) >= 3


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_oracle_reproduces_golden(path):
    from oracle.ap2_oracle import from_problem
    consts, lay, z, J, H = _load(path)
    orc = from_problem(consts, n_k=lay.n_k, d=lay.d)
    V, P = z["V"], z["P"]
    np.testing.assert_allclose(orc.nlp_g(V, P, lay, pb.THETA0_OFF).numpy(), z["g"], rtol=1e-13, atol=1e-13)
    f = float(orc.nlp_f(V, P, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES))
    assert f == pytest.approx(float(z["f"]), rel=1e-13)
    _close_jac(orc.nlp_jac_g(V, P, lay, pb.THETA0_OFF), J)


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_cpu_port_matches_golden(path):
    from oracle.cpu_port import CpuPort
    consts, lay, z, J, H = _load(path)
    port = CpuPort(consts)
    out = port.eval_nlp(z["V"], z["P"])
    _close(out["g"][0], z["g"], "g")
    assert out["f"][0] == pytest.approx(float(z["f"]), rel=1e-12)
    _close(out["grad_f"][0], z["grad_f"], "grad_f")
    _close_jac(port.jac_csc(out["jac"][0]), J)
    Hp = port.hess_csc(port.eval_hess(z["V"], z["P"], float(z["sigma"]), z["lam"])[0])
    _close_hess(Hp, H)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_hip_evaluator_matches_golden(path):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.evaluator import Ap2Evaluator
    consts, lay, z, J, H = _load(path)
    ev = Ap2Evaluator(consts, batch=1)
    out = ev.eval_nlp(z["V"], z["P"])
    _close(out["g"][0], z["g"], "g")
    assert out["f"][0] == pytest.approx(float(z["f"]), rel=1e-12)
    _close(out["grad_f"][0], z["grad_f"], "grad_f")
    _close_jac(ev.jac_csc(out["jac"][0]), J)
    Hk = ev.hess_csc(ev.eval_hess(z["V"], z["P"], float(z["sigma"]), z["lam"])[0])
    _close_hess(Hk, H)
