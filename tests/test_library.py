"""The C-ABI library: builds, loads, exports every symbol of include/awegpu.h, and its CPU-side
sparsity derivation is a superset of the oracle's non-zero pattern (no compute on a GPU here)."""
import os
import re
import subprocess

import numpy as np
import pytest
import scipy.sparse as sp

from awebox_amd import problem as pb
from awebox_amd.build import LIB, build
from awebox_amd.evaluator import EXPORTED_SYMBOLS, load_library, sparsity_jac_static
from awebox_amd.initial_guess import batch_member, initial_guess

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "awegpu.h")


@pytest.fixture(scope="module")
def lib():
    build()
    return load_library()


def test_exports_every_header_symbol(lib):
    declared = set(re.findall(r"^(?:int|const char\*)\s+(awe_\w+)\(", open(HEADER).read(), re.M))
    assert declared == set(EXPORTED_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (awe_\w+)", out))
    assert declared <= exported


@pytest.mark.parametrize("n_k,d", [(40, 4), (5, 3)])
def test_static_sparsity_covers_oracle_pattern(lib, n_k, d):
    from oracle.ap2_oracle import from_problem
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    colind, row = sparsity_jac_static(consts)
    assert colind[-1] == row.size and np.all(np.diff(colind) >= 0)
    for c in range(lay.n_v):                       # CCS rows sorted within each column
        r = row[colind[c]:colind[c + 1]]
        assert np.all(np.diff(r) > 0)
    v0 = initial_guess(consts, lay)
    V = batch_member(v0, lay, 0)
    P = pb.pack_p(lay, consts, v0)
    orc = from_problem(consts, n_k=n_k, d=d)
    J = orc.nlp_jac_g(V, P, lay, pb.THETA0_OFF)
    pat = sp.csc_matrix((np.ones(row.size), row, colind), shape=J.shape)
    nz = (J != 0).astype(float)
    assert (nz - nz.multiply(pat)).nnz == 0, "oracle non-zero outside the evaluator's CCS pattern"


def test_no_device_means_no_fallback(lib):
    from awebox_amd.evaluator import Ap2Evaluator, AwegpuUnavailable
    if lib.awe_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(AwegpuUnavailable):
        Ap2Evaluator()


def test_static_hessian_sparsity_equals_cpu_port(lib):
    from awebox_amd.evaluator import sparsity_hess_static
    from oracle.cpu_port import CpuPort
    consts = pb.build_constants(pb.Ap2Config(n_k=5, d=3))
    colind, row = sparsity_hess_static(consts)
    port = CpuPort(consts)
    port.hess_init()
    assert np.array_equal(colind, port.hcolind) and np.array_equal(row, port.hrow)
    # upper triangle, rows sorted within each column
    cols = np.repeat(np.arange(len(colind) - 1), np.diff(colind))
    assert (row <= cols).all()
    for c in range(len(colind) - 1):
        assert (np.diff(row[colind[c]:colind[c + 1]]) > 0).all()


def test_awelu_exports_every_header_symbol():
    """libawelu.so (batched LU + solve) exports what include/awelu.h declares."""
    from awebox_amd.build import LIB_LU, build_one
    build_one(LIB_LU)
    hdr = os.path.join(os.path.dirname(HEADER), "awelu.h")
    declared = set(re.findall(r"^(?:int|const char\*)\s+(awelu_\w+)\(", open(hdr).read(), re.M))
    assert declared == {"awelu_factor_batched", "awelu_solve_batched", "awelu_btd_factor_batched", "awelu_btd_solve_batched",
                        "awelu_sym_inertia_batched", "awelu_gather_sum", "awelu_gather_sum_wide", "awelu_row_sum", "awelu_bmm",
                        "awelu_ipm_measures", "awelu_ipm_newton", "awelu_ipm_step",
                        "awelu_last_error"}
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_LU], capture_output=True, text=True, check=True).stdout
    assert declared <= set(re.findall(r"\bT (awelu_\w+)", out))


@pytest.mark.parametrize("lib_attr,header,prefix,module", [
    ("LIB_DUAL", "awedual.h", "adl_", "awebox_amd.dual_evaluator"),
    ("LIB_MPC", "awempc.h", "awempc_", "awebox_amd.mpc")])
def test_model_libraries_export_every_header_symbol(lib_attr, header, prefix, module):
    """libawedual.so / libawempc.so export what their headers declare, and the ctypes bindings bind
    every declared entry point (no compute: this runs without a GPU)."""
    import importlib

    from awebox_amd import build as B
    path = getattr(B, lib_attr)
    B.build_one(path)
    hdr = os.path.join(os.path.dirname(HEADER), header)
    declared = set(re.findall(r"^(?:int|const char\*)\s+(" + prefix + r"\w+)\(", open(hdr).read(), re.M))
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    assert declared <= set(re.findall(r"\bT (" + prefix + r"\w+)", out))
    mod = importlib.import_module(module)
    lib = mod.load_library()
    for name in declared:
        assert getattr(lib, name) is not None
    if hasattr(mod, "EXPORTED_SYMBOLS"):
        assert declared == set(mod.EXPORTED_SYMBOLS)
