"""The generated node-Jacobian code (awebox_amd/csrc/ap2_nodejac.gen.hpp, written by
csrc/gen/ap2_jacgen.cpp from the templated node model) against the same model evaluated in
dual-number arithmetic, one forward pass per seed direction with the seeding of awegpu.hip's colour
kernel (csrc/gen/check_ap2_gen.cpp), on the host.  The GPU parity of the generated path against the
oracle is in tests/test_gpu_parity.py (it is the default path of awe_eval_nlp)."""
import json
import os
import subprocess

import numpy as np
import pytest

from awebox_amd import build as B
from awebox_amd import problem as pb
from awebox_amd.initial_guess import initial_guess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "awebox_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("gen")
    exe = str(tmp / "check")
    subprocess.run(["g++", "-O1", "-std=c++17", os.path.join(CSRC, "gen", "check_ap2_gen.cpp"), "-o", exe],
                   check=True)
    return tmp, exe


def test_committed_header_is_current():
    """The header in the tree is what the generator writes for the current model."""
    before = open(B.GEN_HEADER).read()
    B.generate(force=True)
    assert open(B.GEN_HEADER).read() == before, "ap2_nodejac.gen.hpp is stale: run python -m awebox_amd.build"


@pytest.mark.parametrize("k,seed", [(0, 0), (7, 1), (23, 2), (39, 3)])
def test_generated_jacobian_matches_dual_model(checker, k, seed):
    tmp, exe = checker
    consts = pb.build_constants(pb.Ap2Config(n_k=40, d=4))
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    P = pb.pack_p(lay, consts, v0)
    th = P[lay.n_v + pb.NW + pb.NCOST:]
    rng = np.random.default_rng(seed)
    w = np.concatenate([v0[lay.x(k)], v0[lay.xdot(k)], v0[lay.u(k)], v0[lay.z(k)], v0[lay.theta()],
                        v0[lay.phi()][:1]])
    w = w * (1 + 0.05 * rng.standard_normal(w.shape)) + 0.01 * rng.standard_normal(w.shape)
    for name, arr in (("consts", consts.consts), ("th", th), ("w", w)):
        np.savetxt(str(tmp / f"{name}.txt"), arr)
    cxx, inv_tf = 2.0 + rng.random(), 1.0 / (20.0 + 30.0 * rng.random())
    out = subprocess.run([exe, str(tmp / "consts.txt"), str(tmp / "th.txt"), str(tmp / "w.txt"), repr(cxx),
                          repr(inv_tf)], check=True, capture_output=True, text=True)
    rec = json.loads(out.stdout)
    for kind in ("shooting", "radau"):
        r = rec[kind]
        assert r["entries"] == r["n_tan"], "every tangent slot is a pattern entry"
        assert r["value_rel"] < 1e-14, (kind, r)
        assert r["tangent_rel"] < 1e-12, (kind, r)
        assert r["tangent_max"] > 1.0


@pytest.fixture(scope="module")
def hess_checker(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("hgen")
    exe = str(tmp / "check_hess")
    subprocess.run(["g++", "-O1", "-std=c++17", os.path.join(CSRC, "gen", "check_ap2_hess.cpp"), "-o", exe],
                   check=True)
    return tmp, exe


def test_committed_hessian_header_is_current():
    """ap2_nodehess.gen.hpp in the tree is what gen/ap2_hessgen.cpp writes for the current model."""
    before = open(B.HESS_HEADER).read()
    B.generate(force=True)
    assert open(B.HESS_HEADER).read() == before, "ap2_nodehess.gen.hpp is stale: run python -m awebox_amd.build"


@pytest.mark.parametrize("k,seed", [(0, 0), (13, 1), (39, 2)])
def test_generated_hessian_matches_hyperdual_model(hess_checker, k, seed):
    """Every direction pair of the node Hessian pattern (and dL/dxdot at a Radau node) against one
    hyper-dual evaluation of the node Lagrangian per pair (csrc/gen/check_ap2_hess.cpp)."""
    tmp, exe = hess_checker
    consts = pb.build_constants(pb.Ap2Config(n_k=40, d=4))
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    P = pb.pack_p(lay, consts, v0)
    th = P[lay.n_v + pb.NW + pb.NCOST:]
    rng = np.random.default_rng(seed)
    w = np.concatenate([v0[lay.x(k)], v0[lay.xdot(k)], v0[lay.u(k)], v0[lay.z(k)], v0[lay.theta()],
                        v0[lay.phi()][:1], [0.5]])                      # last: phi.psi
    w = w * (1 + 0.05 * rng.standard_normal(w.shape)) + 0.01 * rng.standard_normal(w.shape)
    for name, arr in (("consts", consts.consts), ("th", th), ("w", w)):
        np.savetxt(str(tmp / f"{name}.txt"), arr)
    cxx, inv_tf = 2.0 + rng.random(), 1.0 / (20.0 + 30.0 * rng.random())
    out = subprocess.run([exe, str(tmp / "consts.txt"), str(tmp / "th.txt"), str(tmp / "w.txt"), repr(cxx),
                          repr(inv_tf), "0.37", "-1.9"], check=True, capture_output=True, text=True)
    rec = json.loads(out.stdout)
    for kind in ("shooting", "radau"):
        r = rec[kind]
        assert r["hess_rel"] < 1e-12, (kind, r)
        assert r["grad_rel"] < 1e-12, (kind, r)
        assert r["hess_max"] > 1.0 and r["nonzero"] > 150, (kind, r)


# ---- tracking MPC (3-DOF kite): csrc/gen/kite3_jacgen.cpp -> kite3_nodejac.gen.hpp ----------------
@pytest.fixture(scope="module")
def k3_checker(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("k3gen")
    exe = str(tmp / "check_k3")
    subprocess.run(["g++", "-O1", "-std=c++17", os.path.join(CSRC, "gen", "check_kite3_gen.cpp"), "-o", exe],
                   check=True)
    return tmp, exe


def test_committed_kite3_header_is_current():
    """kite3_nodejac.gen.hpp in the tree is what gen/kite3_jacgen.cpp writes for the current model."""
    before = open(B.K3_HEADER).read()
    B.generate(force=True)
    assert open(B.K3_HEADER).read() == before, "kite3_nodejac.gen.hpp is stale: run python -m awebox_amd.build"


@pytest.mark.parametrize("k,seed", [(0, 0), (9, 1), (19, 2)])
def test_generated_kite3_jacobian_matches_dual_model(k3_checker, k, seed):
    """Every entry of the MPC node Jacobian pattern (both node kinds) against one dual-number pass of
    kite3_node per seed direction (csrc/gen/check_kite3_gen.cpp)."""
    from awebox_amd import kite3 as k3
    tmp, exe = k3_checker
    c = k3.build_constants()
    lay = k3.MpcLayout(20, 4)
    V, p = k3.batch_instance(c, lay, k, 8)
    rng = np.random.default_rng(seed)
    w = np.concatenate([V[lay.x(k)], V[lay.xdot(k)], V[lay.u(k)], V[lay.z(k)], V[lay.theta()], V[lay.phi()][:1]])
    w = w * (1 + 0.05 * rng.standard_normal(w.shape)) + 0.01 * rng.standard_normal(w.shape)
    np.savetxt(str(tmp / "consts.txt"), c.consts)
    np.savetxt(str(tmp / "w.txt"), w)
    u_ref, cxx, inv_tf = 4.0 + 4.0 * rng.random(), 2.0 + rng.random(), 1.0 / (0.5 + rng.random())
    out = subprocess.run([exe, str(tmp / "consts.txt"), str(tmp / "w.txt"), repr(u_ref), repr(cxx), repr(inv_tf)],
                         check=True, capture_output=True, text=True)
    rec = json.loads(out.stdout)
    for kind in ("shooting", "radau"):
        r = rec[kind]
        assert r["entries"] == r["n_tan"], "every tangent slot is a pattern entry"
        assert r["value_rel"] < 1e-14, (kind, r)
        assert r["tangent_rel"] < 1e-12, (kind, r)
        assert r["tangent_max"] > 1.0


# ---- dual kites: csrc/gen/dual_jacgen.cpp -> dual_nodejac.gen.hpp ---------------------------------
@pytest.fixture(scope="module")
def dual_checker(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("dgen")
    exe = str(tmp / "check_dual")
    subprocess.run(["g++", "-O1", "-std=c++17", os.path.join(CSRC, "gen", "check_dual_gen.cpp"), "-o", exe],
                   check=True)
    return tmp, exe


def test_committed_dual_header_is_current():
    """dual_nodejac.gen.hpp in the tree is what gen/dual_jacgen.cpp writes for the current model."""
    before = open(B.DUAL_HEADER).read()
    B.generate(force=True)
    assert open(B.DUAL_HEADER).read() == before, "dual_nodejac.gen.hpp is stale: run python -m awebox_amd.build"


@pytest.mark.parametrize("k,seed", [(0, 0), (41, 1), (59, 2)])
def test_generated_dual_jacobian_matches_dual_model(dual_checker, k, seed):
    """Every entry of the dual-kite node Jacobian pattern (both node kinds, all four wavefront roles),
    the power / side-slip values and the objective terms' directional derivatives against one
    dual-number pass of dual_node per seed direction (csrc/gen/check_dual_gen.cpp)."""
    from awebox_amd import dual as du
    tmp, exe = dual_checker
    mc = du.build_constants(du.MultiConfig(n_k=60, d=4))
    lay = du.layout_for(mc)
    V = du.batch_member(du.initial_guess(mc, lay), lay, seed)
    rng = np.random.default_rng(seed)
    w = np.concatenate([V[lay.x(k)], V[lay.xdot(k)], V[lay.u(k)], V[lay.z(k)], V[lay.node_theta_index(k)],
                        V[lay.phi()][:1]])
    w = w * (1 + 0.05 * rng.standard_normal(w.shape)) + 0.01 * rng.standard_normal(w.shape)
    assert w.size == 127
    np.savetxt(str(tmp / "consts.txt"), mc.consts)
    np.savetxt(str(tmp / "theta0.txt"), mc.theta0)
    np.savetxt(str(tmp / "w.txt"), w)
    cxx, inv_tf = 2.0 + rng.random(), 1.0 / (10.0 + 5.0 * rng.random())
    ex2, ex3 = 0.1 + rng.random(), -(0.1 + rng.random())
    out = subprocess.run([exe, str(tmp / "consts.txt"), str(tmp / "theta0.txt"), str(tmp / "w.txt"), repr(cxx),
                          repr(inv_tf), repr(ex2), repr(ex3)], check=True, capture_output=True, text=True)
    rec = json.loads(out.stdout)
    for kind in ("shooting", "radau"):
        r = rec[kind]
        assert r["entries"] == r["n_tan"], "every tangent slot is a pattern entry"
        assert r["value_rel"] < 1e-13, (kind, r)
        assert r["tangent_rel"] < 1e-11, (kind, r)
        assert r["tangent_max"] > 1.0
    assert rec["radau"]["obv_rel"] < 1e-13 and rec["radau"]["dbp_rel"] < 1e-11, rec["radau"]
