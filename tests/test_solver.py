"""GPU interior-point solver and the AP2 homotopy (row f2).

CPU: the solver's algorithm through the CPU port (oracle/cpu_device.py) on a small problem:
every homotopy step converges, the final point satisfies the KKT conditions to IPOPT's tol and the
bounds, and a cold-started final solve from the returned point stays put.
GPU: the same homotopy at N=10 d=4 on the HIP evaluator."""
import numpy as np
import pytest

from awebox_amd import homotopy as hm
from awebox_amd import problem as pb
from awebox_amd.initial_guess import initial_guess
from awebox_amd.ipm import IpmOptions, solve
from awebox_amd.trajectory import optimize


def _check_solution(consts, lay, V, summary):
    assert all(r["status"] == "solve_succeeded" for r in summary), summary
    assert summary[-1]["kkt_error"] <= 1e-8
    steps = hm.schedule(consts, lay, initial_guess(consts, lay))
    lb, ub = steps[-1].lbx, steps[-1].ubx
    assert (V >= lb - 1e-9).all() and (V <= ub + 1e-9).all()
    phi = V[lay.phi()]
    assert np.abs(phi).max() <= 1e-9             # every homotopy parameter driven to 0
    out = hm.outputs(consts, lay, V)
    assert 20.0 <= out["period_s"] <= 70.0
    assert out["avg_power_W"] > 1000.0            # a power-producing orbit


def test_homotopy_on_cpu_port():
    from oracle.cpu_device import CpuDeviceEvaluator
    consts = pb.build_constants(pb.Ap2Config(n_k=6, d=3))
    lay = pb.NlpLayout(6, 3)
    ev = CpuDeviceEvaluator(consts)
    V, summary, out, _ = optimize(consts, ev, IpmOptions(max_iter=400), device="cpu")
    _check_solution(consts, lay, V, summary)


def _kkt_case(device, evaluator, n_k=5, d=3):
    import torch
    from awebox_amd.ipm import DeviceNlp, StructuredKKT, _dense_A
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    st = hm.schedule(consts, lay, v0)[0]
    lbg, ubg = lay.g_bounds()
    nlp = DeviceNlp(evaluator(consts), pb.pack_p(lay, consts, v0, step=st.cost_step), st.lbx, st.ubx,
                    lbg, ubg, device)
    sk = StructuredKKT(nlp, lay, device)
    gen = torch.Generator().manual_seed(1)
    f64 = dict(dtype=torch.float64)
    hv = torch.randn(len(nlp.h_keep), generator=gen, **f64).to(device)
    jv = torch.randn(len(nlp.j_row), generator=gen, **f64).to(device)
    diag = (torch.rand(nlp.ny, generator=gen, **f64) + 1.0).to(device)
    N, ny = sk.N, nlp.ny
    K = torch.zeros(N, N, dtype=torch.float64, device=device)
    K[nlp.h_r, nlp.h_c] = hv
    K[nlp.h_c[nlp.h_offdiag], nlp.h_r[nlp.h_offdiag]] = hv[nlp.h_offdiag]
    i = torch.arange(ny, device=device)
    K[i, i] += diag
    _dense_A(nlp, jv, ny, K)
    rhs = torch.randn(N, generator=gen, **f64).to(device)
    return nlp, sk, hv, jv, diag, K, rhs


@pytest.mark.gpu
def test_structured_kkt_btd_on_gpu():
    """The GPU separator path (awelu block sweep + border) against the dense LU of the same KKT
    matrix, without refinement: the first elimination solve's backward error."""
    import torch
    from awebox_amd.evaluator import Ap2Evaluator
    nlp, sk, hv, jv, diag, K, rhs = _kkt_case("cuda", lambda c: Ap2Evaluator(c, batch=1))
    sk.factor(hv, diag, jv, 0.0, nlp.mI)
    assert sk.use_btd
    x = sk._solve(rhs)
    backward = (K @ x - rhs).abs().max().item() / (K.abs().sum(1).max().item() * x.abs().max().item()
                                                    + rhs.abs().max().item())
    x_ref = torch.linalg.solve(K.cpu(), rhs.cpu())
    fwd = (x.cpu() - x_ref).abs().max().item() / x_ref.abs().max().item()
    print(f"backward {backward:.3e} forward {fwd:.3e}")
    assert backward <= 1e-12
    assert fwd <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("separators", ["dense", "btd"])
def test_structured_kkt_bitwise_repeatable_on_gpu(separators):
    """Two factor + solve calls on identical inputs give bitwise-identical solutions (fixed-order
    assembly, Schur update and residual products: no atomics anywhere in the KKT solve)."""
    import torch
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import StructuredKKT
    nlp, sk, hv, jv, diag, K, rhs = _kkt_case("cuda", lambda c: Ap2Evaluator(c, batch=1))
    lay = pb.NlpLayout(5, 3)
    xs = []
    for _ in range(2):
        sk = StructuredKKT(nlp, lay, "cuda", separators=separators, deterministic=True)
        sk.factor(hv, diag, jv, 1e-9, nlp.mI)
        xs.append(sk.solve(rhs.clone()))
    assert torch.equal(xs[0], xs[1])


@pytest.mark.parametrize("delta_c,btd", [(0.0, False), (1e-6, False), (0.0, True), (1e-6, True)])
def test_structured_kkt_matches_dense(delta_c, btd):
    """Interval elimination + Schur complement solves the same KKT system as a dense LU; with
    btd=True the separators go through the bordered block-tridiagonal path (awebox_amd/btd.py,
    its host fallback), which the GPU solver uses."""
    import torch
    from oracle.cpu_device import CpuDeviceEvaluator
    from awebox_amd.ipm import DeviceNlp, StructuredKKT, _dense_A
    n_k, d = 5, 3
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    st = hm.schedule(consts, lay, v0)[0]
    lbg, ubg = lay.g_bounds()
    nlp = DeviceNlp(CpuDeviceEvaluator(consts), pb.pack_p(lay, consts, v0, step=st.cost_step), st.lbx, st.ubx,
                    lbg, ubg, "cpu")
    sk = StructuredKKT(nlp, lay, "cpu")
    assert sk.nS < sk.N // 4
    assert sk.btd is not None and sk.btd.nb == n_k + 1 and sk.btd.m == 2 * pb.NX and sk.btd.nG < 2 * pb.NX
    sk.force_btd = btd
    gen = torch.Generator().manual_seed(1)
    f64 = dict(dtype=torch.float64)
    hv = torch.randn(len(nlp.h_keep), generator=gen, **f64)
    jv = torch.randn(len(nlp.j_row), generator=gen, **f64)
    diag = torch.rand(nlp.ny, generator=gen, **f64) + 1.0
    N, ny = sk.N, nlp.ny
    K = torch.zeros(N, N, **f64)
    K[nlp.h_r, nlp.h_c] = hv
    K[nlp.h_c[nlp.h_offdiag], nlp.h_r[nlp.h_offdiag]] = hv[nlp.h_offdiag]
    i = torch.arange(ny)
    K[i, i] += diag
    _dense_A(nlp, jv, ny, K)
    if delta_c:
        K[torch.arange(ny, N), torch.arange(ny, N)] = -delta_c
    rhs = torch.randn(N, generator=gen, **f64)
    sk.factor(hv, diag, jv, delta_c, nlp.mI)
    x = sk.solve(rhs)
    assert sk.n_dense == 0 and sk.use_btd == btd
    backward = (K @ x - rhs).abs().max().item() / (K.abs().sum(1).max().item() * x.abs().max().item()
                                                    + rhs.abs().max().item())
    assert backward <= 1e-12
    x_ref = torch.linalg.solve(K, rhs)
    assert (x - x_ref).abs().max().item() <= 1e-6 * x_ref.abs().max().item()


def test_ipm_handles_fixed_variables_and_inequalities():
    """One solve with the final bounds from the initial guess, cold start."""
    from oracle.cpu_device import CpuDeviceEvaluator
    consts = pb.build_constants(pb.Ap2Config(n_k=4, d=2))
    lay = pb.NlpLayout(4, 2)
    v0 = initial_guess(consts, lay)
    st = hm.schedule(consts, lay, v0)[0]
    lbg, ubg = lay.g_bounds()
    res = solve(CpuDeviceEvaluator(consts), pb.pack_p(lay, consts, v0, step=st.cost_step), v0, st.lbx, st.ubx,
                lbg, ubg, opts=IpmOptions(max_iter=300), device="cpu")
    assert res.status == "solve_succeeded", res.status
    fixed = st.lbx >= st.ubx
    assert np.array_equal(res.x[fixed], st.lbx[fixed])
    g_ineq = lay.g_bounds()[0] == -np.inf
    assert res.constr_viol <= 1e-6


@pytest.mark.gpu
def test_homotopy_on_gpu_n10():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.build import build
    from awebox_amd.evaluator import Ap2Evaluator
    build()
    consts = pb.build_constants(pb.Ap2Config(n_k=10, d=4))
    lay = pb.NlpLayout(10, 4)
    V, summary, out, _ = optimize(consts, Ap2Evaluator(consts, batch=1), IpmOptions(max_iter=600))
    _check_solution(consts, lay, V, summary)


def _fake_point_solver(n_v):
    """Deterministic stand-in for a solve: V encodes u_ref and the number of warm starts."""
    def solve_point(u, prev):
        chain = 0 if prev is None else prev + 1
        V = np.full(n_v, u) + chain
        return V, {"avg_power_W": 1000.0 * u, "period_s": 30.0 + u}, 10 + chain, True, chain
    return solve_point


def _sweep_worker(rank, world, port, q, arch="single"):
    import os

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from awebox_amd.sweep import run_sweep
    if arch == "dual":
        from awebox_amd import dual as du
        n_v = du.layout_for(du.build_constants(du.MultiConfig(n_k=4, d=2))).n_v
    else:
        n_v = pb.NlpLayout(4, 2).n_v
    res = run_sweep([5.0, 5.5, 6.0, 6.5, 7.0], n_k=4, d=2, dist=dist, device="cpu",
                    point_solver=_fake_point_solver(n_v), arch=arch)
    if rank == 0:
        q.put({k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in res.items()})
    dist.destroy_process_group()


@pytest.mark.parametrize("arch", ["single", "dual"])
def test_sweep_collectives_over_two_ranks(arch):
    """world_size 2 over gloo: template broadcast, seeds scattered in contiguous blocks (3 + 2
    points, padded), solutions gathered to rank 0 in point order, warm-start chains per shard
    (AP2 and the dual-kite problem of config 4)."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sweep_worker, args=(r, 2, port, q, arch)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert res["world"] == 2
    assert res["u_ref"] == [5.0, 5.5, 6.0, 6.5, 7.0]
    assert res["iterations"] == [10, 11, 12, 10, 11]          # rank 0: 3 chained points, rank 1: 2
    V = np.asarray(res["V_opt"])
    assert np.array_equal(V[:, 0], np.array([5.0, 6.5, 8.0, 6.5, 8.0]))
    assert res["avg_power_W"] == [1000.0 * u for u in res["u_ref"]]


def test_sweep_single_process_warm_start_chain():
    from awebox_amd.sweep import run_sweep
    from oracle.cpu_device import CpuDeviceEvaluator
    res = run_sweep([10.0, 10.5], n_k=6, d=3, make_evaluator=CpuDeviceEvaluator, device="cpu",
                    opts=IpmOptions(max_iter=500))
    assert all(res["ok"]), res
    assert res["iterations"][1] < res["iterations"][0]        # the warm start is cheaper than the homotopy
    assert res["avg_power_W"][1] > 0


# test_batched_homotopy_matches_single_solves_on_cpu_port (rounds 2-5: a batch of three wind speeds
# within 1e-5 of three separate solves) is now tests/test_det.py's bitwise statement of the same
# property: batched and single solves return the same bits (det.py).


def test_watchdog_reaches_the_same_solution_on_cpu_port():
    """IPOPT's watchdog (IpmOptions.watchdog_*): with the trigger at one shortened step the watchdog
    runs in nearly every iteration of the homotopy -- full steps judged against its starting point,
    returns to that point after three failures -- and the homotopy still converges in every step to
    the solution of the default run."""
    from oracle.cpu_device import CpuDeviceEvaluator
    consts = pb.build_constants(pb.Ap2Config(n_k=4, d=2))
    ev = CpuDeviceEvaluator(consts)
    ref = optimize(consts, ev, IpmOptions(max_iter=400), device="cpu")
    got = optimize(consts, ev, IpmOptions(max_iter=400, watchdog_shortened_iter_trigger=1), device="cpu")
    for _, s, out, _ in (ref, got):
        assert all(r["status"] == "solve_succeeded" for r in s), s
    assert [r["iterations"] for r in ref[1]] != [r["iterations"] for r in got[1]]   # the watchdog ran
    assert abs(got[2]["avg_power_W"] - ref[2]["avg_power_W"]) <= 1e-6 * abs(ref[2]["avg_power_W"])
    assert abs(got[2]["period_s"] - ref[2]["period_s"]) <= 1e-6 * ref[2]["period_s"]


def test_kkt_structure_is_shared_by_evaluators_of_one_layout():
    """ipm._structure caches by layout and pattern: a second evaluator of the same problem (a sweep
    shard's batched warm start after its homotopy) reuses the StructuredKKT and the J^T / H products;
    another fixed-variable set gets its own."""
    from oracle.cpu_device import CpuDeviceEvaluator
    from awebox_amd.ipm import DeviceNlp, IpmOptions, _structure
    n_k, d = 4, 3
    consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
    lay = pb.NlpLayout(n_k, d)
    v0 = initial_guess(consts, lay)
    sched = hm.schedule(consts, lay, v0)
    lbg, ubg = lay.g_bounds()
    opts = IpmOptions()

    def struct(st):
        ev = CpuDeviceEvaluator(consts)
        nlp = DeviceNlp(ev, pb.pack_p(lay, consts, v0, step=st.cost_step), st.lbx, st.ubx, lbg, ubg, "cpu")
        return _structure(ev, nlp, "cpu", opts)

    a, b = struct(sched[-1]), struct(sched[-1])
    assert all(x is y for x, y in zip(a, b))
    c = struct(sched[0])
    if not np.array_equal(sched[0].lbx >= sched[0].ubx, sched[-1].lbx >= sched[-1].ubx):
        assert c[0] is not a[0]


def test_btd_merged_forward_sweep_matches_separate_solve():
    """btd.BorderedBtd._factor_blocks with the border columns E (the forward sweep of T^-1 E inside
    the factorisation's stages, then _t_backward) gives T^-1 E as the separate block solve does
    (host LAPACK path; on the device the two are bitwise equal)."""
    import torch
    from awebox_amd.btd import BorderedBtd
    rng = np.random.default_rng(5)
    B, nb, m, r = 2, 6, 7, 3
    T = torch.tensor(rng.normal(size=(B, nb, 3, m, m)) * 0.2)
    T[:, :, 1] += 3.0 * torch.eye(m, dtype=torch.float64)
    E = torch.tensor(rng.normal(size=(B, nb * m, r)))
    bt = BorderedBtd.__new__(BorderedBtd)
    bt.nb, bt.m, bt.B = nb, m, B
    Y = bt._factor_blocks(T, E.view(B, nb, m, r))
    merged = bt._t_backward(Y)
    bt.fused = False
    separate = bt._t_solve(E)
    np.testing.assert_allclose(merged.numpy(), separate.numpy(), rtol=1e-12, atol=1e-13)
    # and T^-1 E is what a dense solve of the block-tridiagonal matrix gives
    A = torch.zeros(B, nb * m, nb * m, dtype=torch.float64)
    for k in range(nb):
        for s_, dk in ((0, -1), (1, 0), (2, 1)):
            if 0 <= k + dk < nb:
                A[:, k * m:(k + 1) * m, (k + dk) * m:(k + dk + 1) * m] = T[:, k, s_]
    np.testing.assert_allclose(merged.numpy(), torch.linalg.solve(A, E).numpy(), rtol=1e-10, atol=1e-12)
