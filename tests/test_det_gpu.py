"""Batch-invariant reductions and products on MI355X (libawelu awelu_row_sum / awelu_bmm, det.py).

* the kernels return bitwise their elementwise restatement (det.py ``emulate=True``, the order
  DESIGN.md section 9 documents and tests/test_det.py checks against plain Python);
* a row or a matrix gives the same bits alone and inside any batch;
* the structured KKT factor + solve of the AP2 N=40 problem gives an instance the same bits alone and
  inside a batch of 3;
* a fan shard's batched warm-started final step (sweep.run_sweep mode "fan") gives every point the
  same bits whether its 8 points are solved as one batch or split 4 + 4, 2 + 2 + 2 + 2 or one by one
  -- the batches the 1-, 2-, 4- and 8-GPU partitions of an 8-point sweep give each rank."""
import numpy as np
import pytest
import torch

from awebox_amd import det

pytestmark = pytest.mark.gpu


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a machine without a visible GPU")
    from awebox_amd.build import LIB_LU, build_one
    build_one(LIB_LU)


def _spread(gen, shape):
    x = torch.randn(shape, generator=gen, dtype=torch.float64)
    return (x * torch.exp(torch.rand(shape, generator=gen, dtype=torch.float64) * 40 - 20)).cuda()


@pytest.mark.parametrize("n", [0, 1, 63, 256, 257, 1023, 12607])
def test_row_sum_kernel_is_its_restatement(n):
    _need_gpu()
    gen = torch.Generator().manual_seed(n)
    x = _spread(gen, (5, n))
    got = det.row_sum(x)
    assert torch.equal(got, det.row_sum(x, emulate=True))
    for r in range(5):
        assert torch.equal(det.row_sum(x[r:r + 1]), got[r:r + 1])
    # strided rows (a column slice) and a 3-D view
    if n > 2:
        assert torch.equal(det.row_sum(x[:, 1:]), det.row_sum(x[:, 1:], emulate=True))
    big = _spread(gen, (300, n))
    big[7] = x[2]
    assert torch.equal(det.row_sum(big)[7], got[2])


@pytest.mark.parametrize("M,N,K,transA", [(75, 75, 268, True), (75, 1, 268, True), (268, 1, 75, False),
                                          (100, 100, 100, False), (7, 3, 9, False), (33, 17, 1, True),
                                          (5, 40, 300, False)])
def test_bmm_kernel_is_its_restatement(M, N, K, transA):
    _need_gpu()
    gen = torch.Generator().manual_seed(M * 1000 + N)
    nb = 6
    A = _spread(gen, (nb, K, M)).transpose(1, 2) if transA else _spread(gen, (nb, M, K))
    B = _spread(gen, (nb, K, N))
    C = det.bmm(A, B)
    assert torch.equal(C, det.bmm(A, B, emulate=True))
    for b in range(nb):
        assert torch.equal(det.bmm(A[b:b + 1], B[b:b + 1]), C[b:b + 1])
    ref = (A.cpu() @ B.cpu())
    assert torch.allclose(C.cpu(), ref, rtol=1e-10, atol=1e-12 * float(ref.abs().max()))


def _kkt_inputs(nlp, B, seed):
    gen = torch.Generator().manual_seed(seed)
    f64 = dict(dtype=torch.float64)
    hv = torch.randn(B, len(nlp.h_keep), generator=gen, **f64).cuda()
    jv = torch.randn(B, len(nlp.j_row), generator=gen, **f64).cuda()
    diag = (torch.rand(B, nlp.ny, generator=gen, **f64) + 1.0).cuda()
    return hv, jv, diag


def test_structured_kkt_is_batch_invariant():
    """Factor + refined solve of the AP2 N=40 KKT for 3 different instances at once and for each
    alone: the same bits (interval LU, Schur products, block sweep, border, refinement residuals)."""
    _need_gpu()
    from awebox_amd import homotopy as hm
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import DeviceNlp, StructuredKKT
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    st = hm.schedule(consts, lay, v0)[-1]
    lbg, ubg = lay.g_bounds()
    P = pb.pack_p(lay, consts, v0, step=st.cost_step)
    B = 3
    nlp = DeviceNlp(Ap2Evaluator(consts, batch=B), np.tile(P, (B, 1)), st.lbx, st.ubx, lbg, ubg, "cuda")
    hv, jv, diag = _kkt_inputs(nlp, B, 5)
    rhs = torch.randn(B, nlp.ny + nlp.m, generator=torch.Generator().manual_seed(6), dtype=torch.float64).cuda()
    sk = StructuredKKT(nlp, lay, "cuda")
    sk.factor(hv, diag, jv, 1e-9, nlp.mI)
    assert sk.use_btd
    xb = sk.solve(rhs)
    inert_b = sk.inertia()
    for b in range(B):
        sk1 = StructuredKKT(nlp, lay, "cuda")
        sk1.factor(hv[b:b + 1], diag[b:b + 1], jv[b:b + 1], 1e-9, nlp.mI)
        x1 = sk1.solve(rhs[b:b + 1])
        assert torch.equal(x1[0], xb[b]), b
        assert torch.equal(sk1.inertia()[0], inert_b[b])


def test_fan_shard_warm_start_is_partition_invariant():
    """The fan sweep's batched warm start (sweep.run_sweep mode "fan": every point of a shard starts
    from the shard's first solution with the final homotopy step's costs and bounds) for 8 wind speeds
    around the AP2 N=40 default orbit, solved as one batch of 8, as 2 x 4, 4 x 2 and 8 x 1: every point
    returns the same V, multipliers and iteration count in every partition."""
    _need_gpu()
    from awebox_amd import homotopy as hm
    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import IpmOptions, solve_batch
    from awebox_amd.trajectory import hippo_options, optimize
    consts = pb.build_constants()
    lay = pb.NlpLayout(40, 4)
    v0 = initial_guess(consts, lay)
    ev1 = Ap2Evaluator(consts, batch=1)
    _, _, _, res0 = optimize(consts, ev1, IpmOptions(max_iter=2000))
    final = hm.schedule(consts, lay, v0)[-1]
    lbg, ubg = lay.g_bounds()
    us = np.linspace(9.0, 11.0, 8)
    opts = hippo_options("final", IpmOptions(max_iter=600))
    evs = {}

    def run(chunk):
        b = len(chunk)
        if b not in evs:
            evs[b] = Ap2Evaluator(consts, batch=b)
            evs[b].path = "colour"
        P = np.stack([pb.pack_p(lay, consts, v0, step=final.cost_step, u_ref=u) for u in chunk])
        return solve_batch(evs[b], P, np.tile(res0.x, (b, 1)), final.lbx, final.ubx, lbg, ubg,
                           lam0=np.tile(res0.lam_g, (b, 1)), zl0=np.tile(res0.zl, (b, 1)),
                           zu0=np.tile(res0.zu, (b, 1)), opts=opts)

    ref = run(us)
    assert all(r.status in ("solve_succeeded", "solved_to_acceptable_level") for r in ref), [r.status for r in ref]
    for per in (4, 2, 1):
        got = [r for i in range(0, 8, per) for r in run(us[i:i + per])]
        for i, (a, b) in enumerate(zip(ref, got)):
            assert a.iterations == b.iterations, (per, i, a.iterations, b.iterations)
            assert np.array_equal(a.x, b.x), (per, i)
            assert np.array_equal(a.lam_g, b.lam_g), (per, i)


def test_dual_fan_shard_warm_start_is_partition_invariant():
    """The same partition invariance for config 4's dual kites (N=20 d=4, the block recursion of
    100 x 100 separator blocks: det.bmm products and the awelu solve): rank 0's first 4 points of
    linspace(5, 8, 64) warm-started from the homotopy solution at the first point, solved as one batch
    of 4 and one by one, return the same V and iteration counts."""
    _need_gpu()
    from awebox_amd import dual as du
    from awebox_amd import dual_homotopy as dh
    from awebox_amd.ipm import IpmOptions, solve_batch
    from awebox_amd.trajectory import hippo_options
    consts = du.build_constants(du.MultiConfig(n_k=20, d=4))
    lay = du.layout_for(consts)
    v0 = du.initial_guess(consts, lay)
    us = np.linspace(5.0, 8.0, 64)[:5]
    ev1 = dh.make_evaluator(consts, batch=1)
    _, _, _, res0 = dh.optimize(consts, ev1, IpmOptions(max_iter=3000), v_init=v0, u_ref=float(us[0]))
    final = dh.schedule(consts, lay, v0)[-1]
    lbg, ubg = lay.g_bounds()
    opts = hippo_options("final", IpmOptions(max_iter=3000))
    evs = {1: ev1}

    def run(chunk):
        b = len(chunk)
        if b not in evs:
            evs[b] = dh.make_evaluator(consts, batch=b)
        P = np.stack([du.pack_p(lay, consts, v0, step=final.cost_step, u_ref=u) for u in chunk])
        return solve_batch(evs[b], P, np.tile(res0.x, (b, 1)), final.lbx, final.ubx, lbg, ubg,
                           lam0=np.tile(res0.lam_g, (b, 1)), zl0=np.tile(res0.zl, (b, 1)),
                           zu0=np.tile(res0.zu, (b, 1)), opts=opts)

    ref = run(us[1:])
    assert all(r.status in ("solve_succeeded", "solved_to_acceptable_level") for r in ref), [r.status for r in ref]
    got = [run(us[i:i + 1])[0] for i in range(1, 5)]
    for i, (a, b) in enumerate(zip(ref, got)):
        assert a.iterations == b.iterations, (i, a.iterations, b.iterations)
        assert np.array_equal(a.x, b.x), i


def test_batch_mode_sweep_is_partition_invariant():
    """The sweep's "batch" mode (every point its own full homotopy from the standard initial guess,
    the shard's points side by side: sweep.run_sweep) on 4 AP2 N=40 points of config 4's grid, as one
    shard of 4 (one GPU), two shards of 2 (two GPUs) and four shards of 1 (four GPUs): every point
    returns bitwise the same V and iteration count -- a 1/2/4/8-GPU sweep compares the same answers."""
    _need_gpu()
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    u = np.linspace(5.0, 8.0, 64)[[0, 9, 18, 27]]
    mk = lambda c, b=1: Ap2Evaluator(c, batch=b)  # noqa: E731

    def sweep(points):
        return run_sweep(points, n_k=40, d=4, make_evaluator=mk, device="cuda", opts=IpmOptions(max_iter=2000),
                         mode="batch")
    ref = sweep(u)
    assert all(ref["ok"]), ref
    for per in (2, 1):
        parts = [sweep(u[i:i + per]) for i in range(0, 4, per)]
        V = np.concatenate([np.asarray(p["V_opt"]) for p in parts])
        its = [i for p in parts for i in p["iterations"]]
        assert its == ref["iterations"], (per, its, ref["iterations"])
        assert np.array_equal(V, np.asarray(ref["V_opt"])), per
