"""Joining sweep shards into the reference's single chain (sweep.reconcile_shard, run_sweep's
``reconcile``; awebox/sweep.py:148-172 solves every point warm-started from the previous one).

* the decision logic with a stand-in solver: a shard whose re-solved first two points reach the same
  optimum as its own chain keeps the rest of it; one that does not is re-chained from the re-solved
  points, and the flag passed on says whether the shard's last solution changed;
* two gloo ranks on the CPU harness (AP2 N=4 d=2, 2 + 2 points): rank 1's points equal the
  single-process chain's bitwise (they ARE the chain's warm starts from rank 0's last point), and
  every point matches the chain's power."""
import numpy as np
import pytest

from awebox_amd.sweep import SAME_OPTIMUM_RTOL, reconcile_shard, same_optimum


def _fake(offset_family):
    """solve_warm stand-in: the 'power' is u plus the family of the warm start (state[0][0])."""
    def solve_warm(u, state):
        fam = state[0][0]
        st = (np.array([fam]), None, None, None)
        return st, {"avg_power_W": 1000.0 * u + fam, "period_s": 30.0 + fam}, 7, True
    return solve_warm


def test_same_optimum():
    a = {"avg_power_W": 5000.0, "period_s": 35.0}
    assert same_optimum(a, {"avg_power_W": 5000.0 * (1 + 0.5 * SAME_OPTIMUM_RTOL), "period_s": 35.0})
    assert not same_optimum(a, {"avg_power_W": 5000.0 * (1 + 3 * SAME_OPTIMUM_RTOL), "period_s": 35.0})
    assert not same_optimum(a, {"avg_power_W": 5000.0, "period_s": 36.0})
    assert not same_optimum(a, {"avg_power_W": float("nan"), "period_s": 35.0})


def test_reconcile_keeps_a_merged_shard_and_rechains_a_different_one():
    us = [1.0, 2.0, 3.0, 4.0]
    solve_warm = _fake(0)
    fam0 = (np.array([0.0]),) + (None,) * 3

    def shard():
        states = [fam0 for _ in us]
        outs = [{"avg_power_W": 1000.0 * u, "period_s": 30.0} for u in us]
        return states, outs, [50, 9, 9, 9], [True] * 4
    # the previous shard ends on the shard's own family: the first two points re-solved, the rest kept
    states, outs, iters, oks = shard()
    changed = reconcile_shard(solve_warm, us, states, outs, iters, oks, fam0, False)
    assert not changed and iters == [7, 7, 9, 9]
    # the previous shard ends on family 5: the second re-solved point differs -> the rest re-chained
    states, outs, iters, oks = shard()
    changed = reconcile_shard(solve_warm, us, states, outs, iters, oks, (np.array([5.0]),) + (None,) * 3, False)
    assert changed and iters == [7, 7, 7, 7]
    assert [o["avg_power_W"] for o in outs] == [1005.0, 2005.0, 3005.0, 4005.0]
    # speculative re-solves are used only when the predecessor did not change
    spec = [((np.array([0.0]),) + (None,) * 3, {"avg_power_W": 1000.0, "period_s": 30.0}, 3, True),
            ((np.array([0.0]),) + (None,) * 3, {"avg_power_W": 2000.0, "period_s": 30.0}, 3, True)]
    states, outs, iters, oks = shard()
    reconcile_shard(solve_warm, us, states, outs, iters, oks, fam0, False, spec=spec)
    assert iters == [3, 3, 9, 9]
    states, outs, iters, oks = shard()
    reconcile_shard(solve_warm, us, states, outs, iters, oks, fam0, True, spec=spec)
    assert iters == [7, 7, 9, 9]                                # re-solved from pred_state, spec ignored


def _worker(rank, world, port, q, us):
    import os

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    from oracle.cpu_device import CpuDeviceEvaluator
    res = run_sweep(us, n_k=4, d=2, make_evaluator=lambda c, b=1: CpuDeviceEvaluator(c), dist=dist, device="cpu",
                    opts=IpmOptions(max_iter=400), mode="chain", reconcile=True)
    if rank == 0:
        q.put({k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in res.items()})
    dist.destroy_process_group()


def test_reconciled_shards_follow_the_single_chain_on_cpu():
    import socket

    import torch.multiprocessing as mp
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    from oracle.cpu_device import CpuDeviceEvaluator
    us = [9.5, 10.0, 10.5, 11.0]
    chain = run_sweep(us, n_k=4, d=2, make_evaluator=lambda c, b=1: CpuDeviceEvaluator(c), device="cpu",
                      opts=IpmOptions(max_iter=400), mode="chain")
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, us)) for r in range(2)]
    # two solver processes on the container's CPUs: each with a few threads (8 threads each
    # oversubscribe the cores and the OpenMP/MKL pools spin; torch.set_num_threads inside a process
    # trips an MKL fault in dlaswp here, so the limit goes in through the environment at spawn)
    import os
    saved = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "MKL_NUM_THREADS")}
    os.environ.update(OMP_NUM_THREADS="2", MKL_NUM_THREADS="2")
    try:
        for p in procs:
            p.start()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=60)
    assert all(res["ok"]), res
    V, Vc = np.asarray(res["V_opt"]), np.asarray(chain["V_opt"])
    assert np.array_equal(V[0], Vc[0]) and np.array_equal(V[1], Vc[1])   # rank 0's shard is the chain's start
    assert np.array_equal(V[2], Vc[2]) and np.array_equal(V[3], Vc[3])   # rank 1: re-solved as the chain solves them
    for i in range(4):
        assert abs(res["avg_power_W"][i] - chain["avg_power_W"][i]) <= SAME_OPTIMUM_RTOL * abs(chain["avg_power_W"][i]) * 3
