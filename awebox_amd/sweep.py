"""Wind-speed sweeps of the power cycle, sharded across GPUs: the AP2
single kite (``arch='single'``) and the dual kites of config 4 (``arch='dual'``,
examples/dual_kites_power_curve.py).

The reference sweeps the trial over ``user_options.wind.u_ref`` sequentially, warm-starting each
point from the previous one (awebox/sweep.py:120-163, examples/dual_kites_power_curve.py:48-52).
Only ``P.theta0.wind.u_ref`` changes between points; the NLP (layout, scaling, bounds) is built
once.  Here the points are independent work items, one process per GPU:

* rank 0 builds the problem template (model constants + initial guess) and broadcasts it
  (RCCL over xGMI when the backend is nccl, ~0.2 MB);
* the u_ref seeds are scattered: rank r gets the contiguous block [r*P/N, (r+1)*P/N);
* each rank runs the full homotopy for its first point and warm-starts every further point of
  its block from the previous solution (the reference's sweeping warm start), with the final
  homotopy step's costs and bounds;
* the optimal V and the per-point outputs are gathered to rank 0.

There is no data-path collective: evaluation and solves never leave the rank's GPU.

Launch: ``python -m torch.distributed.run --nproc-per-node N -m awebox_amd.sweep --points 64``
(or plain ``python -m awebox_amd.sweep`` for one GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import time

import numpy as np
import torch

from . import homotopy as hm
from . import problem as pb
from .initial_guess import initial_guess
from .ipm import IpmOptions, solve, solve_batch
from .trajectory import hippo_options, optimize

N_OUT = 6   # u_ref, avg power, period, iterations, status ok, seconds


class _Ap2:
    """The AP2 single-kite problem behind the sweep (problem.py, homotopy.py, trajectory.py)."""

    def __init__(self, n_k, d):
        self.consts = pb.build_constants(pb.Ap2Config(n_k=n_k, d=d))
        self.lay = pb.NlpLayout(n_k, d)
        self.nconst = pb.NCONST

    def initial_guess(self):
        return initial_guess(self.consts, self.lay)

    def final_step(self, v0):
        return hm.schedule(self.consts, self.lay, v0)[-1]

    def pack_p(self, v0, step, u):
        return pb.pack_p(self.lay, self.consts, v0, step=step, u_ref=u)

    def outputs(self, V):
        return hm.outputs(self.consts, self.lay, V)

    def optimize(self, ev, opts, device, v0, u):
        return optimize(self.consts, ev, opts, device=device, v_init=v0, u_ref=u)

    def optimize_batch(self, ev, opts, device, v0, us, verbose=False):
        from .trajectory import optimize_batch
        return optimize_batch(self.consts, ev, us, opts, device=device, v_init=v0, verbose=verbose)


class _Dual:
    """The dual-kite problem of config 4 (dual.py, dual_homotopy.py)."""

    def __init__(self, n_k, d):
        from . import dual as du
        self.du = du
        self.consts = du.build_constants(du.MultiConfig(n_k=n_k, d=d))
        self.lay = du.layout_for(self.consts)
        self.nconst = du.NCONST

    def initial_guess(self):
        return self.du.initial_guess(self.consts, self.lay)

    def final_step(self, v0):
        from . import dual_homotopy as dh
        return dh.schedule(self.consts, self.lay, v0)[-1]

    def pack_p(self, v0, step, u):
        return self.du.pack_p(self.lay, self.consts, v0, step=step, u_ref=u)

    def outputs(self, V):
        from . import dual_homotopy as dh
        return dh.outputs(self.consts, self.lay, V)

    def optimize(self, ev, opts, device, v0, u):
        from . import dual_homotopy as dh
        return dh.optimize(self.consts, ev, opts, device=device, v_init=v0, u_ref=u)

    def optimize_batch(self, ev, opts, device, v0, us, verbose=False):
        from . import dual_homotopy as dh
        return dh.optimize_batch(self.consts, ev, us, opts, device=device, v_init=v0, verbose=verbose)


def run_sweep(u_refs, n_k=40, d=4, make_evaluator=None, dist=None, device="cuda", opts: IpmOptions | None = None,
              verbose=False, point_solver=None, arch="single", mode="chain", reconcile=True, coll_device=None,
              return_states=False):
    """Returns (on rank 0) dict with per-point outputs, V_opt [P, n_v] and timing; None elsewhere.

    mode "chain": the reference's sweeping warm start within a shard -- the homotopy for the
    shard's first point, then the warm-started final step for each next point;
    ``point_solver(u, prev) -> (V, outputs, iterations, ok, prev)`` replaces the per-point solve.
    With ``reconcile`` (chain mode, more than one rank) the shards are then joined into the
    reference's single chain (awebox/sweep.py:148-172: every point warm-started from the previous
    point's solution): rank r re-solves its first point warm-started from rank r-1's last solution
    (one point-to-point message of that solution), keeps its shard if the re-solved point is the same
    optimum as its own homotopy's (``same_optimum``) and re-chains its shard from the re-solved point
    otherwise (see reconcile_shard).
    mode "batch": the shard's points are independent trials solved side by side, the full homotopy
    from the standard initial guess for every point as one batched interior-point solve per step
    (``make_evaluator(consts, batch)``).
    mode "fan": the homotopy for the shard's first point, then the other points warm-started from
    its solution in one batched final-step solve.
    ``return_states`` (one process): the result also holds every point's (x, lam_g, zl, zu) under
    "states" (chain mode), the problem under "problem" and the template initial guess under "v0"."""
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    coll_dev = torch.device(coll_device or device)
    prob = _Dual(n_k, d) if arch == "dual" else _Ap2(n_k, d)
    consts, lay, nconst = prob.consts, prob.lay, prob.nconst
    n_pts = len(u_refs)
    per = -(-n_pts // world)

    # ---- template broadcast: model constants + initial guess (rank 0 -> all) ----------------
    tmpl = torch.zeros(nconst + lay.n_v, dtype=torch.float64, device=coll_dev)
    if rank == 0:
        tmpl[:nconst] = torch.tensor(consts.consts)
        tmpl[nconst:] = torch.tensor(prob.initial_guess())
    if dist is not None:
        dist.broadcast(tmpl, src=0)
    consts.consts = tmpl[:nconst].cpu().numpy().copy()
    v0 = tmpl[nconst:].cpu().numpy().copy()

    # ---- seed scatter ---------------------------------------------------------------------------
    seeds = torch.full((per,), float("nan"), dtype=torch.float64, device=coll_dev)
    if dist is not None:
        chunks = None
        if rank == 0:
            padded = np.full(per * world, np.nan)
            padded[:n_pts] = u_refs
            chunks = [torch.tensor(padded[r * per:(r + 1) * per], device=coll_dev) for r in range(world)]
        dist.scatter(seeds, chunks, src=0)
    else:
        seeds[:n_pts] = torch.tensor(np.asarray(u_refs, dtype=np.float64))
    my_u = [u for u in seeds.cpu().numpy() if np.isfinite(u)]

    # ---- local solves ---------------------------------------------------------------------------
    point_solver_is_default = point_solver is None
    if point_solver is None and mode == "chain":
        ev = make_evaluator(consts)
        final = prob.final_step(v0)
        lbg, ubg = lay.g_bounds()
        done = ("solve_succeeded", "solved_to_acceptable_level")

        def point_solver(u, prev):
            if prev is None:
                V, summary, out, res = prob.optimize(ev, opts, device, v0, u)
                return V, out, sum(r["iterations"] for r in summary), all(r["status"] in done for r in summary), res
            P = prob.pack_p(v0, final.cost_step, u)
            res = solve(ev, P, prev.x, final.lbx, final.ubx, lbg, ubg, lam0=prev.lam_g, zl0=prev.zl, zu0=prev.zu,
                        opts=hippo_options("final", opts), device=device)
            return res.x, prob.outputs(res.x), res.iterations, res.status in done, res

    states = [None] * per          # (x, lam_g, zl, zu) of every local point: the reconciliation's warm starts
    res_v = torch.zeros(per, lay.n_v, dtype=torch.float64, device=coll_dev)
    res_o = torch.full((per, N_OUT), float("nan"), dtype=torch.float64, device=coll_dev)
    prev = None
    t_rank = time.perf_counter()
    done = ("solve_succeeded", "solved_to_acceptable_level")
    failures = (RuntimeError, ValueError, FloatingPointError, ArithmeticError)

    def fail(rows, us, exc):
        # a failed solve must not leave the other ranks waiting in the gather below: its points
        # are reported with ok = False and NaN outputs
        print(f"[rank {rank}] u_ref={[round(float(u), 3) for u in us]} failed: {exc}", flush=True)
        for i, u in zip(rows, us):
            res_v[i] = torch.tensor(v0, device=coll_dev)
            res_o[i] = torch.tensor([u, float("nan"), float("nan"), 0.0, 0.0, float("nan")], device=coll_dev)

    def run_batch(rows, us):
        """Independent trials side by side: the full homotopy for every point of ``us``."""
        t0 = time.perf_counter()
        try:
            evb = make_evaluator(consts, len(us))
            Vb, summary, outs, _ = prob.optimize_batch(evb, opts, device, v0, us, verbose=verbose)
        except failures as exc:
            fail(rows, us, exc)
            return
        el = time.perf_counter() - t0
        for i, (row, u) in enumerate(zip(rows, us)):
            iters = sum(r["iterations"][i] for r in summary)
            ok = all(r["status"][i] in done for r in summary)
            res_v[row] = torch.tensor(Vb[i], device=coll_dev)
            res_o[row] = torch.tensor([u, outs[i]["avg_power_W"], outs[i]["period_s"], iters, float(ok), el],
                                      device=coll_dev)
            if verbose:
                print(f"[rank {rank}] u_ref={u:.3f} P={outs[i]['avg_power_W']:.1f} W T={outs[i]['period_s']:.2f} s "
                      f"iters={iters} ok={ok}", flush=True)

    if mode == "fan" and my_u:
        # the reference's sweeping warm start, fanned out: the shard's first point runs the full
        # homotopy, then every other point of the shard is warm-started from that solution (the
        # final homotopy step's costs and bounds), all of them in one batched solve.  If the first
        # point does not converge, the rest run as independent batched homotopies instead.
        t0 = time.perf_counter()
        res0, ok0 = None, False
        try:
            ev1 = make_evaluator(consts, 1)
            V0, summary, out0, res0 = prob.optimize(ev1, opts, device, v0, my_u[0])
            del ev1
            it0 = sum(r["iterations"] for r in summary)
            ok0 = all(r["status"] in done for r in summary)
            el0 = time.perf_counter() - t0
            res_v[0] = torch.tensor(V0, device=coll_dev)
            res_o[0] = torch.tensor([my_u[0], out0["avg_power_W"], out0["period_s"], it0, float(ok0), el0],
                                    device=coll_dev)
            if verbose:
                print(f"[rank {rank}] u_ref={my_u[0]:.3f} P={out0['avg_power_W']:.1f} W T={out0['period_s']:.2f} s "
                      f"iters={it0} ok={ok0} {el0:.1f} s", flush=True)
                if res0.timing:
                    print(f"[rank {rank}] first point, final step timing {res0.timing}", flush=True)
        except failures as exc:
            fail([0], my_u[:1], exc)
        rest = my_u[1:]
        if rest and not ok0:
            run_batch(list(range(1, len(my_u))), rest)
        elif rest:
            t1 = time.perf_counter()
            final = prob.final_step(v0)
            lbg, ubg = lay.g_bounds()
            rb = len(rest)
            try:
                evb = make_evaluator(consts, rb)
                P = np.stack([prob.pack_p(v0, final.cost_step, u) for u in rest])
                res = solve_batch(evb, P, np.tile(res0.x, (rb, 1)), final.lbx, final.ubx, lbg, ubg,
                                  lam0=np.tile(res0.lam_g, (rb, 1)), zl0=np.tile(res0.zl, (rb, 1)),
                                  zu0=np.tile(res0.zu, (rb, 1)), opts=hippo_options("final", opts), device=device)
            except failures as exc:
                fail(list(range(1, len(my_u))), rest, exc)
                res = None
            el1 = time.perf_counter() - t1
            if res is not None:
                if verbose and res[0].timing:
                    print(f"[rank {rank}] batched warm start timing {res[0].timing}", flush=True)
                for i, (u, r) in enumerate(zip(rest, res)):
                    out = prob.outputs(r.x)
                    res_v[1 + i] = torch.tensor(r.x, device=coll_dev)
                    res_o[1 + i] = torch.tensor([u, out["avg_power_W"], out["period_s"], r.iterations,
                                                 float(r.status in done), el1], device=coll_dev)
                    if verbose:
                        print(f"[rank {rank}] u_ref={u:.3f} P={out['avg_power_W']:.1f} W T={out['period_s']:.2f} s "
                              f"iters={r.iterations} ok={r.status in done} (batched warm start, {el1:.1f} s)",
                              flush=True)
        my_u = []
    if mode == "batch" and my_u:
        run_batch(list(range(len(my_u))), my_u)
        my_u = []
    for i, u in enumerate(my_u):
        t0 = time.perf_counter()
        try:
            V, out, iters, ok, prev = point_solver(u, prev)
        except failures as exc:
            # a failed point must not leave the other ranks waiting in the gather below
            print(f"[rank {rank}] u_ref={u:.3f} failed: {exc}", flush=True)
            V, out, iters, ok, prev = v0, {"avg_power_W": float("nan"), "period_s": float("nan")}, 0, False, None
        res_v[i] = torch.tensor(V, device=coll_dev)
        res_o[i] = torch.tensor([u, out["avg_power_W"], out["period_s"], iters, float(ok),
                                 time.perf_counter() - t0], device=coll_dev)
        if prev is not None and hasattr(prev, "lam_g"):
            states[i] = (prev.x, prev.lam_g, prev.zl, prev.zu)
        if verbose:
            print(f"[rank {rank}] u_ref={u:.3f} P={out['avg_power_W']:.1f} W T={out['period_s']:.2f} s "
                  f"iters={iters} ok={ok} {time.perf_counter() - t0:.1f} s", flush=True)
    if reconcile and mode == "chain" and dist is not None and world > 1 and make_evaluator is not None \
            and point_solver_is_default:
        _reconcile_ranks(dist, rank, world, prob, ev, opts, device, v0, seeds.cpu().numpy(), states, res_v, res_o,
                         coll_dev, verbose)
    t_rank = time.perf_counter() - t_rank

    # ---- gather to rank 0 -----------------------------------------------------------------------
    if dist is not None:
        gv = [torch.zeros_like(res_v) for _ in range(world)] if rank == 0 else None
        go = [torch.zeros_like(res_o) for _ in range(world)] if rank == 0 else None
        dist.gather(res_v, gv, dst=0)
        dist.gather(res_o, go, dst=0)
        t = torch.tensor([t_rank], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_rank = float(t.item())
        if rank != 0:
            return None
        V_all = torch.cat(gv).cpu().numpy()
        O_all = torch.cat(go).cpu().numpy()
    else:
        V_all, O_all = res_v.cpu().numpy(), res_o.cpu().numpy()
    keep = np.isfinite(O_all[:, 0])
    O_all, V_all = O_all[keep], V_all[keep]
    extra = {}
    if return_states and dist is None:
        extra = {"states": states[:len(O_all)], "problem": prob, "v0": v0}
    return {**extra, "u_ref": O_all[:, 0].tolist(), "avg_power_W": O_all[:, 1].tolist(), "period_s": O_all[:, 2].tolist(),
            "iterations": O_all[:, 3].astype(int).tolist(), "ok": O_all[:, 4].astype(bool).tolist(),
            "seconds": O_all[:, 5].tolist(), "V_opt": V_all, "wall_s": t_rank, "world": world,
            "trials_per_s": len(O_all) / t_rank}


SAME_OPTIMUM_RTOL = 1e-4      # relative power and period difference of two solutions of one optimum


def same_optimum(out_a, out_b, rtol=SAME_OPTIMUM_RTOL) -> bool:
    """Whether two converged solutions of one sweep point are the same local optimum: average power
    and period agree to ``rtol`` (a different orbit family differs by percents; a different KKT point
    of a flat optimum reached from another warm start by 1e-3 -- profiles/r05/config4/compare.json)."""
    pa, pb = out_a["avg_power_W"], out_b["avg_power_W"]
    ta, tb = out_a["period_s"], out_b["period_s"]
    if not all(np.isfinite(v) for v in (pa, pb, ta, tb)):
        return False
    return abs(pa - pb) <= rtol * abs(pb) and abs(ta - tb) <= rtol * abs(tb)


def warm_point_solver(prob, ev, opts, device, v0):
    """solve(u, state) -> (state, outputs, iterations, ok): the reference's sweeping warm start of one
    point (the final homotopy step's costs and bounds, multipliers kept)."""
    final = prob.final_step(v0)
    lbg, ubg = prob.lay.g_bounds()
    done = ("solve_succeeded", "solved_to_acceptable_level")

    def solve_warm(u, state):
        x, lam, zl, zu = state
        P = prob.pack_p(v0, final.cost_step, u)
        r = solve(ev, P, x, final.lbx, final.ubx, lbg, ubg, lam0=lam, zl0=zl, zu0=zu,
                  opts=hippo_options("final", opts), device=device)
        return (r.x, r.lam_g, r.zl, r.zu), prob.outputs(r.x), r.iterations, r.status in done
    return solve_warm


def reconcile_shard(solve_warm, us, states, outs, iters, oks, pred_state, pred_changed, spec=None, depth=2):
    """Join one shard to the chain of the shards before it (the reference solves the sweep as one
    chain, awebox/sweep.py:148-172).  ``pred_state``: the final solution of the previous shard's last
    point.  The shard's first ``depth`` points are re-solved as the chain solves them -- the first
    warm-started from ``pred_state``, each next one from the one before (``spec``: those re-solves,
    done beforehand from the previous shard's own last point, valid when ``pred_changed`` is False).
    If the last re-solved point is the same optimum as the shard's own (same_optimum), the chains have
    merged and the rest of the shard stands; otherwise the rest is re-chained from the re-solved points.
    (One point is not enough: a shard's first point comes from its own homotopy and can sit 1e-3 off
    the chain's on a flat optimum even where the next warm start already agrees to 1e-5,
    profiles/r06/config4/.)  Lists are updated in place; returns whether the shard's last solution
    changed."""
    depth = max(1, min(depth, len(us)))
    if spec is None or pred_changed:
        spec, st = [], pred_state
        for i in range(depth):
            spec.append(solve_warm(us[i], st))
            st = spec[-1][0]
    keep = all(r[3] for r in spec) and oks[depth - 1] and same_optimum(spec[-1][1], outs[depth - 1])
    for i, r in enumerate(spec):
        states[i], outs[i], iters[i], oks[i] = r
    if keep:
        return depth == len(us)
    for i in range(depth, len(us)):
        states[i], outs[i], iters[i], oks[i] = solve_warm(us[i], states[i - 1])
    return True


def speculate(solve_warm, us, pred_state, depth=2):
    """reconcile_shard's re-solves from a predecessor's (possibly provisional) last solution."""
    out, st = [], pred_state
    for i in range(max(1, min(depth, len(us)))):
        out.append(solve_warm(us[i], st))
        st = out[-1][0]
    return out


def _pack_state(state, n_v, n_g, dev, flag=0.0):
    t = torch.zeros(1 + 3 * n_v + n_g, dtype=torch.float64, device=dev)
    t[0] = flag
    if state is not None:
        x, lam, zl, zu = state
        t[1:1 + n_v] = torch.as_tensor(x)
        t[1 + n_v:1 + n_v + n_g] = torch.as_tensor(lam)
        t[1 + n_v + n_g:1 + 2 * n_v + n_g] = torch.as_tensor(zl)
        t[1 + 2 * n_v + n_g:] = torch.as_tensor(zu)
    return t


def _unpack_state(t, n_v, n_g):
    a = t.cpu().numpy()
    return float(a[0]), (a[1:1 + n_v].copy(), a[1 + n_v:1 + n_v + n_g].copy(),
                         a[1 + n_v + n_g:1 + 2 * n_v + n_g].copy(), a[1 + 2 * n_v + n_g:].copy())


_NO_STATE = 2.0        # message flag: the sender has no usable last solution (0: unchanged, 1: changed)


def _reconcile_ranks(dist, rank, world, prob, ev, opts, device, v0, seeds, states, res_v, res_o, coll_dev, verbose):
    """reconcile_shard across the ranks, with the first re-solves speculative and parallel: every rank
    sends its last solution to the next rank and re-solves its first points from the one it receives
    (all ranks at once); then, in rank order, each rank learns whether the previous shard's last
    solution changed (re-solving again only then), keeps or re-chains its shard, and passes the flag and
    its final last solution on.  Only point-to-point messages of one solution between neighbours.
    Every rank takes part in both message rounds whatever happens locally -- a rank without points
    forwards its predecessor's messages, a failed solve passes a flag instead of a solution -- so no
    rank waits forever on a neighbour."""
    n_v, n_g = prob.lay.n_v, int(len(prob.lay.g_bounds()[0]))
    failures = (RuntimeError, ValueError, FloatingPointError, ArithmeticError)
    us = [float(u) for u in seeds if np.isfinite(u)]
    n = len(us)
    t0 = time.perf_counter()
    solve_warm = warm_point_solver(prob, ev, opts, device, v0)
    outs = [{"avg_power_W": float(res_o[i, 1]), "period_s": float(res_o[i, 2])} for i in range(n)]
    iters = [int(res_o[i, 3]) for i in range(n)]
    oks = [bool(res_o[i, 4] > 0) for i in range(n)]
    sts = list(states[:n])
    valid = n > 0 and all(st is not None for st in sts)
    my_last = sts[-1] if valid else None
    recv = lambda: _unpack_state(_recv(dist, _pack_state(None, n_v, n_g, coll_dev), rank - 1), n_v, n_g)  # noqa: E731
    # speculative phase: last solution -> next rank, first points re-solved from the previous rank's
    spec = None
    if n > 0:
        reqs = []
        if rank + 1 < world:
            reqs.append(dist.isend(_pack_state(my_last, n_v, n_g, coll_dev, 0.0 if valid else _NO_STATE), dst=rank + 1))
        if rank > 0:
            flag, pred_spec = recv()
            if valid and flag != _NO_STATE:
                try:
                    spec = speculate(solve_warm, us, pred_spec)
                except failures as exc:
                    print(f"[rank {rank}] speculative re-solve failed: {exc}", flush=True)
        for rq in reqs:
            rq.wait()
    elif rank > 0:                                          # no points: the predecessor's state passes on
        flag, pred_spec = recv()
        if rank + 1 < world:
            dist.send(_pack_state(pred_spec, n_v, n_g, coll_dev, flag), dst=rank + 1)
    # sequential phase, in rank order
    changed, out_flag, out_state = False, (0.0 if valid else _NO_STATE), my_last
    if rank > 0:
        flag, pred_final = recv()
        if n == 0:
            out_flag, out_state = flag, pred_final
        elif valid and flag != _NO_STATE:
            try:
                changed = reconcile_shard(solve_warm, us, sts, outs, iters, oks, pred_final, flag == 1.0, spec=spec)
            except failures as exc:
                print(f"[rank {rank}] reconciliation failed, shard kept: {exc}", flush=True)
                changed = True
            out_flag, out_state = (1.0 if changed else 0.0), sts[-1]
    if rank + 1 < world:
        dist.send(_pack_state(out_state, n_v, n_g, coll_dev, out_flag if out_state is not None else _NO_STATE),
                  dst=rank + 1)
    el = time.perf_counter() - t0
    for i in range(n):
        if sts[i] is not None:
            res_v[i] = torch.as_tensor(sts[i][0], device=coll_dev)
        res_o[i, 1], res_o[i, 2] = outs[i]["avg_power_W"], outs[i]["period_s"]
        res_o[i, 3], res_o[i, 4] = iters[i], float(oks[i])
    if verbose:
        print(f"[rank {rank}] reconciled with the previous shard: {'re-chained' if changed else 'kept'} "
              f"({el:.1f} s)", flush=True)


def _recv(dist, buf, src):
    dist.recv(buf, src=src)
    return buf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=64)
    ap.add_argument("--arch", choices=["single", "dual"], default="single",
                    help="single: AP2 power curve; dual: dual-kite power curve (config 4)")
    ap.add_argument("--u-min", type=float, default=5.0)
    ap.add_argument("--u-max", type=float, default=8.0)
    ap.add_argument("--n-k", type=int, default=40)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--max-iter", type=int, default=600)
    ap.add_argument("--out", default="gpurun_out/sweep.json")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--ipm-verbose", action="store_true", help="print every interior-point iteration")
    ap.add_argument("--profile", action="store_true", help="phase timings of the interior-point solver")
    ap.add_argument("--separators", choices=["dense", "btd"], default="btd",
                    help="separator solve of the structured KKT (awebox_amd/btd.py for btd)")
    ap.add_argument("--mode", choices=["chain", "batch", "fan"], default="chain",
                    help="chain (default): the reference's sweeping warm start (sweep.py:154-172) within each "
                         "shard; batch: independent trials, the shard's points as one batched homotopy; fan "
                         "(throughput, opt-in): homotopy for the first point, batched warm start for the rest -- "
                         "results then depend on how the points are sharded")
    ap.add_argument("--grid", type=int, default=0,
                    help="take the points from linspace(u-min, u-max, GRID) (config 4: 64), the first --points of it")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    from .build import build
    from .evaluator import Ap2Evaluator
    if local_rank == 0:
        build()
    if dist is not None:
        dist.barrier()
    u = np.linspace(args.u_min, args.u_max, args.points)
    if args.grid:
        u = np.linspace(args.u_min, args.u_max, args.grid)[:args.points]
    if args.arch == "dual":
        from .dual_homotopy import make_evaluator
        mk = lambda c, b=1: make_evaluator(c, device=f"cuda:{local_rank}", batch=b)  # noqa: E731
    else:
        mk = lambda c, b=1: Ap2Evaluator(c, batch=b)  # noqa: E731
    res = run_sweep(u, n_k=args.n_k, d=args.d, make_evaluator=mk, dist=dist, device=f"cuda:{local_rank}",
                    opts=IpmOptions(max_iter=args.max_iter, separators=args.separators, verbose=args.ipm_verbose,
                                    profile=args.profile), verbose=args.verbose, arch=args.arch, mode=args.mode)
    if res is not None:
        res = dict(res)
        res.pop("V_opt")
        res.update(n_k=args.n_k, d=args.d, arch=args.arch, gpus=world, mode=args.mode,
                   metric=f"sweep trials/sec, {'dual-kite' if args.arch == 'dual' else 'AP2'} power curve")
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)
        print(json.dumps({k: res[k] for k in ("gpus", "trials_per_s", "wall_s")}))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
