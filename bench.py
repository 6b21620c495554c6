#!/usr/bin/env python3
"""Benchmark: batched NLP evaluations {f, g, grad f, J_g} of the AP2 OCP (N=40, d=4) on MI355X.

Contract (see the task's bench section): `python bench.py --gpus N --steps K --warmup W`.  One
*step* = one batched evaluation of B NLP instances (synthetic batch members of SURVEY.md section
8(d): V_b = V0 + 0.01 N(0,1), seed 20261015+b), inputs resident in HBM before the timed region.
For N > 1 (torch.distributed.run, one process per GPU) every rank evaluates its own B instances
(weak scaling, no data-path collective); the timed region is bracketed by barriers and the max
over ranks is reported.  `value` = evaluations/s of the whole job.

Also reported:
  roofline     -- the dominant kernel (ap2_interval_kernel): algorithmic HBM bytes per launch
                  (SURVEY 8(d) formula with the exact nnz, x B) / its mean duration from HIP events
                  on the launch stream, against 8 TB/s;
  cpu_baseline -- the CPU oracle (PyTorch float64 restatement, "port"; the reference CasADi/IPOPT
                  stack cannot be installed) on a bounded sample, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X spec (MI355X_MICROARCH.md); 6.3 TB/s measured float4 copy
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="NLP instances per step and GPU")
    ap.add_argument("--cpu-sample", type=int, default=4, help="oracle evaluations in the CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from awebox_amd import problem as pb
    from awebox_amd.build import build
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import batch_member, initial_guess

    if rank == 0:
        build()
    if dist is not None:
        dist.barrier()

    consts = pb.build_constants()
    lay = pb.NlpLayout(consts.cfg.n_k, consts.cfg.d)
    v0 = initial_guess(consts, lay)
    B = args.batch
    members = range(rank * B, (rank + 1) * B)
    Vh = np.stack([batch_member(v0, lay, b) for b in members])
    Ph = np.stack([pb.pack_p(lay, consts, v0)] * B)
    ev = Ap2Evaluator(consts, batch=B)
    dev = torch.device("cuda", local_rank)
    V = torch.tensor(Vh, device=dev)
    P = torch.tensor(Ph, device=dev)
    f = torch.empty(B, dtype=torch.float64, device=dev)
    g = torch.empty(B, ev.n_g, dtype=torch.float64, device=dev)
    gr = torch.empty(B, ev.n_v, dtype=torch.float64, device=dev)
    jac = torch.empty(B, ev.nnz, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        ev.eval_nlp_device(V, P, f, g, gr, jac, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant-kernel duration from the HIP events the library records on the launch stream
    kms, fms = [], []
    for _ in range(min(args.steps, 20)):
        step()
        a, b_ = ev.last_kernel_ms()
        kms.append(a)
        fms.append(b_)
    torch.cuda.synchronize()
    finite = bool(torch.isfinite(jac).all().item() and torch.isfinite(g).all().item())

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    evals = B * args.steps * world
    value = evals / elapsed
    kernel_ms = float(np.mean(kms))
    bytes_per_eval = 8 * (lay.n_v + lay.n_v + pb.NTHETA0 + pb.NW + pb.NCOST + lay.n_g + lay.n_v + ev.nnz + 1)
    achieved = bytes_per_eval * B / (kernel_ms * 1e-3) / 1e9
    line = {
        "metric": "NLP f/g/Jacobian evals/sec, AP2 N=40 d=4",
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (standard circular-orbit initial guess + 0.01 N(0,1), SURVEY 8(d))",
        "config": {"workload": f"AP2 single kite, direct collocation radau N=40 d=4 zoh, "
                               f"{B} NLP instances per step and GPU, one eval = f + g + grad f + J_g",
                   "n_v": lay.n_v, "n_g": lay.n_g, "nnz_jac": ev.nnz, "batch_per_gpu": B,
                   "parallelism": f"replicas x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": "ap2_interval_kernel", "kernel_ms": kernel_ms,
                     "finalize_ms": float(np.mean(fms)), "bytes_per_eval": bytes_per_eval},
        "outputs_finite": finite,
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(consts, lay, v0, args.cpu_sample)
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(consts, lay, v0, n):
    """Time the CPU oracle (test infrastructure, never the product) on the host cores."""
    import torch

    from awebox_amd import problem as pb
    from awebox_amd.initial_guess import batch_member
    from oracle.ap2_oracle import from_problem

    orc = from_problem(consts)
    P = pb.pack_p(lay, consts, v0)
    V = batch_member(v0, lay, 0)
    # warm-up (first-call overheads of torch.func)
    orc.nlp_g(V, P, lay, pb.THETA0_OFF)
    t0 = time.perf_counter()
    for b in range(n):
        V = batch_member(v0, lay, b)
        orc.nlp_f(V, P, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES)
        orc.nlp_g(V, P, lay, pb.THETA0_OFF)
        orc.nlp_grad_f(V, P, lay, pb.THETA0_OFF, pb.COST_NAMES, pb.PHI_NAMES)
        orc.nlp_jac_g(V, P, lay, pb.THETA0_OFF)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "evals/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} full evaluations (f, g, grad f, J_g) of the AP2 N=40 d=4 NLP by the PyTorch "
                      f"float64 oracle, {dt:.1f} s"}


if __name__ == "__main__":
    main()
