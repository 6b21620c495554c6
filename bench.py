#!/usr/bin/env python3
"""Benchmark: batched NLP evaluations {f, g, grad f, J_g} of the AP2 OCP (N=40, d=4) on MI355X.

Contract (see the task's bench section): `python bench.py --gpus N --steps K --warmup W`.  One
*step* = one batched evaluation of B NLP instances (synthetic batch members of SURVEY.md section
8(d): V_b = V0 + 0.01 N(0,1), seed 20261015+b), inputs resident in HBM before the timed region.
For N > 1 (torch.distributed.run, one process per GPU) every rank evaluates its own B instances
(weak scaling, no data-path collective); the timed region is bracketed by barriers and the max
over ranks is reported.  `value` = evaluations/s of the whole job.

Also reported:
  roofline     -- one evaluation = ap2_node_kernel (generated straight-line node Jacobians, one
                  thread per collocation node) + ap2_gather_kernel (J_g values, gradient): the
                  algorithmic HBM bytes per launch (SURVEY 8(d) formula with the exact nnz, x B) /
                  the two kernels' duration from HIP events on the launch stream, against 8 TB/s;
                  per-kernel times and rates in roofline.kernels.  `traffic` is the HBM byte rate
                  from the rocprofv3 FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE passes recorded
                  in profiles/pmc_traffic.json, used only when that record was taken for the same
                  kernel sources and batch size (else null).
  fp64         -- algorithmic FP64 rate (the op-counting count of profiles/r03/flops_ap2.json /
                  kernel time) and the issued FP64 lane rate of the PMC record, both against the
                  FP64 vector peak; their ratio is the work the SIMT forward mode repeats.
  sweep        -- the metric's second half: wind-speed sweep trials/s, --sweep-points per GPU of
                  config 4's grid linspace(5, 8, 64) (first point: full homotopy; the rest: one
                  batched warm-started solve), collectives over RCCL; dual_sweep: the same for the
                  dual kites (config 4 itself).
  cpu_baseline -- the CPU port of the evaluator (oracle/cpu, C++ with OpenMP over (instance,
                  interval), "port"; the reference CasADi/IPOPT stack cannot be installed) on a
                  bounded sample, rank 0, N=1 only, at all host threads and at one thread.
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
PMC_RECORD = os.path.join(ROOT, "profiles", "pmc_traffic.json")
FLOPS_RECORD = os.path.join(ROOT, "profiles", "r03", "flops_ap2.json")


def flops_record():
    """The algorithmic flop count per evaluation (tools/count_flops.py) for these model sources."""
    try:
        with open(FLOPS_RECORD) as fh:
            rec = json.load(fh)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from count_flops import source_hash
    except (OSError, ValueError, ImportError):
        return None
    return rec if rec.get("source_hash") == source_hash() else None


def kernel_source_hash() -> str:
    """Hash of the evaluator sources: a PMC record is only valid for the code it was taken on."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "awebox_amd", "csrc")
    for name in ("ap2_model.hpp", "ap2_tables.hpp", "awegpu.hip", "scalar.hpp", "ap2_nodejac.gen.hpp"):
        with open(os.path.join(csrc, name), "rb") as fh:
            h.update(name.encode() + fh.read())
    with open(os.path.join(ROOT, "include", "awegpu.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


SOURCES = {   # the files each evaluator kernel is built from (a PMC record is tied to their hash)
    "ap2": ["awebox_amd/csrc/ap2_model.hpp", "awebox_amd/csrc/ap2_tables.hpp", "awebox_amd/csrc/awegpu.hip",
            "awebox_amd/csrc/scalar.hpp", "awebox_amd/csrc/ap2_nodejac.gen.hpp", "include/awegpu.h"],
    "dual": ["awebox_amd/csrc/dual_model.hpp", "awebox_amd/csrc/dual_tables.hpp", "awebox_amd/csrc/awedual.hip",
             "awebox_amd/csrc/awedual_gen.hip", "awebox_amd/csrc/dual_nodejac.gen.hpp", "awebox_amd/csrc/im_layout.hpp",
             "awebox_amd/csrc/ap2_model.hpp", "awebox_amd/csrc/ap2_tables.hpp", "awebox_amd/csrc/scalar.hpp",
             "include/awedual.h", "include/awegpu.h"],
    "mpc": ["awebox_amd/csrc/kite3_model.hpp", "awebox_amd/csrc/kite3_tables.hpp", "awebox_amd/csrc/awempc.hip",
            "awebox_amd/csrc/kite3_nodejac.gen.hpp", "awebox_amd/csrc/im_layout.hpp",
            "awebox_amd/csrc/ap2_tables.hpp", "awebox_amd/csrc/scalar.hpp", "include/awempc.h", "include/awegpu.h"],
}
PMC_RECORD_CONFIGS = os.path.join(ROOT, "profiles", "pmc_traffic_configs.json")


def sources_hash(which: str) -> str:
    import hashlib
    h = hashlib.sha256()
    for rel in SOURCES[which]:
        with open(os.path.join(ROOT, rel), "rb") as fh:
            h.update(os.path.basename(rel).encode() + fh.read())
    return h.hexdigest()[:16]


def config_traffic(which: str, batch: int, kernel_ms: float):
    """HBM traffic of the config-3 / config-5 kernels from their committed PMC record (2 x FETCH_SIZE
    + WRITE_SIZE per dispatch, the gfx950 correction of MI355X_MICROARCH.md), or None when the
    record is missing or was taken on other sources or another batch size."""
    try:
        with open(PMC_RECORD_CONFIGS) as fh:
            rec = json.load(fh).get(which)
    except (OSError, ValueError):
        return None
    if not rec or rec.get("source_hash") != sources_hash(which) or rec.get("batch") != batch:
        return None
    b = (2.0 * rec["FETCH_SIZE_kB"] + rec["WRITE_SIZE_kB"]) * 1024
    out = {"traffic": b / (kernel_ms * 1e-3) / 1e9, "traffic_bytes_per_launch": b,
           "pmc_record": os.path.relpath(PMC_RECORD_CONFIGS, ROOT)}
    f64 = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"]
    if all(k in rec for k in f64 + ["SQ_INSTS_VALU", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"]):
        flops = 64.0 * (rec[f64[0]] + rec[f64[1]] + 2.0 * rec[f64[2]] + rec[f64[3]])
        tf = flops / (kernel_ms * 1e-3) / 1e12
        out["fp64_issued"] = {"achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS,
                              "valu_f64_share": sum(rec[k] for k in f64) / rec["SQ_INSTS_VALU"],
                              "wait_frac": rec["SQ_WAIT_ANY"] / rec["SQ_WAVE_CYCLES"],
                              "note": "FP64 VALU instructions x 64 lanes (FMA = 2) from the PMC record"}
        # the counters decide what limits the kernel: FP64 issue + latency when its issued FP64 rate
        # is well above its HBM fraction
        hbm_frac = out["traffic"] / HBM_PEAK_GBS
        out["measured_limiter"] = ("fp64 VALU issue + latency (SQ_WAIT_ANY {:.0%} of wave cycles)".format(
            out["fp64_issued"]["wait_frac"]) if tf / FP64_PEAK_TFLOPS > hbm_frac else "hbm")
    return out


def gen_kernels(ev, lay, B, node_ms, gather_ms):
    """Per-kernel view of the generated path: the node kernel's operation rate (the generated
    program's adds / multiplies / reciprocals per node, ap2_nodejac.gen.hpp kFlops, x nodes) against
    the FP64 vector peak, and the gather kernel's algorithmic byte rate (its nodebuf run in, J_g and
    the gradient out) against HBM peak."""
    import re
    txt = open(os.path.join(ROOT, "awebox_amd", "csrc", "ap2_nodejac.gen.hpp")).read()
    fl = [int(x) for x in re.search(r"kFlops\[2\] = \{(\d+), (\d+)\}", txt).groups()]
    tr = [int(x) for x in re.search(r"kTranscendental\[2\] = \{(\d+), (\d+)\}", txt).groups()]
    nt = [int(x) for x in re.search(r"kNTan\[2\] = \{(\d+), (\d+)\}", txt).groups()]
    n_k, d = lay.n_k, lay.d
    node_ops = n_k * fl[0] + n_k * d * fl[1]
    tf_node = node_ops * B / (node_ms * 1e-3) / 1e12
    obj = (2 * d * 64 + d + 1) & ~1
    gather_bytes = 8 * (n_k * (obj + nt[0] + d * nt[1]) + ev.nnz + lay.n_v) + 8 * lay.n_v   # run in; J, grad out; V (tf)
    gbs = gather_bytes * B / (gather_ms * 1e-3) / 1e9
    return {"ap2_node_kernel": {"ms": node_ms, "bound": "fp64",
                                "achieved": tf_node, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                "frac": tf_node / FP64_PEAK_TFLOPS, "ops_per_eval": node_ops,
                                "transcendentals_per_eval": n_k * tr[0] + n_k * d * tr[1],
                                "note": "adds, multiplies and reciprocals of the generated node programs "
                                        "(kFlops of ap2_nodejac.gen.hpp) x nodes / node-kernel time"},
            "ap2_gather_kernel": {"ms": gather_ms, "bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS, "bytes_per_eval": gather_bytes,
                                  "note": "nodebuf run read + J_g and gradient written per evaluation"}}


def measured_limiter(rec, hbm_frac, fp64_frac):
    """What the PMC record says limits the evaluation: per kernel the share of wave cycles spent
    waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES) and the share with a VALU instruction issuing, against
    the HBM and FP64 fractions -- latency-bound when waves mostly wait while neither HBM nor FP64 is
    near its peak."""
    per = {}
    for name, k in (rec.get("kernels") or {"evaluation": rec}).items():
        cyc = k.get("SQ_WAVE_CYCLES")
        if not cyc:
            continue
        per[name] = {"wait_frac": k.get("SQ_WAIT_ANY", 0.0) / cyc,
                     "valu_active_frac": k.get("SQ_ACTIVE_INST_VALU", 0.0) / cyc}
    if not per:
        return None
    wait = max(v["wait_frac"] for v in per.values())
    fp = fp64_frac if fp64_frac is not None else 0.0
    fp_txt = "FP64 at {:.1%} of peak".format(fp64_frac) if fp64_frac is not None else "FP64 not measured"
    bound = ("latency (waves waiting on memory / LDS while HBM is at {:.0%} of peak and {})".format(
        hbm_frac, fp_txt) if wait > 0.5 and hbm_frac < 0.6 and fp < 0.6 else "hbm" if hbm_frac >= fp else "fp64")
    return {"bound": bound, "kernels": per}


def soa_kernels(ev, lay, B, ms):
    """Per-kernel view of the instance-minor path (HIP events per kernel, mean over the timed
    launches): algorithmic bytes of each kernel against HBM peak, and the node kernels' generated
    operation rate against the FP64 vector peak.  ms: input transpose, shooting + Radau node
    kernels, interval kernel, finalize, output transpose."""
    import re
    txt = open(os.path.join(ROOT, "awebox_amd", "csrc", "ap2_nodejac.gen.hpp")).read()
    fl = [int(x) for x in re.search(r"kFlops\[2\] = \{(\d+), (\d+)\}", txt).groups()]
    ndbp = int(re.search(r"kNDbp = (\d+)", txt).group(1))
    nth = int(re.search(r"kNThUsed = (\d+)", txt).group(1))
    n_k, d = lay.n_k, lay.d
    obj = n_k * d * (2 + ndbp)
    stride = 2 * 23 + 10 + 1 + d * 24
    by = {"ap2_soa_in_kernel": 8 * 2 * (lay.n_v + lay.n_p),                      # V, P in; VT, PT out
          # the interval slices + theta0 rows each node workgroup stages; J_g, g, objective terms out
          "ap2_soa_shoot + ap2_soa_radau": 8 * (n_k * (stride + 2 * (nth + 6)) + ev.nnz + lay.n_g + obj),
          # V and P slices, objective terms in; gradient, continuity rows, partials out
          "ap2_soa_interval_kernel": 8 * (n_k * (stride + 23) + lay.n_v + 59 + 20 + 2 + obj + lay.n_v
                                          + n_k * 23 + n_k * 4)}
    names = ["ap2_soa_in_kernel", "ap2_soa_shoot + ap2_soa_radau", "ap2_soa_interval_kernel", "ap2_finalize_kernel",
             "soa_to_aos_kernel"]
    out = {}
    for i, name in enumerate(names):
        t = float(ms[i])
        if t <= 0 or (name == "ap2_soa_in_kernel" and t < 0.01):   # no transpose (instance-minor inputs)
            continue
        o = {"ms": t}
        if name in by:
            gbs = by[name] * B / (t * 1e-3) / 1e9
            o.update({"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": gbs / HBM_PEAK_GBS, "bytes_per_eval": by[name]})
        if name == "ap2_soa_shoot + ap2_soa_radau":
            ops = n_k * fl[0] + n_k * d * fl[1]
            o["fp64_generated_ops"] = {"achieved": ops * B / (t * 1e-3) / 1e12, "peak": FP64_PEAK_TFLOPS,
                                       "unit": "TFLOP/s", "ops_per_eval": ops}
        out[name] = o
    return out


def path_ab(ev, V, P, f, g, gr, B, dev, stream, reps=10):
    """The same evaluation on every path and J_g layout, HIP-event time per call (ms): the
    instance-minor path writing the solver's layout (the headline) or per-instance J_g (plus the
    transpose), the node + gather path and the colour path."""
    import torch
    import numpy as np
    keep = ev.path
    out = {}
    jac_aos, gr_aos = ev.alloc_jac(dev, instance_minor=False), ev.alloc_grad(dev, instance_minor=False)
    jac_im, gr_im = ev.alloc_jac(dev, instance_minor=True), ev.alloc_grad(dev, instance_minor=True)
    for name, path, jac, grd in (("soa_instance_minor", "soa", jac_im, gr_im), ("soa_per_instance", "soa", jac_aos, gr_aos),
                                 ("generated", "generated", jac_aos, gr_aos), ("colour", "colour", jac_aos, gr_aos)):
        try:
            ev.path = path
        except Exception:
            continue
        ms = []
        for _ in range(reps + 2):
            ev.eval_nlp_device(V, P, f, g, grd, jac, stream=stream.cuda_stream)
            a, b_ = ev.last_kernel_ms()
            ms.append(a + b_)
        out[name] = float(np.mean(ms[2:]))
    ev.path = keep
    torch.cuda.synchronize()
    del jac_aos, jac_im, gr_aos, gr_im
    return out


def pmc_record(batch: int):
    """The committed PMC record for these sources and batch size, or None."""
    try:
        with open(PMC_RECORD) as fh:
            rec = json.load(fh)
    except (OSError, ValueError):
        return None
    if rec.get("source_hash") != kernel_source_hash() or rec.get("batch") != batch:
        return None
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2048, help="NLP instances per step and GPU")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="CPU baseline time per thread setting")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hessian", action="store_true", help="skip the nlp_hess_l timing block")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the batch-1 host round-trip block (its launches share the AP2 kernel's name)")
    ap.add_argument("--mpc-batch", type=int, default=256,
                    help="MPC instances for the config-5 block (3-DOF tracking MPC, N=20 d=4; 0: skip)")
    ap.add_argument("--pmpc-loops", type=int, default=64,
                    help="closed loops per GPU for the converged-MPC block (Pmpc.step on the batched IPM; 0: skip)")
    ap.add_argument("--dual-batch", type=int, default=128,
                    help="dual-kite NLP instances for the config-3 block (N=60 d=4 single_reelout; 0: skip)")
    ap.add_argument("--no-dual-chain", action="store_true",
                    help="skip the chain-mode (sequential warm start) rate of the config-4 shard")
    ap.add_argument("--dual-sweep-points", type=int, default=8,
                    help="dual-kite u_ref sweep points per GPU (config 4: 8 of linspace(5, 8, 64), example "
                         "discretization N=20; 0: skip)")
    ap.add_argument("--sweep-mode", choices=["fan", "batch", "chain"], default="fan",
                    help="AP2 sweep mode (awebox_amd/sweep.py run_sweep)")
    ap.add_argument("--sweep-points", type=int, default=8,
                    help="u_ref sweep points solved per GPU for the sweep block, as one batched homotopy (0: skip)")
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
    # J_g and grad f in the layout the batched solver reads: instance-minor ([n, B] storage, [B, n] view)
    gr = ev.alloc_grad(dev, instance_minor=True)
    jac = ev.alloc_jac(dev, instance_minor=True)
    stream = torch.cuda.current_stream(dev)
    # on the instance-minor path the decision vectors and parameters are handed over instance-minor
    # too (awe_eval_nlp_imv: no input transposition), the layout a batched caller keeps them in; the
    # per-instance inputs' rate is paths.soa_instance_minor (awe_eval_nlp_im)
    V_in, P_in, input_layout = V, P, "per-instance"
    if ev.path == "soa":
        V_in, P_in = ev.alloc_inputs(dev)
        V_in.copy_(V)
        P_in.copy_(P)
        input_layout = "instance-minor"

    def step():
        ev.eval_nlp_device(V_in, P_in, f, g, gr, jac, stream=stream.cuda_stream)

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
    kms, fms, nms, gms, sms = [], [], [], [], []
    gen = ev.path == "generated"
    soa = ev.path == "soa"
    for _ in range(min(args.steps, 20)):
        step()
        a, b_ = ev.last_kernel_ms()
        kms.append(a + b_ if soa else a)
        fms.append(b_)
        if gen:
            n_, g_ = ev.last_kernel_ms_gen()
            nms.append(n_)
            gms.append(g_)
        if soa:
            sms.append(ev.last_kernel_ms_soa())
    torch.cuda.synchronize()
    finite = bool(torch.isfinite(jac).all().item() and torch.isfinite(g).all().item())
    paths = path_ab(ev, V, P, f, g, gr, B, dev, stream) if rank == 0 else None

    dual = None
    if args.dual_batch > 0:
        dual = dual_block(args.dual_batch, rank, dev, dist, world,
                          cpu_seconds=0.0 if (args.no_cpu_baseline or world > 1) else args.cpu_seconds / 2)
    mpc = None
    if args.mpc_batch > 0:
        mpc = mpc_block(args.mpc_batch, rank, dev, dist, world)
        if args.pmpc_loops > 0:
            from awebox_amd import kite3 as k3
            mpc["converged"] = pmpc_block(k3.build_constants(), args.pmpc_loops, dev, dist, world)
    sweep = None
    if args.sweep_points > 0:
        sweep = sweep_block(args.sweep_points, world, dist, dev, consts, mode=args.sweep_mode)
    dual_sweep = None
    if args.dual_sweep_points > 0:
        dual_sweep = dual_sweep_block(args.dual_sweep_points, world, dist, dev, with_chain=not args.no_dual_chain)
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
                     "kernel": ("ap2_soa_shoot + ap2_soa_radau + ap2_soa_interval + ap2_finalize "
                                "(one evaluation, V and P instance-minor)"
                                if soa else "ap2_node_kernel + ap2_gather_kernel" if gen else "ap2_interval_kernel"),
                     "kernel_ms": kernel_ms, "finalize_ms": float(np.mean(fms)), "bytes_per_eval": bytes_per_eval},
        "outputs_finite": finite,
        "eval_path": ev.path,
        "input_layout": input_layout,
    }
    if gen:
        line["roofline"]["kernels"] = gen_kernels(ev, lay, B, float(np.mean(nms)), float(np.mean(gms)))
    if soa:
        line["roofline"]["kernels"] = soa_kernels(ev, lay, B, np.mean(np.array(sms), axis=0))
    if paths is not None:
        line["paths"] = paths
    rec = pmc_record(B)
    if rec is not None and rec.get("path", "colour") != ev.path:
        rec = None
    fp64 = {}
    alg = flops_record()
    if alg is not None:
        # useful work: the op-counting restatement's flops per evaluation (tools/count_flops.py)
        tf_alg = alg["flops_per_eval"] * B / (kernel_ms * 1e-3) / 1e12
        fp64["algorithmic"] = {"achieved": tf_alg, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                               "frac": tf_alg / FP64_PEAK_TFLOPS, "flops_per_eval": alg["flops_per_eval"],
                               "record": os.path.relpath(FLOPS_RECORD, ROOT),
                               "note": "value ops once per node + forward-mode tangent ops per structurally "
                                       "nonzero colour + assembly (tools/flops/ap2_flops.cpp)"}
    if rec is not None:
        hbm_bytes = 2.0 * rec["FETCH_SIZE_kB"] * 1024 + rec["WRITE_SIZE_kB"] * 1024
        line["roofline"]["traffic"] = hbm_bytes / (kernel_ms * 1e-3) / 1e9
        line["roofline"]["traffic_bytes_per_launch"] = hbm_bytes
        line["roofline"]["pmc_record"] = os.path.relpath(PMC_RECORD, ROOT)
        f64 = ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"]
        if all(k in rec for k in f64):
            flops = 64.0 * (rec[f64[0]] + rec[f64[1]] + 2.0 * rec[f64[2]] + rec[f64[3]])
            tf = flops / (kernel_ms * 1e-3) / 1e12
            issued = {"achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS,
                      "flops_per_launch": flops,
                      "note": "FP64 VALU instructions x 64 lanes (FMA = 2) from the PMC record: issued lane "
                              "operations, idle and redundant lanes included -- an upper bound on useful work"}
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"):
                if k in rec:
                    issued[k] = rec[k]
            if "SQ_INSTS_VALU" in rec:
                issued["valu_f64_share"] = sum(rec[k] for k in f64) / rec["SQ_INSTS_VALU"]
            fp64["issued"] = issued
            if "algorithmic" in fp64:
                fp64["issued_over_algorithmic"] = flops / (fp64["algorithmic"]["flops_per_eval"] * B)
    if fp64:
        line["fp64"] = fp64
    if rec is not None:
        # FP64: the issued fraction from the PMC record when it has the FP64 counters, else the
        # algorithmic one (the instance-minor record carries no TRANS_F64 count)
        line["roofline"]["measured_limiter"] = measured_limiter(
            rec, line["roofline"]["frac"],
            fp64.get("issued", {}).get("frac", fp64.get("algorithmic", {}).get("frac")))
    if dual is not None:
        line["dual"] = dual
    if mpc is not None:
        line["mpc"] = mpc
    if sweep is not None:
        line["sweep"] = sweep
    if dual_sweep is not None:
        line["dual_sweep"] = dual_sweep
    if not args.no_hessian:
        line["hessian"] = hessian_block(ev, V, P, B, lay, dev)
    if world == 1 and not args.no_latency:
        line["latency_batch1"] = latency_block(consts, lay, v0, with_cpu=not args.no_cpu_baseline)
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(consts, lay, v0, args.cpu_seconds)
    if rank == 0:
        line["casadi_probe"] = casadi_probe()
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def dual_block(B, rank, dev, dist, world, steps=20, warmup=3, cpu_seconds=0.0):
    """Config 3: B dual-kite NLP instances per GPU (architecture {1:0, 2:1, 3:1},
    N=60, d=4, single_reelout; examples/dual_kites_power_curve.py), synthetic members
    V0 + 0.01 N(0,1) of the standard multi-kite initial guess; one step = one batched
    {f, g, grad f, J_g} evaluation.  Weak scaling, max over ranks."""
    import numpy as np
    import torch

    from awebox_amd import dual as du
    from awebox_amd.dual_evaluator import DualEvaluator, colour_counts

    c = du.build_constants()
    lay = du.layout_for(c)
    v0 = du.initial_guess(c, lay)
    V = torch.tensor(np.stack([du.batch_member(v0, lay, rank * B + b) for b in range(B)]), device=dev)
    P = torch.tensor(np.stack([du.pack_p(lay, c, v0)] * B), device=dev)
    ev = DualEvaluator(c, batch=B)
    f = torch.empty(B, dtype=torch.float64, device=dev)
    g = torch.empty(B, ev.n_g, dtype=torch.float64, device=dev)
    # the generated instance-minor path (adl_eval_nlp_im) when it serves these constants; the colour
    # kernel (adl_eval_nlp, per-instance layout) is timed beside it for the record
    gen = ev.generated_available
    gr, jac = ev.alloc_grad(dev, instance_minor=gen), ev.alloc_jac(dev, instance_minor=gen)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(warmup):
        ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kms, fms, parts = [], [], []
    for _ in range(10):
        ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
        if gen:
            pt = ev.last_kernel_ms_im()
            parts.append(pt)
            kms.append(sum(pt[:3]))
            fms.append(pt[3])
        else:
            a, b_ = ev.last_kernel_ms()
            kms.append(a)
            fms.append(b_)
    finite = bool(torch.isfinite(jac).all().item() and torch.isfinite(g).all().item())
    colour_ms = None
    if gen:
        gr_c, jac_c = ev.alloc_grad(dev), ev.alloc_jac(dev)
        cms = []
        for _ in range(5):
            ev.eval_nlp_device(V, P, f, g, gr_c, jac_c, stream=s)
            cms.append(sum(ev.last_kernel_ms()))
        colour_ms = float(np.mean(cms))
        del gr_c, jac_c
    m = c.model
    bytes_per_eval = 8 * (lay.n_v + lay.n_v + pb_ntheta0() + m.nw + 20 + lay.n_g + lay.n_v + ev.nnz + 1)
    kernel_ms = float(np.mean(kms)) + float(np.mean(fms))
    achieved = bytes_per_eval * B / (kernel_ms * 1e-3) / 1e9
    ncol = colour_counts(c)
    cpu = None
    if cpu_seconds > 0 and rank == 0:
        from oracle.dual_cpu_port import DualCpuPort
        port = DualCpuPort(c)
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)

        def rate(nb, nthreads):
            Vh = np.stack([du.batch_member(v0, lay, b) for b in range(nb)])
            Ph = np.stack([du.pack_p(lay, c, v0)] * nb)
            port.eval_nlp(Vh, Ph, threads=nthreads)
            n, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < cpu_seconds:
                port.eval_nlp(Vh, Ph, threads=nthreads)
                n += nb
            return n / (time.perf_counter() - t0), n

        r_all, n_all = rate(max(threads, 4), threads)
        r_one, n_one = rate(1, 1)
        cpu = {"value": r_all, "unit": "evals/s", "cores": threads, "kind": "port", "value_1core": r_one,
               "sample": f"C++ CPU port of the dual-kite evaluator (oracle/cpu/dual_cpu.cpp, the kernel's algorithm, "
                         f"OpenMP over (instance, interval)): {n_all} evaluations on {threads} threads and {n_one} "
                         f"on 1 thread, ~{cpu_seconds:.0f} s each"}
    return {"metric": "dual-kite NLP f/g/Jacobian evals/sec, N=60 d=4 single_reelout (config 3)",
            "value": B * steps * world / el, "unit": "evals/s", "instances_per_gpu": B,
            "ms_per_step": el / steps * 1e3, "n_v": lay.n_v, "n_g": lay.n_g, "nnz_jac": ev.nnz,
            "colours_shooting_radau": [ncol[0], ncol[1]],
            "finite": finite,
            "eval_path": "generated instance-minor (adl_eval_nlp_im)" if gen else "colour kernel",
            "colour_kernel_ms": colour_ms,
            "roofline": dict({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": achieved / HBM_PEAK_GBS,
                              "kernel": ("dual_gen_in + dual_gen_node + dual_gen_interval + dual_gen_finalize "
                                         "(one evaluation)" if gen else "dual_interval_kernel<4> + dual_finalize_kernel"),
                              "kernel_ms": kernel_ms, "finalize_ms": float(np.mean(fms)),
                              "bytes_per_eval": bytes_per_eval, "traffic": None},
                             **({"kernel_ms_parts": dict(zip(("transpose_in", "node", "interval", "finalize"),
                                                             np.mean(parts, axis=0).tolist()))} if gen else {}),
                             **((config_traffic("dual", B, kernel_ms) or {}) if gen else {})),
            "cpu_baseline": cpu}


def pb_ntheta0():
    from awebox_amd import problem as pb
    return pb.NTHETA0


def mpc_block(B, rank, dev, dist, world, steps=50, warmup=5):
    """Config 5: B tracking-MPC NLP instances of the 3-DOF AP2 kite (N=20, d=4) per
    GPU, instance i starting at phase i T / B of the reference orbit with 0.01 N(0,1) noise (seed
    99 + i); one step = one batched {f, g, grad f, J_g} evaluation (the linearisation of one
    real-time iteration of every instance).  Weak scaling, max over ranks."""
    import numpy as np
    import torch

    from awebox_amd import kite3 as k3
    from awebox_amd.mpc import MpcEvaluator

    c = k3.build_constants()
    lay = k3.MpcLayout(c.cfg.n_k, c.cfg.d)
    orbit = k3.CircularOrbit(c.cfg)
    inst = [k3.batch_instance(c, lay, rank * B + i, B * world, orbit=orbit) for i in range(B)]
    V = torch.tensor(np.stack([v for v, _ in inst]), device=dev)
    P = torch.tensor(np.stack([p for _, p in inst]), device=dev)
    ev = MpcEvaluator(c, batch=B)
    f = torch.empty(B, dtype=torch.float64, device=dev)
    g = torch.empty(B, ev.n_g, dtype=torch.float64, device=dev)
    # the layout the batched solvers use: instance-minor J_g / grad f from the generated node code
    # (awempc_eval_nlp_im) when it serves these constants
    gen = ev.generated_available
    gr, jac = ev.alloc_grad(dev), ev.alloc_jac(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(warmup):
        ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    kms, parts = [], []
    for _ in range(10):
        ev.eval_nlp_device(V, P, f, g, gr, jac, stream=s)
        if gen:
            t_in, t_node, t_fin = ev.last_kernel_ms_im()
            kms.append(t_in + t_node + t_fin)
            parts.append((t_in, t_node, t_fin))
        else:
            kms.append(sum(ev.last_kernel_ms()))
    bytes_per_eval = 8 * (lay.n_v + lay.n_p + lay.n_g + lay.n_v + ev.nnz + 1)
    kernel_ms = float(np.mean(kms))
    achieved = bytes_per_eval * B / (kernel_ms * 1e-3) / 1e9
    finite = bool(torch.isfinite(jac).all().item())
    nnz = ev.nnz
    # the dual-number kernel (awempc_eval_nlp, per-instance layout) on the same inputs, for the record
    gr_d, jac_d = ev.alloc_grad(dev, instance_minor=False), ev.alloc_jac(dev, instance_minor=False)
    dms = []
    for _ in range(10):
        ev.eval_nlp_device(V, P, f, g, gr_d, jac_d, stream=s)
        dms.append(sum(ev.last_kernel_ms()))
    del ev, f, g, gr, jac, gr_d, jac_d
    rti = rti_block(c, B, dev, dist, world)
    return {"metric": "MPC NLP f/g/Jacobian evals/sec, 3-DOF AP2 tracking MPC N=20 d=4 (config 5)",
            "value": B * steps * world / el, "unit": "evals/s", "instances_per_gpu": B,
            "ms_per_step": el / steps * 1e3, "n_v": lay.n_v, "n_g": lay.n_g, "nnz_jac": nnz,
            "finite": finite,
            "roofline": dict({"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": achieved / HBM_PEAK_GBS,
                              "kernel": ("mpc_gen_in + mpc_gen_node (Radau, shooting and interval tiles) + mpc_gen_finalize (one evaluation)"
                                         if gen else "mpc_interval_kernel<4> + mpc_finalize_kernel"),
                              "kernel_ms": kernel_ms, "bytes_per_eval": bytes_per_eval, "traffic": None},
                             **({"kernel_ms_parts": dict(zip(("transpose_in", "node", "finalize"),
                                                             np.mean(parts, axis=0).tolist()))} if gen else {}),
                             **((config_traffic("mpc", B, kernel_ms) or {}) if gen else {})),
            "eval_path": "generated instance-minor (awempc_eval_nlp_im)" if gen else "dual-number kernel",
            "dual_kernel_ms": float(np.mean(dms)),
            "rti": rti}


def rti_block(c, B, dev, dist, world, steps=10, warmup=3):
    """Config 5 closed loop: B tracking-MPC loops per GPU, each advanced by one real-time
    iteration per sampling time (awebox_amd/rti.py: batched linearisation on the HIP evaluator,
    Gauss-Newton KKT solve by interval elimination on the awelu kernel, radau-collocation plant
    step, horizon shift).  value = loop-steps/s (loops x sampling times), max over ranks."""
    import torch

    from awebox_amd.rti import BatchedRti

    r = BatchedRti(c, B, device=str(dev))
    r.start(seed=99 + dist.get_rank() * B if dist is not None else 99, x0_entries=CONSISTENT_X0)
    r.simulate_reference(warmup + steps + c.cfg.n_k + 1)
    for _ in range(warmup):
        r.step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = r.step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return {"metric": "closed-loop real-time iterations/sec (loops x sampling times), 3-DOF tracking MPC N=20 d=4",
            "value": B * steps * world / el, "unit": "loop-steps/s", "loops_per_gpu": B,
            "ms_per_step": el / steps * 1e3, "sampling_time_s": c.cfg.ts,
            "realtime_factor": c.cfg.ts / (el / steps),
            "kkt_blocks": {"interval": [B * r.nk, r.nI], "separator": [B, r.nS]},
            "plant_residual_max": float(out["plant_residual"].max()),
            "eq_residual_median": float(out["eq_residual"].median()),
            "tracking_error_median": float(out["tracking_error"].median()),
            "tracking_error_max": float(out["tracking_error"].max()),
            "reference": REFERENCE_NOTE,
            "finite": bool(torch.isfinite(r.V).all().item())}


CONSISTENT_X0 = (6, 7, 10)     # CL, roll, reel acceleration: x0 noise that keeps the tether invariants
REFERENCE_NOTE = ("each loop tracks a trajectory of the 3-DOF model (BatchedRti.simulate_reference: the plant "
                  "integrated from the circle's state at the loop's phase), x0 = reference + 0.01 N(0,1) on CL, "
                  "roll and reel acceleration")


def pmpc_block(c, B, dev, dist, world, steps=3, warmup=1):
    """Config 5 with the reference's solver semantics: B tracking-MPC loops per GPU, every sampling
    time solved to convergence (awebox_amd/mpc_solve.py: Pmpc.step's 2-iteration pre-solve and
    tol 1e-6 IPOPT solve with bounds, path inequalities and the exact Hessian, as one batched
    interior-point solve of all loops), then the plant step and the shift.  x0 perturbed on the
    invariant-free states.  value = loop-steps/s, max over ranks."""
    import numpy as np
    import torch

    from awebox_amd.mpc_solve import BatchedPmpc

    r = BatchedPmpc(c, B, device=str(dev))
    r.start(seed=99 + dist.get_rank() * B if dist is not None else 99)
    r.simulate_reference(warmup + steps + c.cfg.n_k + 1)
    for _ in range(warmup):
        r.step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    its, ok = [], []
    for _ in range(steps):
        out = r.step()
        its.append(out["iterations"])
        ok.append(np.array([s_ == "solve_succeeded" for s_ in out["status"]]))
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    its, ok = np.concatenate(its), np.concatenate(ok)
    return {"metric": "closed-loop converged MPC solves/sec (loops x sampling times), 3-DOF tracking MPC N=20 d=4",
            "value": B * steps * world / el, "unit": "loop-steps/s", "loops_per_gpu": B,
            "ms_per_step": el / steps * 1e3, "sampling_time_s": c.cfg.ts,
            "realtime_factor": c.cfg.ts / (el / steps), "solved_fraction": float(ok.mean()),
            "ipm_iterations_median": float(np.median(its)), "ipm_iterations_max": int(its.max()),
            "plant_residual_max": float(out["plant_residual"].max()),
            "tracking_error_median": float(out["tracking_error"].median()),
            "tracking_error_max": float(out["tracking_error"].max()),
            "reference": REFERENCE_NOTE,
            "solver": "batched IPM (mu_init 1e-3, tol 1e-6, 2-iteration homotopy pre-solve), bounds and path "
                      "inequalities, exact Hessian of the Lagrangian (awempc_eval_hess: hyper-dual direction-pair kernel)"
                      if r.hessian == "exact" else "batched IPM, Hessian by coloured central differences",
            "hessian_ms_last": r.ev.last_hess_ms() if r.hessian == "exact" else None}


SWEEP_GRID = 64       # config 4: u_ref = linspace(5, 8, 64), 8 contiguous points per GPU


def sweep_profile(arch: str):
    """GPU utilisation of the sweep block from its committed rocprofv3 record (tools/sweep_record.py):
    busy fraction and the dominant solver kernels, or None when the solver / evaluator sources
    changed since the record was taken."""
    path = os.path.join(ROOT, "profiles", "r06", "sweep", f"sweep_profile_{arch}.json")
    try:
        with open(path) as fh:
            rec = json.load(fh)
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from sweep_record import sources_hash
    except (OSError, ValueError, ImportError):
        return None
    if rec.get("source_hash") != sources_hash(arch):
        return None
    return {"record": os.path.relpath(path, ROOT), "gpu_busy_frac": rec["gpu_busy_frac"],
            "gpu_kernel_s": rec["gpu_kernel_s"], "wall_s_profiled": rec["wall_s"],
            "dominant_kernel": rec["top_kernels"][0]["kernel"],
            "dominant_share_of_gpu_time": rec["top_kernels"][0]["share_of_gpu_time"],
            "top_kernels": [{k: t[k] for k in ("kernel", "share_of_gpu_time", "avg_ms", "calls")}
                            for t in rec["top_kernels"][:4]]}


def solver_kernels(n_k, batches, reps=5):
    """Rooflines of the sweep's KKT kernels at the block shapes of its last solves (the structure
    cache of ipm.solve_batch, interval count n_k), for each batch size in `batches` (the shard's
    homotopy at B = 1, the fan's batched warm start): the separator sweep (awelu_btd_factor_batched,
    nb stages of m x m blocks; the dual kites' m > 48 run the block recursion, whose pivot-block LUs
    are awelu_factor_batched) and the interval blocks' inertia (awelu_sym_inertia_batched, n_k blocks
    of nI rows per instance).  HIP events on the launch stream around `reps` launches on fresh copies
    of random blocks (diagonally weighted, symmetric for the inertia).  Algorithmic work per system:
    Gauss-Jordan sweep (nb - 1) 2 m^3 + nb 6 m^3 flops and 6 m^2 doubles per stage (read L, D, U;
    write D', W, D'^-1); Bunch-Kaufman n^3 / 3 flops and n^2 doubles read; LU 2 n^3 / 3 flops and
    2 n^2 doubles.  These chains are latency-bound (a barrier-separated pivot step per column), so
    both fractions are small; they say how far from either roof the kernels sit."""
    import ctypes

    import torch

    from awebox_amd import batched_lu as bl
    from awebox_amd.ipm import ZERO_PIVOT, cached_kkt_structures
    sks = [s for s in cached_kkt_structures() if s.n_k == n_k and s.btd is not None]
    if not sks or not torch.cuda.is_available():
        return None
    sk = sks[-1]
    nb, m, nI = sk.btd.nb, sk.btd.m, sk.nI
    lib = bl.load_library()
    dev = torch.device("cuda", torch.cuda.current_device())
    stream = torch.cuda.current_stream(dev)
    gen = torch.Generator(device=dev).manual_seed(7)
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def timed(launch, inputs):
        launch(inputs[0])                                   # warm-up (code object load)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for x in inputs[1:]:
            launch(x)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / (len(inputs) - 1)

    def line(kernel, shape, systems, ms, flops, doubles):
        tf = flops * systems / (ms * 1e-3) / 1e12
        gbs = doubles * 8 * systems / (ms * 1e-3) / 1e9
        return {"kernel": kernel, "shape": shape, "systems": systems, "ms": ms,
                "fp64": {"achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS},
                "hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS},
                "bound": "latency (dependent pivot columns, one workgroup per system)"}

    out = []
    f64 = dict(dtype=torch.float64, device=dev)
    for B in batches:
        eye = torch.eye(m, **f64)
        if m <= bl.BTD_MAX_M:
            T = torch.randn(B, nb, 3, m, m, generator=gen, **f64)
            T[:, :, 1] += 4.0 * m ** 0.5 * eye
            Ts = [T.clone() for _ in range(reps + 1)]
            Dinv = torch.empty(B, nb, m, m, **f64)
            ms = timed(lambda x: lib.awelu_btd_factor_batched(nb, m, B, ptr(x), ptr(Dinv), ctypes.c_void_p(stream.cuda_stream)), Ts)
            out.append(line("btd_factor_kernel", f"nb={nb} m={m}", B, ms, (nb - 1) * 2 * m ** 3 + nb * 6 * m ** 3,
                            nb * 6 * m * m))
            del Ts
        else:
            A = torch.randn(B * nb, m, m, generator=gen, **f64) + 4.0 * m ** 0.5 * eye
            As = [A.clone() for _ in range(reps + 1)]
            piv = torch.empty(B * nb, m, dtype=torch.int32, device=dev)
            ms = timed(lambda x: lib.awelu_factor_batched(m, B * nb, ptr(x), ptr(piv), ctypes.c_void_p(stream.cuda_stream)), As)
            out.append(line("lu_batched_kernel (separator pivot blocks)", f"n={m}", B * nb, ms, 2 * m ** 3 / 3,
                            2 * m * m))
            del As
        S = torch.randn(B * n_k, nI, nI, generator=gen, **f64)
        S = S + S.transpose(1, 2)
        Ss = [S.clone() for _ in range(reps + 1)]
        counts = torch.empty(B * n_k, 3, dtype=torch.int32, device=dev)
        ms = timed(lambda x: lib.awelu_sym_inertia_batched(nI, B * n_k, ptr(x), ctypes.c_double(ZERO_PIVOT), ptr(counts),
                                                           ctypes.c_void_p(stream.cuda_stream)), Ss)
        out.append(line("sym_inertia_kernel (interval blocks)", f"n={nI}", B * n_k, ms, nI ** 3 / 3, nI * nI))
        del Ss
    return out


def _grid_points(per_gpu, world):
    """The points of the sweep: the first per_gpu x world of linspace(5, 8, 64) (config 4's grid;
    rank r gets the contiguous block [r per_gpu, (r + 1) per_gpu)), or an even spread over 5..8 m/s
    when more points are asked for than the grid holds."""
    import numpy as np
    n_pts = per_gpu * world
    if n_pts <= SWEEP_GRID:
        return np.linspace(5.0, 8.0, SWEEP_GRID)[:n_pts]
    return np.linspace(5.0, 8.0, n_pts)


def sweep_block(per_gpu, world, dist, dev, consts, mode="fan"):
    """Second half of the headline metric: wind-speed sweep trials/s on config 4's recipe (points of
    u_ref = linspace(5, 8, 64), contiguous blocks of `per_gpu` per GPU, template broadcast / seed
    scatter / solution gather over RCCL), the AP2 N=40 d=4 trial.  Per shard (weak scaling): the
    full homotopy for the first point, then the other points warm-started from its solution in one
    batched interior-point solve (sweep.py mode "fan": the reference's sweeping warm start,
    fanned out).  Timed between barriers, max over ranks (run_sweep's clock, all-reduced)."""
    import torch

    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep

    u = _grid_points(per_gpu, world)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    res = run_sweep(u, n_k=consts.cfg.n_k, d=consts.cfg.d, make_evaluator=lambda c, b=1: Ap2Evaluator(c, batch=b),
                    dist=dist, device=str(dev), opts=IpmOptions(max_iter=1000), mode=mode)
    if res is None:
        return None
    return {"metric": "sweep trials/sec, AP2 N=40 d=4 power curve", "value": res["trials_per_s"], "mode": mode,
            "unit": "trials/s", "points": len(u), "points_per_gpu": per_gpu, "wall_s": res["wall_s"],
            "u_ref": [round(x, 4) for x in res["u_ref"]],
            "all_converged": bool(all(res["ok"])), "iterations": res["iterations"],
            "avg_power_W": [round(p, 1) for p in res["avg_power_W"]],
            "period_s": [round(t, 2) for t in res["period_s"]], "scaling": "weak",
            "solver": "GPU interior point (awebox_amd/ipm.py): homotopy for the shard's first point, batched "
                      "warm start (solve_batch) for the rest; structured KKT (batched interval LU + "
                      "block-tridiagonal separators), exact Hessian, IPOPT inertia correction from exact KKT "
                      "inertia, second-order corrections",
            "utilisation": sweep_profile("ap2"),
            "solver_kernels": solver_kernels(consts.cfg.n_k, sorted({1, max(1, per_gpu - 1)}))}


def dual_sweep_block(per_gpu, world, dist, dev, n_k=20, d=4, with_chain=True):
    """Config 4: the dual-kite power curve (examples/dual_kites_power_curve.py: architecture
    {1:0, 2:1, 3:1}, N=20 d=4 as in the example, single_reelout), each GPU's shard of
    u_ref = linspace(5, 8, 64): `per_gpu` contiguous points (weak scaling), template broadcast / seed
    scatter / solution gather over RCCL; per shard the homotopy for the first point and one batched
    warm-started solve for the rest (the HIP dual-kite evaluator, the exact Hessian kernel
    dual_hess_kernel, exact-inertia interior point).  Timed by run_sweep between barriers, max over ranks."""
    import torch

    from awebox_amd.dual_homotopy import make_evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep

    u = _grid_points(per_gpu, world)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    res = run_sweep(u, n_k=n_k, d=d, make_evaluator=lambda c, b=1: make_evaluator(c, device=str(dev), batch=b),
                    dist=dist, device=str(dev), opts=IpmOptions(max_iter=3000), arch="dual", mode="fan")
    chain = None
    if with_chain:
        # the reference's own sweep order (awebox/sweep.py:154-163): the shard's points one after
        # the other, each warm-started from the previous solution
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        rc = run_sweep(u, n_k=n_k, d=d, make_evaluator=lambda c, b=1: make_evaluator(c, device=str(dev), batch=b),
                       dist=dist, device=str(dev), opts=IpmOptions(max_iter=3000), arch="dual", mode="chain")
        if rc is not None:
            chain = {"value": rc["trials_per_s"], "unit": "trials/s", "wall_s": rc["wall_s"],
                     "all_converged": bool(all(rc["ok"])), "iterations": rc["iterations"],
                     "avg_power_W": [round(p, 1) for p in rc["avg_power_W"]],
                     "mode": "chain: homotopy for the shard's first point, then each point warm-started from the "
                             "previous one, sequentially (the reference's sweep)"}
    if res is None:
        return None
    return {"metric": f"sweep trials/sec, dual-kite power curve N={n_k} d={d} (config 4)",
            "value": res["trials_per_s"], "unit": "trials/s", "points": len(u), "points_per_gpu": per_gpu,
            "grid": f"linspace(5, 8, {SWEEP_GRID}), contiguous shards", "u_ref": [round(x, 4) for x in res["u_ref"]],
            "wall_s": res["wall_s"], "all_converged": bool(all(res["ok"])), "iterations": res["iterations"],
            "avg_power_W": [round(p, 1) for p in res["avg_power_W"]],
            "period_s": [round(t, 2) for t in res["period_s"]], "scaling": "weak",
            "solver": "GPU interior point (awebox_amd/ipm.py): homotopy for the shard's first point, batched warm "
                      "start for the rest; structured KKT with the block-recursion separator sweep, exact KKT "
                      "inertia; exact Hessian of the Lagrangian (dual_hess_kernel: colour-pair hyper-dual forward mode)",
            "mode": "fan: homotopy for the shard's first point, one batched warm start for the rest",
            "chain": chain, "utilisation": sweep_profile("dual"),
            "solver_kernels": solver_kernels(n_k, sorted({1, max(1, per_gpu - 1)}))}


def hess_gen_counts():
    """Algorithmic work of one node Hessian from the generated code (csrc/ap2_nodehess.gen.hpp:
    kFlops = adds / muls / reciprocals, kTranscendental = sqrt / exp / log / sin / cos calls, per
    node kind: 0 shooting, 1 Radau)."""
    import re
    txt = open(os.path.join(ROOT, "awebox_amd", "csrc", "ap2_nodehess.gen.hpp")).read()
    get = lambda name: [int(x) for x in re.search(r"%s\[2\] = \{(\d+), (\d+)\}" % name, txt).groups()]  # noqa: E731
    return get("kFlops"), get("kTranscendental")


def hessian_block(ev, V, P, B, lay, dev, steps=10):
    """nlp_hess_l throughput (sigma = 1, lam ~ N(0,1) seed 7), reported beside the
    headline metric; kernel time from the library's HIP events.  The default Hessian at this batch is
    the generated one (awe_eval_hess_im, H instance-minor as the solver reads it); the hyper-dual
    colour-pair kernel is timed beside it (3 calls)."""
    import numpy as np
    import torch
    sig = torch.ones(B, dtype=torch.float64, device=dev)
    lam = torch.tensor(np.random.default_rng(7).standard_normal((B, lay.n_g)), device=dev)
    out = {}
    for path, n in (("generated", steps), ("hyperdual", 3)):
        ev.hess_path = path
        if path == "generated":
            H = ev.alloc_hess(dev)
            call = lambda: ev.eval_hess_device_im(V, P, sig, lam, H)  # noqa: E731
        else:
            H = torch.empty(B, ev.nnz_h, dtype=torch.float64, device=dev)
            call = lambda: ev.eval_hess_device(V, P, sig, lam, H)  # noqa: E731
        call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kms = []
        for _ in range(n):
            call()
            kms.append(ev.last_hess_ms())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        rec = {"metric": "nlp_hess_l evals/sec", "value": B / dt, "unit": "evals/s", "ms_per_step": dt * 1e3,
               "kernel_ms": float(np.mean(kms)), "nnz_h": ev.nnz_h, "batch": B,
               "finite": bool(torch.isfinite(H).all().item())}
        if path == "generated":
            out.update(rec)
            out["path"] = "generated (ap2_hgen_*: forward-over-reverse node code + assembly, H instance-minor)"
            (f0, f1), (t0_, t1_) = hess_gen_counts()
            d = lay.d
            flops = lay.n_k * ((f0 + t0_) + d * (f1 + t1_))       # node code per instance; transcendentals as 1
            byts = 8.0 * (lay.n_v + lay.n_p + lay.n_g + 1 + ev.nnz_h)   # V, P, lam, sigma in; H out
            kms_mean = float(np.mean(kms)) * 1e-3
            out["roofline"] = {
                "bound": "fp64", "unit": "TFLOP/s", "peak": FP64_PEAK_TFLOPS,
                "flops_per_eval": flops, "achieved": flops * B / kms_mean / 1e12,
                "frac": flops * B / kms_mean / 1e12 / FP64_PEAK_TFLOPS,
                "hbm": {"bytes_per_eval": byts, "achieved_GBps": byts * B / kms_mean / 1e9,
                        "frac": byts * B / kms_mean / 1e9 / HBM_PEAK_GBS},
                "note": "algorithmic: the generated node code's operations (kFlops + kTranscendental of "
                        "csrc/ap2_nodehess.gen.hpp) per node, assembly not counted; bytes = V, P, lam, sigma in "
                        "and H out once"}
        else:
            out["hyperdual"] = rec
            rl = hess_roofline(B, float(np.mean(kms)))
            if rl is not None:
                out["hyperdual"]["roofline"] = rl
    ev.hess_path = "follow"
    return out


def hess_roofline(B, kernel_ms):
    """FP64 issue roofline of ap2_hess_kernel from its committed PMC record (profiles/pmc_hess.json,
    tools/gpu_pmc_all.sh at 256 instances): FP64 lane operations per instance (ADD + MUL + 2 FMA +
    TRANS, x 64 lanes; they scale with the instance count) x B / the kernel time, against the
    78.6 TFLOP/s FP64 vector peak; HBM bytes 2 x FETCH + WRITE likewise.  None if the record was
    taken on other sources."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_hess.json")) as fh:
            rec = json.load(fh)
    except (OSError, ValueError):
        return None
    if rec.get("source_hash") != kernel_source_hash():
        return None
    per = rec["batch"]
    ops = (rec["SQ_INSTS_VALU_ADD_F64"] + rec["SQ_INSTS_VALU_MUL_F64"] + 2.0 * rec["SQ_INSTS_VALU_FMA_F64"]
           + rec["SQ_INSTS_VALU_TRANS_F64"]) * 64.0 / per
    f64 = rec["SQ_INSTS_VALU_ADD_F64"] + rec["SQ_INSTS_VALU_MUL_F64"] + rec["SQ_INSTS_VALU_FMA_F64"] + \
        rec["SQ_INSTS_VALU_TRANS_F64"]
    achieved = ops * B / (kernel_ms * 1e-3) / 1e12
    hbm = (2.0 * rec["FETCH_SIZE_kB"] + rec["WRITE_SIZE_kB"]) * 1024 / per * B / (kernel_ms * 1e-3) / 1e9
    return {"bound": "fp64", "achieved": achieved, "peak": 78.6, "unit": "TFLOP/s", "frac": achieved / 78.6,
            "kernel": "ap2_hess_kernel<4>", "valu_f64_share": f64 / rec["SQ_INSTS_VALU"],
            "wait_frac": rec["SQ_WAIT_ANY"] / rec["SQ_WAVE_CYCLES"], "occupancy_waves_per_simd": 1,
            "hbm_GBps": hbm, "pmc_record": "profiles/pmc_hess.json"}


def casadi_probe():
    """BASELINE.md's CPU-baseline rule: probe `import casadi` on the box; the reference's CasADi +
    IPOPT path is the CPU baseline only if it imports (it never has: no casadi wheel in the image),
    otherwise the C++ CPU port is (cpu_baseline.kind = "port").  A child process, so a failing import
    cannot disturb this one."""
    import subprocess
    r = subprocess.run([sys.executable, "-c", "import casadi; print(casadi.__version__)"], capture_output=True,
                       text=True, timeout=120)
    return {"importable": r.returncode == 0,
            "detail": (r.stdout.strip() if r.returncode == 0 else (r.stderr.strip().splitlines() or [""])[-1])[:200]}


def latency_block(consts, lay, v0, with_cpu=True, reps=50):
    """Config 2's drop-in case: IPOPT on the host calls one NLP evaluation at a time through the
    CasADi Callback.  Host round-trip latency (host arrays in and out, one instance) of the C-ABI's
    host entry points -- awe_eval_f_host / awe_eval_g_host (value-only kernel) and
    awe_eval_nlp_host (f, g, grad f, J_g) -- median of `reps`, beside the 1-thread CPU port."""
    import numpy as np

    from awebox_amd import problem as pb
    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.initial_guess import batch_member
    ev = Ap2Evaluator(consts, batch=1)
    V = batch_member(v0, lay, 0).reshape(1, -1)
    P = pb.pack_p(lay, consts, v0).reshape(1, -1)

    def med(fn):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3

    lam = np.random.default_rng(7).standard_normal((1, lay.n_g))
    out = {"unit": "ms", "instances": 1,
           "nlp_f_host": med(lambda: ev.eval_f(V, P)), "nlp_g_host": med(lambda: ev.eval_g(V, P)),
           "nlp_f_g_grad_jac_host": med(lambda: ev.eval_nlp(V, P)),
           # nlp_hess_l: once per IPOPT iteration through the Callback; default at batch 1 the
           # hyper-dual kernel (follows the colour evaluation path), the generated one beside it
           "nlp_hess_l_host": med(lambda: ev.eval_hess(V, P, 1.0, lam))}
    ev.hess_path = "generated"
    out["nlp_hess_l_host_generated"] = med(lambda: ev.eval_hess(V, P, 1.0, lam))
    ev.hess_path = "follow"
    if with_cpu:
        from oracle.cpu_port import CpuPort
        port = CpuPort(consts)
        out["cpu_port_1thread_f_g_grad_jac"] = med(lambda: port.eval_nlp(V, P, threads=1))
    return out


def cpu_baseline(consts, lay, v0, seconds):
    """Time the CPU port of the evaluator (test/baseline infrastructure, never the product) on
    the host cores: all threads OpenMP grants (OMP_NUM_THREADS), and one thread."""
    import numpy as np

    from awebox_amd import problem as pb
    from awebox_amd.initial_guess import batch_member
    from oracle.cpu_port import CpuPort

    port = CpuPort(consts)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)

    def rate(B, nthreads):
        V = np.stack([batch_member(v0, lay, b) for b in range(B)])
        P = np.stack([pb.pack_p(lay, consts, v0)] * B)
        port.eval_nlp(V, P, threads=nthreads)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            port.eval_nlp(V, P, threads=nthreads)
            n += B
        return n / (time.perf_counter() - t0), n

    all_rate, n_all = rate(max(4 * threads, 16), threads)
    one_rate, n_one = rate(8, 1)
    return {"value": all_rate, "unit": "evals/s", "cores": threads, "kind": "port",
            "value_1core": one_rate,
            "sample": f"C++ CPU port of the evaluator (oracle/cpu, vector-dual forward mode, OpenMP over "
                      f"(instance, interval)): {n_all} evaluations (f, g, grad f, J_g) of the AP2 N=40 d=4 NLP "
                      f"on {threads} threads and {n_one} on 1 thread, ~{seconds:.0f} s each"}


if __name__ == "__main__":
    main()
