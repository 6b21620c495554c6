"""GPU-busy fraction of the interior-point solver's workloads: the converged MPC (BatchedPmpc, 64
loops, N=20 d=4) and the AP2 sweep's batched warm start, under torch.profiler -- per step the
wall time, the summed device-kernel time, the number of kernel launches and the top kernels.

    python tools/solver_gpu_busy.py [--what mpc|sweep|both] [--out gpurun_out/solver_gpu_busy.json]
"""
import argparse
import collections
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _profile(fn, steps):
    import torch
    from torch.profiler import ProfilerActivity, profile
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
    dev_us = 0.0
    n_k = 0
    per = collections.Counter()
    cnt = collections.Counter()
    n_sync = 0
    for e in prof.events():
        dt = getattr(e, "device_type", None)
        if dt is not None and str(dt).endswith("CUDA"):
            d = e.device_time if hasattr(e, "device_time") else e.cuda_time
            dev_us += d
            n_k += 1
            per[e.name[:60]] += d
            cnt[e.name[:60]] += 1
        elif e.name in ("cudaStreamSynchronize", "hipStreamSynchronize", "cudaDeviceSynchronize",
                        "hipDeviceSynchronize", "hipMemcpyWithStream", "cudaMemcpyAsync", "hipMemcpyAsync"):
            n_sync += 1
    top = [{"kernel": k, "ms_per_step": v / 1e3 / steps, "launches_per_step": cnt[k] / steps}
           for k, v in per.most_common(15)]
    ops = sorted(((a.key, a.count) for a in prof.key_averages() if a.key.startswith("aten::")),
                 key=lambda t: -t[1])[:30]
    return {"ms_per_step": wall / steps * 1e3, "kernel_ms_per_step": dev_us / 1e3 / steps,
            "gpu_busy": dev_us / 1e6 / wall, "launches_per_step": n_k / steps,
            "copy_or_sync_calls_per_step": n_sync / steps, "top": top,
            "aten_ops_per_step": {k: c / steps for k, c in ops}}


def mpc(steps):
    import torch

    from awebox_amd import kite3 as k3
    from awebox_amd.mpc_solve import BatchedPmpc
    c = k3.build_constants()
    pm = BatchedPmpc(c, 64, device="cuda")
    pm.start()
    pm.simulate_reference(steps + 3 + c.cfg.n_k + 1)
    pm.step()
    torch.cuda.synchronize()
    return _profile(pm.step, steps)


def sweep(steps):
    import numpy as np

    from awebox_amd.evaluator import Ap2Evaluator
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    u = np.linspace(5.0, 8.0, 64)[:8]                 # rank 0's shard, as bench.py's sweep block
    state = {}

    def one():
        state["r"] = run_sweep(u, n_k=40, d=4, make_evaluator=lambda c, b=1: Ap2Evaluator(c, batch=b),
                               device="cuda", opts=IpmOptions(max_iter=1000), mode="fan")
    one()
    return _profile(one, steps)


def dual_sweep(steps):
    import numpy as np

    from awebox_amd.ipm import IpmOptions
    from awebox_amd.sweep import run_sweep
    from awebox_amd.dual_homotopy import make_evaluator
    u = np.linspace(5.0, 8.0, 64)[:8]                 # rank 0's shard of config 4
    state = {}

    def one():
        state["r"] = run_sweep(u, n_k=20, d=4, make_evaluator=lambda c, b=1: make_evaluator(c, device="cuda", batch=b),
                               device="cuda",
                               opts=IpmOptions(max_iter=3000), arch="dual", mode="fan")
    return _profile(one, steps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="both")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "solver_gpu_busy.json"))
    args = ap.parse_args()
    out = {}
    if args.what in ("mpc", "both"):
        out["mpc_converged_64"] = mpc(args.steps)
        print(json.dumps({k: v for k, v in out["mpc_converged_64"].items() if k != "top"}), flush=True)
    if args.what in ("sweep", "both"):
        out["ap2_sweep_8"] = sweep(1)
        print(json.dumps({k: v for k, v in out["ap2_sweep_8"].items() if k != "top"}), flush=True)
    if args.what == "dual":
        out["dual_sweep_8"] = dual_sweep(1)
        print(json.dumps({k: v for k, v in out["dual_sweep_8"].items() if k != "top"}), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
