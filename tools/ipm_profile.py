"""Profile the interior-point solver's phases on the AP2 problem (first homotopy step, N=40 d=4):
per-phase seconds (evaluations, Hessian, KKT factor / solve), and one structured KKT
factor + solve under torch.profiler.  Writes gpurun_out/ipm_profile.json."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-k", type=int, default=40)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--separators", default="dense", help="separator solve of the structured KKT: dense | btd")
    args = ap.parse_args()
    import numpy as np
    import torch
    from awebox_amd import homotopy as hm
    from awebox_amd import problem as pb
    from awebox_amd.initial_guess import initial_guess
    from awebox_amd.ipm import DeviceNlp, IpmOptions, StructuredKKT, solve
    from awebox_amd.trajectory import hippo_options
    if args.device == "cuda":
        from awebox_amd.build import build
        from awebox_amd.evaluator import Ap2Evaluator
        build()
        make = lambda c: Ap2Evaluator(c, batch=1)  # noqa: E731
    else:
        from oracle.cpu_device import CpuDeviceEvaluator as make
    consts = pb.build_constants(pb.Ap2Config(n_k=args.n_k, d=4))
    lay = pb.NlpLayout(args.n_k, 4)
    ev = make(consts)
    v0 = initial_guess(consts, lay)
    st = hm.schedule(consts, lay, v0)[0]
    lbg, ubg = lay.g_bounds()
    P = pb.pack_p(lay, consts, v0, step=st.cost_step)
    opts = hippo_options("initial", IpmOptions(max_iter=args.iters, profile=True,
                                                      separators=args.separators))
    res = solve(ev, P, v0, st.lbx, st.ubx, lbg, ubg, opts=opts, device=args.device)
    out = {"iterations": res.iterations, "status": res.status, "seconds": res.seconds,
           "timing": res.timing, "kkt_solves": res.kkt_solves, "kkt_dense": res.kkt_dense}
    print(json.dumps(out, indent=1), flush=True)
    # one factor + solve in isolation
    nlp = DeviceNlp(ev, P, st.lbx, st.ubx, lbg, ubg, args.device)
    sk = StructuredKKT(nlp, lay, args.device, separators=args.separators)
    x = torch.tensor(v0[nlp.free], device=args.device)
    f, grad, g, jv = nlp.eval_all(x)
    hv = nlp.hess(x, torch.zeros(nlp.m, dtype=torch.float64, device=args.device))
    diag = torch.ones(nlp.ny, dtype=torch.float64, device=args.device)
    rhs = torch.randn(sk.N, dtype=torch.float64, device=args.device)
    for _ in range(2):
        sk.factor(hv, diag, jv, 0.0, nlp.mI)
        sol = sk.solve(rhs)
    bwd = float(((rhs - sk.matvec(sol.unsqueeze(0))[0]).abs().max()
                 / (sk.k_norm[0] * sol.abs().max() + rhs.abs().max())).item())
    print(json.dumps({"separator_path": "btd" if getattr(sk, "use_btd", False) else "dense",
                      "backward_error": bwd, "n_dense": sk.n_dense}), flush=True)
    sync = torch.cuda.synchronize if args.device == "cuda" else (lambda: None)
    sync()
    t = time.perf_counter()
    for _ in range(5):
        sk.factor(hv, diag, jv, 0.0, nlp.mI)
    sync()
    t_f = (time.perf_counter() - t) / 5
    t = time.perf_counter()
    for _ in range(5):
        sk.solve(rhs)
    sync()
    t_s = (time.perf_counter() - t) / 5
    out.update(N=sk.N, nS=sk.nS, nI=sk.nI, L=sk.L, factor_ms=t_f * 1e3, solve_ms=t_s * 1e3)
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if args.device == "cuda" else [])
    with profile(activities=acts) as prof:
        sk.factor(hv, diag, jv, 0.0, nlp.mI)
        sk.solve(rhs)
        sync()
    table = prof.key_averages().table(sort_by="cuda_time_total" if args.device == "cuda" else "cpu_time_total",
                                      row_limit=25)
    print(table, flush=True)
    print(json.dumps({k: out[k] for k in ("N", "nS", "nI", "L", "factor_ms", "solve_ms")}), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ipm_profile.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
