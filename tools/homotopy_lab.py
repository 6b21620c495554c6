"""Solver lab: run the AP2 N=40 homotopy once per IpmOptions variant (JSON list of overrides) on
the GPU and print, per variant, every step's iterations, status, period and power -- the data
for locating where a solver variant's path leaves the reference's 35 s orbit family."""
import argparse
import dataclasses
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default='[{}]', help="JSON list of IpmOptions overrides")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "homotopy_lab.jsonl"))
    ap.add_argument("--u-ref", type=float, default=10.0)
    ap.add_argument("--cpu", action="store_true")
    args = ap.parse_args()
    from awebox_amd import problem as pb
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.trajectory import optimize
    consts = pb.build_constants(pb.Ap2Config(u_ref=args.u_ref))
    if args.cpu:
        from oracle.cpu_device import CpuDeviceEvaluator
        ev, device = CpuDeviceEvaluator(consts), "cpu"
    else:
        from awebox_amd.evaluator import Ap2Evaluator
        ev, device = Ap2Evaluator(consts, batch=1), "cuda"
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    lay = pb.NlpLayout(consts.cfg.n_k, consts.cfg.d)
    i_tf = int(lay.theta()[1])
    s_tf = float(consts.scaling[pb.W_TH0 + 1])
    for var in json.loads(args.variants):
        periods = []

        def cb(it, V, stepped):
            periods.append(float(V[0, i_tf]) * s_tf)
        opts = dataclasses.replace(IpmOptions(max_iter=2000, callback=cb), **var)
        t0 = time.perf_counter()
        V, summary, out, _ = optimize(consts, ev, opts, device=device, keep_logs=True)
        steps, pos = [], 0
        for s in summary:
            log = s["log"]
            n_it = len(log)
            rec_s = {k: s[k] for k in ("step", "status", "iterations", "f", "period_s", "avg_power_W")}
            if s["step"].startswith("final"):
                tr = periods[pos:pos + n_it]
                rec_s["trace"] = [dict(T=round(t, 3), mu=l["mu"], a=round(l["alpha"], 4), dw=l["delta_w"],
                                       bt=l["backtracks"], soc=l["soc"], f=round(l["f"], 6))
                                  for t, l in zip(tr, log)]
            pos += n_it
            steps.append(rec_s)
        rec = {"variant": var, "seconds": time.perf_counter() - t0, "outputs": out, "steps": steps}
        line = json.dumps(rec, default=float)
        print(line, flush=True)
        with open(args.out, "a") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
