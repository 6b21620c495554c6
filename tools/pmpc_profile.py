"""Where the converged MPC's sampling time goes: BatchedPmpc (64 loops, N=20 d=4) for a few steps
with the interior-point phase timer (IpmOptions.profile, synchronising) and, separately, cProfile
of the host side without the timer."""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loops", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmpc_profile.json"))
    args = ap.parse_args()
    import torch

    from awebox_amd import kite3 as k3
    from awebox_amd.ipm import IpmOptions
    from awebox_amd.mpc_solve import BatchedPmpc
    c = k3.build_constants()
    out = {}
    for mode in ("phases", "cprofile"):
        pm = BatchedPmpc(c, args.loops, device="cuda", opts=IpmOptions(profile=(mode == "phases")))
        pm.start()
        pm.simulate_reference(args.steps + 2 + c.cfg.n_k + 1)
        pm.step()
        torch.cuda.synchronize()
        prof = cProfile.Profile() if mode == "cprofile" else None
        t0 = time.perf_counter()
        timing, iters = {}, []
        if prof:
            prof.enable()
        for _ in range(args.steps):
            o = pm.step()
            iters.append(o["iterations"].tolist())
            for r in pm.results[:1]:
                for k, v in (r.timing or {}).items():
                    timing[k] = timing.get(k, 0.0) + v
        torch.cuda.synchronize()
        if prof:
            prof.disable()
        el = time.perf_counter() - t0
        out[mode] = {"ms_per_step": el / args.steps * 1e3, "iterations": iters,
                     "phase_ms_per_step": {k: v / args.steps * 1e3 for k, v in timing.items()}}
        if prof:
            s = io.StringIO()
            pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(40)
            pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(60)
            st = pstats.Stats(prof, stream=s)
            st.print_callees("solve_batch")
            st.print_callers("method 'cpu'")
            st.print_callers("method 'item'")
            st.print_callers("torch.tensor")
            out[mode]["top"] = s.getvalue()
        print(json.dumps({k: v for k, v in out[mode].items() if k != "top"}), flush=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(out["cprofile"]["top"])


if __name__ == "__main__":
    main()
