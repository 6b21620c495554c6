#!/bin/bash
# AP2 sweep (rank 0's 8 points of linspace(5, 8, 64), N=40 d=4) in the three run_sweep modes, one GPU
# session: fan (homotopy of the first point + one batched warm start), batch (independent trials,
# every point's full homotopy side by side: awebox.Sweep.run's default, apply_sweeping_warmstart=False)
# and chain (sequential warm start, the config-4 example's apply_sweeping_warmstart=True).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mode in fan batch chain fan batch; do
    timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --batch 256 --no-cpu-baseline --no-hessian --no-latency \
        --mpc-batch 0 --dual-batch 0 --dual-sweep-points 0 --sweep-mode $mode > gpurun_out/sweep_mode_$mode.log 2>&1 || exit $?
    python -c "
import json,sys
for l in open('gpurun_out/sweep_mode_$mode.log'):
    if l.startswith('{'):
        s=json.loads(l)['sweep']; print('$mode', round(s['value'],3), s['wall_s'], s['iterations'], s['avg_power_W'], s['period_s'], flush=True)
"
done
