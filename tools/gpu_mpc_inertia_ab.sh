#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for arm in 512 1000000000 512 1000000000 512 1000000000; do
  AWE_EARLY_INERTIA_MAX_BLOCKS=$arm timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --batch 256 --no-cpu-baseline --no-hessian --no-latency --mpc-batch 32 --dual-batch 0 --sweep-points 0 --dual-sweep-points 0 > gpurun_out/mpc_ab_$arm.log 2>&1 || exit $?
  python -c "
import json
for l in open('gpurun_out/mpc_ab_$arm.log'):
    if l.startswith('{'):
        m=json.loads(l)['mpc']['converged']; print('$arm', round(m['ms_per_step'],1), m['ipm_iterations_max'], m['tracking_error_max'], flush=True)
"
done
