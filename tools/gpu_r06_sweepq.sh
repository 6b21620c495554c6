#!/bin/bash
# Quick: the bench's AP2 and dual sweep blocks only, then a kernel-trace summary of the converged
# MPC block alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/sweepq
mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --no-hessian --no-latency --no-dual-chain > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.readline())
for k in ('sweep','dual_sweep'):
    v=d.get(k)
    if isinstance(v,dict): print(k, {kk: v.get(kk) for kk in ('value','wall_s','iterations')})
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pmpc_prof -o run --output-format csv -- python -u bench.py --steps 1 --warmup 0 --batch 8 --no-cpu-baseline --no-hessian --no-latency --dual-batch 0 --mpc-batch 64 --pmpc-loops 64 --sweep-points 0 --dual-sweep-points 0 > $O/pmpc_prof.log 2>&1 || { tail -20 $O/pmpc_prof.log; exit 1; }
find $O/pmpc_prof -name '*_trace.csv' -delete
echo SWEEPQ_DONE
