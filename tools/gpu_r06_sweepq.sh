#!/bin/bash
# Quick: the bench's AP2 and dual sweep blocks only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
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
