#!/bin/bash
# The wide gather-sum lists in one launch: bitwise tests, then the bench's sweep and MPC blocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
O=gpurun_out/wide
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gather_sum.py tests/test_det_gpu.py -m gpu -k "gather or kkt or fan_shard_warm" > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 600 python -u bench.py --steps 1 --warmup 0 --batch 8 --no-cpu-baseline --no-hessian --no-latency --dual-batch 0 --mpc-batch 64 --pmpc-loops 64 --no-dual-chain > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.readline())
for k in ('sweep','dual_sweep'):
    v=d[k]; print(k, v['value'], v['iterations'], v['avg_power_W'])
c=d['mpc']['converged']; print('pmpc', c['ms_per_step'], c['realtime_factor'], c['ipm_iterations_max'], c['tracking_error_max'])
"
