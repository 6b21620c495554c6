#!/bin/bash
# KKT kernel tests, then the bench's converged-MPC block alone (64 loops) and its RTI block
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mpc_check
export TMPDIR=/tmp
O=gpurun_out/mpc_check
timeout -k 10 300 python -u tools/awelu_ab.py --base abv/libawelu_r05base.so --reps 10 > $O/ab.log 2>&1 || exit 1
grep -c '"factors_bitwise_equal": false\|"solution_bitwise_equal": false' $O/ab.log
grep '"op": "inertia"' $O/ab.log | cut -c1-200
timeout -k 10 600 python -u -m pytest tests/test_batched_lu.py tests/test_inertia.py tests/test_solver.py tests/test_mpc_solve.py tests/test_rti.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --steps 1 --warmup 0 --batch 8 --no-cpu-baseline --no-hessian --no-latency --dual-batch 0 --mpc-batch 256 --pmpc-loops 64 --sweep-points 0 --dual-sweep-points 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['mpc']['converged']; r=d['mpc']['rti']
print('pmpc ms', c['ms_per_step'], 'rt', c['realtime_factor'], 'it max', c['ipm_iterations_max'], 'track', c['tracking_error_median'], c['tracking_error_max'], 'rti', r['value'])"
