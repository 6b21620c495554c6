#!/bin/bash
# Config-5 session: MPC GPU tests (evaluator, Hessian, converged MPC), then the bench's MPC blocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mpc.py tests/test_mpc_solve.py -m gpu -x -v --durations=10 --timeout 300 --timeout-method thread > gpurun_out/pytest_mpc.log 2>&1 || { tail -30 gpurun_out/pytest_mpc.log; exit 1; }
tail -15 gpurun_out/pytest_mpc.log
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --batch 8 --no-cpu-baseline --no-hessian --no-latency --dual-batch 0 --sweep-points 0 --dual-sweep-points 0 > gpurun_out/bench_mpc.log 2>&1 || { tail -30 gpurun_out/bench_mpc.log; exit 1; }
tail -c 2500 gpurun_out/bench_mpc.log
echo MPC_DONE
