#!/bin/bash
# Block-tridiagonal kernels after a change: their GPU tests and the solver tests, then the sweep
# block alone under the kernel tracer (btd_factor / btd_apply averages, sweep wall time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_batched_lu.py tests/test_solver.py tests/test_regression.py -m gpu > gpurun_out/pytest_btd.log 2>&1 || exit $?
echo TESTS_OK
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --dual-sweep-points 0 --no-hessian > gpurun_out/bench_sweep.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sweep2 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --dual-sweep-points 0 --no-hessian > gpurun_out/rocprof_sweep2.log 2>&1 || exit $?
find gpurun_out/prof_sweep2 -name '*_trace.csv' -size +4M -delete
echo BTD_DONE
