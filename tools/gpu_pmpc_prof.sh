#!/bin/bash
# kernel-trace statistics of the bench's converged-MPC block alone (64 loops)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pmpc_prof -o run --output-format csv -- python -u bench.py --steps 1 --warmup 0 --batch 8 --no-cpu-baseline --no-hessian --no-latency --dual-batch 0 --mpc-batch 64 --pmpc-loops 64 --sweep-points 0 --dual-sweep-points 0 > gpurun_out/pmpc_prof.log 2>&1 || exit 1
find gpurun_out/pmpc_prof -name '*_trace.csv' -size +4M -delete
tail -c 400 gpurun_out/pmpc_prof.log
