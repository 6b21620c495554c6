#!/bin/bash
# Measurement half of the round-end check (the GPU suite and smoke are tools/gpu_check.sh): the
# default bench, rocprof stats of the bench's AP2 block alone and of the sweep block alone, and
# the host-side profile of the batched solver (tools/solver_pstats.py).  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -2 "gpurun_out/$log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 600 bench.log python bench.py
step 300 rocprof_ap2.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ap2 -o run --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --sweep-points 0 --dual-sweep-points 0 --no-hessian --no-latency
find gpurun_out/prof_ap2 -name '*_trace.csv' -size +4M -delete
step 400 rocprof_sweep.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sweep -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --dual-sweep-points 0 --no-hessian
find gpurun_out/prof_sweep -name '*_trace.csv' -size +4M -delete
step 300 solver_pstats.log python -u tools/solver_pstats.py
echo BENCH_DONE
