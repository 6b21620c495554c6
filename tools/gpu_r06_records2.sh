#!/bin/bash
# Round 6 final records on the fused-solver sources: the default bench, and the kernel-trace
# statistics of the bench's AP2 and dual-kite sweep blocks alone (tools/sweep_record.py inputs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rec2
export TMPDIR=/tmp
O=gpurun_out/rec2
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "$O/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 300 "$O/$log"; echo
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 700 bench.log python -u bench.py
step 400 rocprof_sweep.log rocprofv3 --kernel-trace --stats -d $O/prof_sweep -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --dual-sweep-points 0 --no-hessian --no-latency
find $O/prof_sweep -name '*_trace.csv' -delete
step 400 rocprof_dsweep.log rocprofv3 --kernel-trace --stats -d $O/prof_dsweep -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --sweep-points 0 --no-hessian --no-latency --no-dual-chain
find $O/prof_dsweep -name '*_trace.csv' -delete
echo R06_RECORDS2_DONE
