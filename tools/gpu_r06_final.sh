#!/bin/bash
# Round 6 round-end record: default bench, rocprof stats of the bench's AP2 block alone and of the
# AP2 sweep block alone.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 400 "gpurun_out/$log"; echo
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 700 bench.log python bench.py
step 300 rocprof_ap2.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ap2 -o run --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --sweep-points 0 --dual-sweep-points 0 --no-hessian --no-latency
find gpurun_out/prof_ap2 -name '*_trace.csv' -size +4M -delete
step 400 rocprof_sweep.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sweep -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --dual-sweep-points 0 --no-hessian
find gpurun_out/prof_sweep -name '*_trace.csv' -size +4M -delete
echo R06_FINAL_DONE
