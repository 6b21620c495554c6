#!/bin/bash
# Instance-minor evaluation path: path parity (bitwise against node + gather, rounding against
# colour), oracle parity, the bench's AP2 block (per-path A/B in "paths"), and the rocprof kernel
# statistics of the same block.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 1500 "gpurun_out/$log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
AP2="--no-cpu-baseline --no-hessian --no-latency --mpc-batch 0 --pmpc-loops 0 --dual-batch 0 --dual-sweep-points 0 --sweep-points 0"
step 400 pytest_soa.log python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gen_path_gpu.py tests/test_gpu_parity.py -m gpu
step 300 bench_soa.log python -u bench.py --steps 30 --warmup 5 $AP2
step 300 rocprof_soa.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_soa -o run --output-format csv -- python bench.py --steps 30 --warmup 5 $AP2
find gpurun_out/prof_soa -name '*_trace.csv' -size +4M -delete
echo SOA_DONE
