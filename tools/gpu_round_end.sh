#!/bin/bash
# Round-end records in one GPU session: GPU suite, smoke, default bench, rocprof kernel statistics
# of the bench's AP2 block alone (the instance-minor path's kernels), the PMC passes of those kernels
# (tools/gpu_pmc_soa.sh) and of the config-3 / config-5 kernels (tools/gpu_pmc_configs.sh).  A
# failure ends the script.
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
step 900 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations 10
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
step 600 bench.log python bench.py
step 300 rocprof_ap2.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ap2 -o run --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --sweep-points 0 --dual-sweep-points 0 --no-hessian --no-latency
find gpurun_out/prof_ap2 -name '*_trace.csv' -size +4M -delete
step 500 pmc_soa.log bash tools/gpu_pmc_soa.sh
step 400 pmc_configs.log bash tools/gpu_pmc_configs.sh
echo ROUND_END_DONE
