#!/bin/bash
# Quick GPU round: evaluator parity (oracle + generated vs colour), the AP2 bench block alone
# (HIP-event kernel times), then the final-step ensembles.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 1200 "gpurun_out/$log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 400 pytest_parity.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gen_path_gpu.py -m gpu
step 300 bench_ap2.log python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-hessian --no-latency \
    --mpc-batch 0 --pmpc-loops 0 --dual-batch 0 --dual-sweep-points 0 --sweep-points 0
if [ "${1:-}" = "ens" ]; then
    step 400 ens_gen.log python -u tools/final_step_ensemble.py --path generated --k 16 --eps 1e-13 --trace gpurun_out/ens_trace_gen.json
    step 400 ens_col.log python -u tools/final_step_ensemble.py --path colour --k 16 --eps 1e-13 --trace gpurun_out/ens_trace_col.json
fi
if [ "${2:-}" = "c4" ]; then
    step 1100 config4_full.log python -u tools/config4_full.py --mode fan --shards 0-7
fi
echo QUICK_DONE
