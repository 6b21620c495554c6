#!/bin/bash
# Round 6: instance-minor inputs (awe_eval_nlp_imv) -- the bitwise test, the AP2 headline block of
# bench.py alone, the headline PMC passes on the new call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 600 "gpurun_out/$log"; echo
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 300 imv_test.log python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gen_path_gpu.py tests/test_gpu_parity.py
step 300 bench_ap2.log python -u bench.py --steps 20 --warmup 3 --no-hessian --no-latency --no-cpu-baseline --mpc-batch 0 --dual-batch 0 --sweep-points 0 --dual-sweep-points 0
bash tools/gpu_pmc_soa.sh || exit $?
echo R06_IMV_DONE
