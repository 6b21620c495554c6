#!/bin/bash
# Round 6, batch invariance on MI355X: the det.py kernels against their restatements, the structured
# KKT and the fan shard's warm start alone and batched, the default homotopy alone and at B = 128;
# then the headline PMC record (tools/gpu_pmc_soa.sh).  A pytest assertion failure (rc 1) lets the
# next step run; a crash, abort or time limit ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -4 "gpurun_out/$log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 600 det_gpu.log python -u -m pytest -x -v --durations=10 --timeout 300 --timeout-method thread tests/test_det_gpu.py
step 900 regress.log python -u -m pytest -v -s --durations=10 --timeout 800 --timeout-method thread tests/test_regression.py -k "converges_and_repeats or default_path_meets or b128"
if [ "${SKIP_PMC:-0}" = "0" ]; then bash tools/gpu_pmc_soa.sh || exit $?; fi
echo R06_INV_DONE
