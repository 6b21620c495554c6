#!/bin/bash
# Round 6, after the inertia-kernel barrier fix: the lazy probe (4 batched final steps of 128
# identical instances), the det GPU tests, the default homotopy alone and at B = 128.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -4 "gpurun_out/$log" | cut -c1-1000
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 700 lazy2.log python -u tools/lazy_probe.py --B 128 --runs 4
step 600 det_gpu2.log python -u -m pytest -x -v --durations=10 --timeout 300 --timeout-method thread tests/test_det_gpu.py tests/test_batched_lu.py tests/test_inertia.py
step 900 regress2.log python -u -m pytest -v -s --durations=10 --timeout 800 --timeout-method thread tests/test_regression.py -k "converges_and_repeats or default_path_meets or b128"
echo R06_INV2_DONE
