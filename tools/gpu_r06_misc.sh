#!/bin/bash
# Round 6: the batch-mode sweep partition test, and where the converged MPC's sampling time goes
# (tools/pmpc_profile.py: phase timer and cProfile).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 600 "gpurun_out/$log"; echo
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 500 batch_sweep_test.log python -u -m pytest -x -v -s --timeout 450 --timeout-method thread tests/test_det_gpu.py -k batch_mode
step 400 pmpc_profile.log python -u tools/pmpc_profile.py
echo R06_MISC_DONE
