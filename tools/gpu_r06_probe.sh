#!/bin/bash
# Round 6: the det kernels' GPU tests, then the batch-consistency probe (tools/batch_consistency_probe.py).
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
step 600 det_gpu.log python -u -m pytest -v --durations=10 --timeout 300 --timeout-method thread tests/test_det_gpu.py
step 600 probe.log python -u tools/batch_consistency_probe.py --K 64
echo R06_PROBE_DONE
