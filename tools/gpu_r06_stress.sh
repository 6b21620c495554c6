#!/bin/bash
# Round 6: determinism of the batched inertia / LU kernels (tools/inertia_stress.py), and the batch
# consistency probe on the final step without the side-stream inertia pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -3 "gpurun_out/$log" | cut -c1-1500
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 300 stress.log python -u tools/inertia_stress.py
AWE_EARLY_INERTIA_MAX_BLOCKS=0 step 300 probe_noearly.log python -u tools/batch_consistency_probe.py --K 128
echo R06_STRESS_DONE
