#!/bin/bash
# Round 6: which setting lets identical instances of a batched final step diverge
# (tools/batch_final_members.py, B = 128, two repeats each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; grep rep "gpurun_out/$log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 300 race_default.log python -u tools/batch_final_members.py
AWE_DET_OFF=1 step 300 race_detoff.log python -u tools/batch_final_members.py
AWE_EARLY_INERTIA_MAX_BLOCKS=0 step 300 race_noearly.log python -u tools/batch_final_members.py
echo R06_RACE_DONE
