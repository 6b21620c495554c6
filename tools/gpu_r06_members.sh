#!/bin/bash
# Round 6: identical instances through a batched homotopy (tools/batch_members.py): default, without
# the side-stream inertia pass, and with the consistency probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -4 "gpurun_out/$log" | cut -c1-1500
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 300 members_default.log python -u tools/batch_members.py --B 128
AWE_EARLY_INERTIA_MAX_BLOCKS=0 step 300 members_noearly.log python -u tools/batch_members.py --B 128
step 400 members_probe.log python -u tools/batch_members.py --B 128 --probe
echo R06_MEMBERS_DONE
