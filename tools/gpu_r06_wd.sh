#!/bin/bash
# Round 6: the watchdog's effect on the final step's branches (colour path, 32 members, with and
# without), and the chunking A/B of the instance-minor path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 800 "gpurun_out/$log"; echo
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 200 chunks_ab.log python -u tools/soa_chunks_ab.py
step 500 ens_wd.log python -u tools/final_step_ensemble.py --path colour --k 32 --eps 1e-13 --variants '[{"watchdog_shortened_iter_trigger": 0}, {}]'
step 400 ens_wd_gen.log python -u tools/final_step_ensemble.py --path generated --k 32 --eps 1e-13 --variants '[{}]'
echo R06_WD_DONE
