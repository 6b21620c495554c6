#!/bin/bash
# Final-step branch records: the unperturbed homotopy per evaluation path
# (tools/homotopy_branch.py), then 16-member 1e-13 ensembles of the final step per path
# (tools/final_step_ensemble.py), the Hessian following the path.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 2500 "gpurun_out/$log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 500 branch.log python -u tools/homotopy_branch.py
for p in colour generated soa; do
    step 400 ens_$p.log python -u tools/final_step_ensemble.py --path $p --k 16 --eps 1e-13 \
        --out gpurun_out/final_step_ensemble.jsonl
done
step 600 batch_homotopy.log python -u tools/batch_homotopy.py 128
echo BRANCH_DONE
