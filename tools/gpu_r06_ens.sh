#!/bin/bash
# Round 6: final-step branch ensembles (32 members, 1e-13) on the three evaluation paths with the
# batch-invariant solver; the dual fan-shard partition test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 700 "gpurun_out/$log"; echo
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step 400 ens_col.log python -u tools/final_step_ensemble.py --path colour --k 32 --eps 1e-13
step 400 ens_gen.log python -u tools/final_step_ensemble.py --path generated --k 32 --eps 1e-13
step 400 ens_soa.log python -u tools/final_step_ensemble.py --path soa --k 32 --eps 1e-13
step 500 dual_part.log python -u -m pytest -x -v -s --timeout 450 --timeout-method thread tests/test_det_gpu.py -k dual
echo R06_ENS_DONE
