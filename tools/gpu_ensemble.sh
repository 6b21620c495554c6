#!/bin/bash
# Final-step branch ensembles on the GPU (tools/final_step_ensemble.py): K members from the power1
# point perturbed by eps, per evaluation path and solver variant.  A failure ends the script.
#   tools/gpu_ensemble.sh [variants-json]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VARS=${1:-'[{}]'}
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 1500 "gpurun_out/$log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 400 ens_gen.log python -u tools/final_step_ensemble.py --path generated --k 16 --eps 1e-13 \
    --variants "$VARS" --trace gpurun_out/ens_trace_gen.json
step 400 ens_col.log python -u tools/final_step_ensemble.py --path colour --k 16 --eps 1e-13 \
    --variants "$VARS" --trace gpurun_out/ens_trace_col.json
echo ENSEMBLE_DONE
