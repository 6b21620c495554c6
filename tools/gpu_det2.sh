#!/bin/bash
# Deterministic KKT assembly as the default: GPU solver tests, the dual-kite 4-point sweep and
# the default bench.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -1 "gpurun_out/$log" | cut -c1-300
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 400 solver_gpu_tests.log python -u -m pytest tests/test_solver.py tests/test_fd_hessian.py -m gpu -x -q --timeout 300 --timeout-method thread
step 400 sweep_dual.log python -u -m awebox_amd.sweep --arch dual --points 4 --n-k 20 --d 4 --max-iter 1500 --out gpurun_out/sweep_dual_n20_4pts.json
step 300 sweep_ap2.log python -u -m awebox_amd.sweep --points 4 --out gpurun_out/sweep_ap2_4pts.json
step 600 bench.log python bench.py
