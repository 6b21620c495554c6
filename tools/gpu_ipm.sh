#!/bin/bash
# Interior-point solver on the GPU: solver tests, N=40 profile, the AP2 N=40 homotopy and the AP2 /
# dual-kite 4-point sweeps (dense separator LU).  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -2 "gpurun_out/$log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step 400 solver_gpu_tests.log python -u -m pytest tests/test_solver.py tests/test_fd_hessian.py -m gpu -x -q --timeout 300 --timeout-method thread
step 200 ipm_profile_n40.log python -u tools/ipm_profile.py --n-k 40 --iters 40
step 300 solve_ap2.log python -u tools/solve_ap2.py --n-k 40 --out gpurun_out/solve_ap2_n40.json
step 300 sweep_ap2.log python -u -m awebox_amd.sweep --points 4 --out gpurun_out/sweep_ap2_4pts.json
step 400 sweep_dual.log python -u -m awebox_amd.sweep --arch dual --points 4 --n-k 20 --d 4 --max-iter 1500 --out gpurun_out/sweep_dual_n20_4pts.json
