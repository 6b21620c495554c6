#!/bin/bash
# Deterministic KKT assembly: the N=40 homotopy and the 2-point bench sweep (u_ref = 5, 8), each
# twice, to check reproducibility and convergence.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u tools/solve_ap2.py --n-k 40 --max-iter 1000 --deterministic --out gpurun_out/solve_ap2_det_$i.json > gpurun_out/solve_det_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/solve_det_$i.log | cut -c1-200
  timeout -k 10 300 python -u -m awebox_amd.sweep --points 2 --deterministic --out gpurun_out/sweep_det_$i.json > gpurun_out/sweep_det_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/sweep_det_$i.log
done
