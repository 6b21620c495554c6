#!/bin/bash
# Reproducibility of the N=40 homotopy with the deterministic KKT assembly and matvec: two runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python -u tools/solve_ap2.py --n-k 40 --out gpurun_out/solve_ap2_det_$i.json > gpurun_out/solve_det_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/solve_det_$i.log | cut -c1-200
done
