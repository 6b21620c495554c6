#!/bin/bash
# Phase timings of the batched interior-point solver (8 AP2 wind speeds, N=40 d=4,
# IpmOptions(profile=True): evaluations, Hessian, KKT factor / solve, inertia, line search).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/batch_profile.py --batch 8 --profile --out gpurun_out/batch_profile_b8.json > gpurun_out/batch_profile_b8.log 2>&1 || exit $?
echo PROFILE_DONE
