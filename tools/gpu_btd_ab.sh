#!/bin/bash
# btd_factor A/B against a baseline build of libawelu (abv/libawelu_r05base.so): times and
# bitwise identity of factors and solutions on the AP2 / MPC chain shapes and random-pivot chains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/btd_ab
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/awelu_ab.py --base abv/libawelu_r05base.so --reps 10 > gpurun_out/btd_ab/ab.log 2>&1
rc=$?
cat gpurun_out/btd_ab/ab.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/btd_timing.py > gpurun_out/btd_ab/timing.log 2>&1
rc2=$?
cat gpurun_out/btd_ab/timing.log
exit $rc2
