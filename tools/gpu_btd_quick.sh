#!/bin/bash
# separator-sweep kernels only: awelu A/B against the round-5 baseline (times, bitwise identity)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/btd_quick
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/awelu_ab.py --base abv/libawelu_r05base.so --reps 10 --btd-only > gpurun_out/btd_quick/ab.log 2>&1
