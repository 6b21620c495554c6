#!/bin/bash
# A/B of the block-tridiagonal apply launch (right-hand sides split over workgroups) against the
# previous build: times and bitwise identity of factors and solutions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
O=gpurun_out/btdab
mkdir -p $O
timeout -k 10 300 python -u tools/awelu_ab.py --btd-only --base tools/ab_r06/libawelu_base.so > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.log | cut -c1-400
