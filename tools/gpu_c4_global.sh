#!/bin/bash
# Config 4 in the reference's order: one chain over all 64 points on one GPU
# (tools/config4_full.py --global-chain).  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1050 python -u tools/config4_full.py --global-chain > gpurun_out/config4_global_chain.log 2>&1
rc=$?
tail -c 3000 gpurun_out/config4_global_chain.log
exit $rc
