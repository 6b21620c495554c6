#!/bin/bash
# Round 6: config 4 in the reference's order from 8 reconciled shards (tools/config4_reconcile.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1130 python -u tools/config4_reconcile.py > gpurun_out/c4_reconcile.log 2>&1
rc=$?; echo "=== c4 rc=$rc"; tail -c 1500 gpurun_out/c4_reconcile.log
