#!/bin/bash
# The default bench on the current sources, then the rocprof kernel-trace records of the bench's AP2
# and dual-kite sweep blocks (tools/gpu_records.sh STAGES=sweep; tools/sweep_record.py turns them into
# the bench's utilisation records).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -c 600 gpurun_out/bench.log
STAGES=sweep bash tools/gpu_records.sh
