#!/bin/bash
# GPU check: the named pytest selection (default: the whole -m gpu suite), then smoke.
# A failure ends the script.  Usage: tools/gpu_check.sh [pytest args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -3 "gpurun_out/$log"
    if [ $rc -ne 0 ]; then exit $rc; fi
}
if [ $# -eq 0 ]; then set -- tests -m gpu; fi
step 1100 pytest_gpu.log python -u -m pytest -x -v --durations=25 --timeout 600 --timeout-method thread "$@"
step 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
echo CHECK_DONE
