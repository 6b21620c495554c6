#!/bin/bash
# Round 6: chunking A/B of the instance-minor path, then the whole GPU suite and smoke.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== $log rc=$rc"; tail -c 1500 "gpurun_out/$log"; echo
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}

step 1000 pytest_gpu.log python -u -m pytest -v --durations=30 --timeout 600 --timeout-method thread tests -m gpu
step 200 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
echo R06_SUITE_DONE
