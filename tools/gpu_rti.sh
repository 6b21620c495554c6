#!/bin/bash
# One GPU session for the config-5 closed loop: RTI GPU tests, the 256-loop closed-loop run, then
# (optionally) the stages of tools/gpu_check.sh.  A crash / timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rti.py -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/rti_tests.log 2>&1
rc=$?
tail -5 gpurun_out/rti_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/mpc_closed_loop.py --batch 256 --steps ${RTI_STEPS:-30} \
    --out gpurun_out/mpc_rti.json > gpurun_out/mpc_rti.log 2>&1 || exit $?
tail -2 gpurun_out/mpc_rti.log
if [ -n "$STAGES" ]; then bash tools/gpu_check.sh; fi
