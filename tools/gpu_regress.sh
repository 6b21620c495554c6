#!/bin/bash
# The AP2 regression tests on the GPU (anchors, branch ensembles, batched homotopy).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_regression.py -m gpu > gpurun_out/pytest_regress.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|colour \{|generated \{" gpurun_out/pytest_regress.log | tail -30
exit $rc
