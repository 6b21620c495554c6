#!/bin/bash
# Dual-kite generated path: parity tests (generated vs oracle and colour kernel), path timing.
# A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dual_gen
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_dual_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k generated > gpurun_out/dual_gen/pytest.log 2>&1 || { tail -40 gpurun_out/dual_gen/pytest.log; exit 1; }
tail -5 gpurun_out/dual_gen/pytest.log
timeout -k 10 300 python -u tools/dual_paths.py "$@" > gpurun_out/dual_gen/paths.log 2>&1 || { cat gpurun_out/dual_gen/paths.log; exit 1; }
cat gpurun_out/dual_gen/paths.log
