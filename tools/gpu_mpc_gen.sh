#!/bin/bash
# GPU session: MPC generated path parity + path timing + kernel trace
set -o pipefail
mkdir -p gpurun_out/mpc_gen
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_mpc.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/mpc_gen/pytest_mpc.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/mpc_paths.py > gpurun_out/mpc_gen/paths.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/mpc_gen/prof -o prof -- python3 tools/mpc_paths.py --steps 50 > gpurun_out/mpc_gen/prof.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_mpc_solve.py tests/test_rti.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/mpc_gen/pytest_solve.log 2>&1 || exit 1
