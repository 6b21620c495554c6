#!/bin/bash
# Generated vs hyper-dual Hessian: GPU parity tests of both paths, then tools/hess_paths.py timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "hessian" > gpurun_out/pytest_hess.log 2>&1 || { tail -60 gpurun_out/pytest_hess.log; exit 1; }
tail -12 gpurun_out/pytest_hess.log
timeout -k 10 300 python -u tools/hess_paths.py 2048 > gpurun_out/hess_paths.log 2>&1 || { cat gpurun_out/hess_paths.log; exit 1; }
cat gpurun_out/hess_paths.log
