#!/bin/bash
# Instance-minor path after a kernel change: path + oracle parity tests, then the bench's AP2 block
# timing (tools/soa_variants.py on the in-tree library) with output checksums.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gen_path_gpu.py tests/test_gpu_parity.py -m gpu -k "not hessian" > gpurun_out/pytest_soa_check.log 2>&1 || { tail -40 gpurun_out/pytest_soa_check.log; exit 1; }
tail -2 gpurun_out/pytest_soa_check.log
timeout -k 10 300 python -u tools/soa_variants.py awebox_amd/libawegpu.so > gpurun_out/soa_check.log 2>&1 || { cat gpurun_out/soa_check.log; exit 1; }
cat gpurun_out/soa_check.log
