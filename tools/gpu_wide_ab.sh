#!/bin/bash
# Wide (paired 16-byte) vs narrow J_g stores on the instance-minor path: path and oracle parity tests
# on the default (wide) build, then tools/soa_variants.py over both store widths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gen_path_gpu.py tests/test_gpu_parity.py -m gpu > gpurun_out/pytest_wide.log 2>&1 || { tail -40 gpurun_out/pytest_wide.log; exit 1; }
tail -3 gpurun_out/pytest_wide.log
timeout -k 10 500 python -u tools/soa_variants.py awebox_amd/libawegpu.so awebox_amd/libawegpu.so:AWE_SOA_NARROW=1 > gpurun_out/wide_ab.log 2>&1 || { cat gpurun_out/wide_ab.log; exit 1; }
cat gpurun_out/wide_ab.log
