#!/bin/bash
# Instance-minor path A/B: path parity tests, then tools/soa_variants.py over the product library and
# the variant libraries given as arguments (tools/ab/*.so).  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gen_path_gpu.py -m gpu > gpurun_out/pytest_path.log 2>&1 || { tail -30 gpurun_out/pytest_path.log; exit 1; }
tail -3 gpurun_out/pytest_path.log
timeout -k 10 400 python -u tools/soa_variants.py awebox_amd/libawegpu.so "$@" > gpurun_out/soa_variants.log 2>&1 || { cat gpurun_out/soa_variants.log; exit 1; }
cat gpurun_out/soa_variants.log
