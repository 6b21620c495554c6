#!/bin/bash
# Instance-minor node kernels: destination-offset prefetch (AWE_SOA_PF) and leaf-load lookahead
# (AWE_GEN_LOOKAHEAD) variants, timed with tools/soa_variants.py after the path parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gen_path_gpu.py -m gpu > gpurun_out/pytest_pf.log 2>&1 || { tail -40 gpurun_out/pytest_pf.log; exit 1; }
tail -2 gpurun_out/pytest_pf.log
timeout -k 10 600 python -u tools/soa_variants.py awebox_amd/libawegpu.so tools/ab/libawegpu_pf0.so tools/ab/libawegpu_pf16.so tools/ab/libawegpu_la16.so tools/ab/libawegpu_la32.so > gpurun_out/soa_pf.log 2>&1 || { cat gpurun_out/soa_pf.log; exit 1; }
cat gpurun_out/soa_pf.log
