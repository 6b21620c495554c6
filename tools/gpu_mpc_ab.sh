#!/bin/bash
# MPC generated path A/B: the product library's parity tests, then tools/mpc_im_variants.py over the
# product library and the variant libraries given as arguments.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mpc_ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mpc.py -m gpu -k generated > gpurun_out/mpc_ab/pytest.log 2>&1 || { tail -30 gpurun_out/mpc_ab/pytest.log; exit 1; }
tail -3 gpurun_out/mpc_ab/pytest.log
timeout -k 10 500 python -u tools/mpc_im_variants.py awebox_amd/libawempc.so "$@" > gpurun_out/mpc_ab/variants.log 2>&1 || { cat gpurun_out/mpc_ab/variants.log; exit 1; }
cat gpurun_out/mpc_ab/variants.log
