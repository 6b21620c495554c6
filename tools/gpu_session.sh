#!/bin/bash
# Round-2 kernel session: AP2 seed-variant timings (tools/ap2_variants.py), PMC traffic of the
# config-3/5 kernels, and the config-5 / config-4 GPU tests.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ap2_variants.py tools/exp_build/libawegpu_base.so tools/exp_build/libawegpu_seedcvt.so tools/exp_build/libawegpu_seedA.so tools/exp_build/libawegpu_seedB.so > gpurun_out/ap2_variants.log 2>&1 || exit $?
echo variants-ok
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_mpc_fetch -o run --output-format csv -- python -u tools/pmc_kernels.py > gpurun_out/pmc_mpc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_mpc_write -o run --output-format csv -- python -u tools/pmc_kernels.py > gpurun_out/pmc_mpc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_mpc_trace -o run --output-format csv -- python -u tools/pmc_kernels.py > gpurun_out/pmc_mpc_trace.log 2>&1 || exit $?
echo pmc-ok
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_mpc.py tests/test_mpc_solve.py tests/test_rti.py tests/test_config4.py -m gpu > gpurun_out/pytest_sel.log 2>&1 || exit $?
echo tests-ok
