#!/bin/bash
# PMC passes (one counter group per run, kernel trace only) over tools/pmc_kernels.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/pmc_kernels.py > gpurun_out/pmc_cfg_plain.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_cfg_fetch -o run --output-format csv -- python -u tools/pmc_kernels.py > gpurun_out/pmc_cfg_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_cfg_write -o run --output-format csv -- python -u tools/pmc_kernels.py > gpurun_out/pmc_cfg_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_cfg_trace -o run --output-format csv -- python -u tools/pmc_kernels.py > gpurun_out/pmc_cfg_trace.log 2>&1 || exit $?
echo PMC_DONE
