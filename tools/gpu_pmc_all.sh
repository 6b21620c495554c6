#!/bin/bash
# PMC passes (one counter group per run, kernel trace only) over the config-3/5 evaluators
# (tools/pmc_kernels.py) and the AP2 Hessian kernel (--hess): FETCH_SIZE, WRITE_SIZE, FP64 and
# wave-state counters for the Hessian; kernel-trace statistics of each program.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <dir> <args> -- counters...
    local d=$1 args=$2; shift 2
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "gpurun_out/$d" -o run --output-format csv -- python -u tools/pmc_kernels.py $args > "gpurun_out/$d.log" 2>&1 || exit $?
    echo "=== $d ok"
}
timeout -k 10 120 python -u tools/pmc_kernels.py > gpurun_out/pmc_cfg_plain.log 2>&1 || exit $?
run pmc_cfg_fetch "" FETCH_SIZE
run pmc_cfg_write "" WRITE_SIZE
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_cfg_trace -o run --output-format csv -- python -u tools/pmc_kernels.py > gpurun_out/pmc_cfg_trace.log 2>&1 || exit $?
run pmc_hess_fetch --hess FETCH_SIZE
run pmc_hess_write --hess WRITE_SIZE
run pmc_hess_f64 --hess SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES
run pmc_hess_wait --hess SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_hess_trace -o run --output-format csv -- python -u tools/pmc_kernels.py --hess > gpurun_out/pmc_hess_trace.log 2>&1 || exit $?
echo PMC_ALL_DONE
