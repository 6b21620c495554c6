#!/bin/bash
# PMC passes over the instance-minor evaluation path (ap2_soa_in / shoot / radau, the interval
# kernel, B=2048, tools/pmc_kernels.py --ap2): HBM bytes (FETCH_SIZE, WRITE_SIZE), instruction mix,
# wave-state cycles, one counter group per run with the kernel trace only; then the kernel-trace
# statistics of the same program.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <dir> <counters...>
    local d=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "gpurun_out/$d" -o run --output-format csv -- python -u tools/pmc_kernels.py --ap2 > "gpurun_out/$d.log" 2>&1 || exit $?
    echo "=== $d ok"
}
run pmc_soa_fetch FETCH_SIZE
run pmc_soa_write WRITE_SIZE
run pmc_soa_inst SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES
run pmc_soa_wait SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
run pmc_soa_lds SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_soa_trace -o run --output-format csv -- python -u tools/pmc_kernels.py --ap2 > gpurun_out/pmc_soa_trace.log 2>&1 || exit $?
echo PMC_SOA_DONE
