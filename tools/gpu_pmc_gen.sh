#!/bin/bash
# PMC passes over the generated evaluation path (ap2_node_kernel + ap2_assemble_kernel, B=2048,
# tools/pmc_kernels.py --ap2): FETCH_SIZE, WRITE_SIZE, FP64/VALU instruction counts, wave-state
# cycles, one counter group per run with the kernel trace only; then the kernel-trace statistics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <dir> <counters...>
    local d=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "gpurun_out/$d" -o run --output-format csv -- python -u tools/pmc_kernels.py --ap2 > "gpurun_out/$d.log" 2>&1 || exit $?
    echo "=== $d ok"
}
run pmc_gen_fetch FETCH_SIZE
run pmc_gen_write WRITE_SIZE
run pmc_gen_f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES
run pmc_gen_wait SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc_gen_trace -o run --output-format csv -- python -u tools/pmc_kernels.py --ap2 > gpurun_out/pmc_gen_trace.log 2>&1 || exit $?
echo PMC_GEN_DONE
