#!/bin/bash
# PMC passes over ap2_hess_kernel<4> (tools/pmc_kernels.py --hess), one counter group per run with the
# kernel trace only, for profiles/pmc_hess.json (tools/pmc_summary.py --record-hess).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <dir> <counters...>
    local d=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "gpurun_out/$d" -o run --output-format csv -- python -u tools/pmc_kernels.py --hess > "gpurun_out/$d.log" 2>&1 || exit $?
    echo "=== $d ok"
}
rm -rf gpurun_out/pmc_hess_*
run pmc_hess_fetch FETCH_SIZE
run pmc_hess_write WRITE_SIZE
run pmc_hess_f64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES
run pmc_hess_wait SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD
echo PMC_HESS_DONE
