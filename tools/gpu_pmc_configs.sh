#!/bin/bash
# PMC passes over the config-3 (dual kites, B = 128) and config-5 (tracking MPC, B = 256) evaluator
# kernels of tools/pmc_kernels.py, one counter group per run with the kernel trace only: HBM bytes
# (FETCH_SIZE, WRITE_SIZE) and the FP64 / VALU / wave-state counters bench.py reads from
# profiles/pmc_traffic_configs.json (tools/pmc_summary.py --record-configs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <dir> <counters...>
    local d=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "gpurun_out/$d" -o run --output-format csv -- python -u tools/pmc_kernels.py > "gpurun_out/$d.log" 2>&1 || exit $?
    echo "=== $d ok"
}
rm -rf gpurun_out/pmc_cfg_fetch gpurun_out/pmc_cfg_write gpurun_out/pmc_cfg_sq
run pmc_cfg_fetch FETCH_SIZE
run pmc_cfg_write WRITE_SIZE
run pmc_cfg_sq SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES
echo PMC_CONFIGS_DONE
