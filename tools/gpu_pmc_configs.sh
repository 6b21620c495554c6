#!/bin/bash
# PMC passes over the config-3 (dual kites, B = 128) and config-5 (tracking MPC, B = 256) evaluator
# kernels of tools/pmc_kernels.py, one counter group per run with the kernel trace only: HBM bytes
# (FETCH_SIZE, WRITE_SIZE) and the FP64 / VALU / wave-state counters bench.py reads from
# profiles/pmc_traffic_configs.json (tools/pmc_summary.py --record-configs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <dir> <driver flag> <counters...>
    local d=$1 f=$2; shift 2
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "gpurun_out/$d" -o run --output-format csv -- python -u tools/pmc_kernels.py $f > "gpurun_out/$d.log" 2>&1 || exit $?
    echo "=== $d ok"
}
for w in dual mpc; do
    rm -rf gpurun_out/pmc_cfg_${w}_fetch gpurun_out/pmc_cfg_${w}_write gpurun_out/pmc_cfg_${w}_sq
    run pmc_cfg_${w}_fetch --$w FETCH_SIZE
    run pmc_cfg_${w}_write --$w WRITE_SIZE
    run pmc_cfg_${w}_sq --$w SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES
done
python tools/pmc_summary.py --record-configs 'gpurun_out/pmc_cfg_{which}_fetch' 'gpurun_out/pmc_cfg_{which}_write' 'gpurun_out/pmc_cfg_{which}_sq'
cp profiles/pmc_traffic_configs.json gpurun_out/pmc_traffic_configs.json
echo PMC_CONFIGS_DONE
