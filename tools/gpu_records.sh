#!/bin/bash
# Measurement records for the current sources, one GPU session, every step under its own limit,
# the first failure ends the script:
#   ap2    -- PMC passes over ap2_interval_kernel at B = 2048 (FETCH, WRITE, FP64 / VALU, wave states)
#   cfg    -- the same four groups over the dual-kite and MPC interval kernels (tools/pmc_kernels.py)
#   hess   -- the AP2 Hessian kernel's groups
#   sweep  -- kernel-trace statistics of the bench's AP2 sweep block and of its dual-kite sweep block
# Usage: STAGES="ap2 cfg hess sweep" tools/gpu_records.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
F64="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
WAIT="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD"
pmc() {  # pmc <dir> <driver args> <counters...>
    local d=$1 args=$2; shift 2
    timeout -s KILL 150 rocprofv3 --pmc "$@" -d "gpurun_out/$d" -o run --output-format csv -- python -u tools/pmc_kernels.py $args > "gpurun_out/$d.log" 2>&1 || { echo "=== $d failed"; exit 1; }
    echo "=== $d ok"
}
trace() {  # trace <dir> <limit> <program args...>
    local d=$1 limit=$2; shift 2
    timeout -s KILL "$limit" rocprofv3 --kernel-trace --stats -d "gpurun_out/$d" -o run --output-format csv -- "$@" > "gpurun_out/$d.log" 2>&1 || { echo "=== $d failed"; exit 1; }
    find "gpurun_out/$d" -name '*_trace.csv' -size +4M -delete
    echo "=== $d ok"
}
STAGES=${STAGES:-"ap2 cfg hess sweep"}
for s in $STAGES; do
  case $s in
    ap2)
      timeout -k 10 150 python -u tools/pmc_kernels.py --ap2 > gpurun_out/pmc_ap2_plain.log 2>&1 || exit 1
      pmc pmc_ap2_fetch --ap2 FETCH_SIZE
      pmc pmc_ap2_write --ap2 WRITE_SIZE
      pmc pmc_ap2_f64 --ap2 $F64
      pmc pmc_ap2_wait --ap2 $WAIT
      trace pmc_ap2_trace 150 python -u tools/pmc_kernels.py --ap2 ;;
    cfg)
      pmc pmc_cfg_fetch "" FETCH_SIZE
      pmc pmc_cfg_write "" WRITE_SIZE
      pmc pmc_cfg_f64 "" $F64
      pmc pmc_cfg_wait "" $WAIT
      trace pmc_cfg_trace 150 python -u tools/pmc_kernels.py ;;
    hess)
      pmc pmc_hess_fetch --hess FETCH_SIZE
      pmc pmc_hess_write --hess WRITE_SIZE
      pmc pmc_hess_f64 --hess $F64
      pmc pmc_hess_wait --hess $WAIT
      trace pmc_hess_trace 150 python -u tools/pmc_kernels.py --hess ;;
    sweep)
      trace sweep_ap2_prof 300 python -u bench.py --steps 1 --warmup 1 --batch 8 --no-cpu-baseline --no-hessian --no-latency --mpc-batch 0 --dual-batch 0 --dual-sweep-points 0 --sweep-points 8
      trace sweep_dual_prof 400 python -u bench.py --steps 1 --warmup 1 --batch 8 --no-cpu-baseline --no-hessian --no-latency --mpc-batch 0 --dual-batch 0 --sweep-points 0 --dual-sweep-points 8 --no-dual-chain ;;
  esac
done
echo RECORDS_DONE
