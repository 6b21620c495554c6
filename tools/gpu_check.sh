#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprof kernel trace.  Every GPU step has its
# own time limit; a crash / fault / timeout (exit code other than 0 or 1) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
run() {  # run <limit> <log> <cmd...>
    local limit=$1 log=$2; shift 2
    echo "=== $* (limit ${limit}s)" | tee -a $OUT/steps.log
    timeout -k 10 "$limit" "$@" > "$OUT/$log" 2>&1
    local rc=$?
    echo "=== rc=$rc" | tee -a $OUT/steps.log
    tail -3 "$OUT/$log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
    return 0
}
STAGES=${STAGES:-"test smoke bench prof"}
for s in $STAGES; do
  case $s in
    test)  run 900 pytest_gpu.log python -m pytest tests -m gpu -x -q ;;
    smoke) run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 600 bench.log python bench.py --steps ${BENCH_STEPS:-30} --warmup 5 ${BENCH_ARGS} ;;
    prof)  run 600 rocprof.log rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} && \
           find $OUT/prof -name '*_trace.csv' -size +4M -delete ;;
    pmc)   run 600 rocprof_pmc.log rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} && \
           run 600 rocprof_pmc2.log rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} ;;
    sq)    i=0; IFS=';' read -ra GROUPS_ARR <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY}"
           for grp in "${GROUPS_ARR[@]}"; do
             i=$((i+1))
             run 600 rocprof_sq$i.log rocprofv3 --pmc $grp -d $OUT/sq$i -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}
           done ;;
    listc) run 120 counters.log rocprofv3 -L ;;
  esac
done
echo ALL_DONE
