#!/bin/bash
# Dual-kite (config 3) GPU session: parity tests, then a short bench with only the dual block.
# Every GPU step has its own time limit; exit codes other than 0/1 end the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local limit=$1 log=$2; shift 2
    echo "=== $* (limit ${limit}s)" | tee -a gpurun_out/steps.log
    timeout -k 10 "$limit" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "=== rc=$rc" | tee -a gpurun_out/steps.log
    tail -5 "gpurun_out/$log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
    return 0
}
STAGES=${STAGES:-"test bench"}
for s in $STAGES; do
  case $s in
    test)  run 600 dual_tests.log python -u -m pytest tests/test_dual_gpu.py -x -v --timeout 300 --timeout-method thread ;;
    bench) run 300 dual_bench.log python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-hessian --mpc-batch 0 --sweep-points 0 ${BENCH_ARGS} ;;
    prof)  run 300 dual_rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/dprof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-hessian --mpc-batch 0 --sweep-points 0 ${BENCH_ARGS} && \
           find gpurun_out/dprof -name '*_trace.csv' -size +4M -delete ;;
  esac
done
echo ALL_DONE
