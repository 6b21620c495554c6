#!/bin/bash
# Round 6 records on the final sources: the headline PMC passes (tools/gpu_pmc_soa.sh) and the
# kernel-trace statistics of the bench's dual-kite sweep block alone (tools/sweep_record.py input).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_pmc_soa.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dsweep -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --sweep-points 0 --no-hessian --no-dual-chain > gpurun_out/rocprof_dsweep.log 2>&1 || exit $?
find gpurun_out/prof_dsweep -name '*_trace.csv' -size +4M -delete
timeout -k 10 200 python -u tools/soa_chunks_ab.py --B 4096 --settings 1,1 > gpurun_out/b4096.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/soa_chunks_ab.py --B 1024 --settings 1,1 > gpurun_out/b1024.log 2>&1 || exit $?
echo R06_RECORDS_DONE
