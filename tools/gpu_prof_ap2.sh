#!/bin/bash
# rocprof kernel-trace stats of the bench's AP2 block alone (no sweep, no batch-1 latency launches)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ap2b -o run --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --sweep-points 0 --dual-sweep-points 0 --no-hessian --no-latency > gpurun_out/rocprof_ap2b.log 2>&1 || exit $?
find gpurun_out/prof_ap2b -name '*_trace.csv' -size +4M -delete
echo PROF_DONE
# the config-4 dual sweep block alone (8 points, fan mode) under the kernel tracer
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dualsweep -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --sweep-points 0 --no-hessian --no-latency > gpurun_out/rocprof_dualsweep.log 2>&1 || exit $?
find gpurun_out/prof_dualsweep -name '*_trace.csv' -size +4M -delete
echo DUAL_PROF_DONE
