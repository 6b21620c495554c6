#!/bin/bash
# Dual-kite checks and the config-4 shard's device profile: the generated-path parity tests, the
# instance-minor AP2 layout tests, the evaluator path timing, then the bench's dual sweep block alone
# under the kernel tracer.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dual_sweep
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dual_gpu.py tests/test_gen_path_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/dual_sweep/pytest.log 2>&1 || { tail -40 gpurun_out/dual_sweep/pytest.log; exit 1; }
tail -3 gpurun_out/dual_sweep/pytest.log
timeout -k 10 300 python -u tools/dual_paths.py > gpurun_out/dual_sweep/paths.log 2>&1 || { cat gpurun_out/dual_sweep/paths.log; exit 1; }
cat gpurun_out/dual_sweep/paths.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/dual_sweep/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --batch 64 --dual-batch 0 --mpc-batch 0 --pmpc-loops 0 --sweep-points 0 --no-hessian --no-latency --no-dual-chain > gpurun_out/dual_sweep/rocprof.log 2>&1 || { tail -20 gpurun_out/dual_sweep/rocprof.log; exit 1; }
find gpurun_out/dual_sweep/prof -name '*_trace.csv' -size +4M -delete
tail -1 gpurun_out/dual_sweep/rocprof.log | cut -c1-400
echo DONE
