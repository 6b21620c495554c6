#!/bin/bash
# Dual-kite evaluator A/B: GPU parity tests of the product library, then the bench's config-3 block
# (B = 128, N = 60) with the product library and with tools/ab/libawedual_old.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DUAL="--no-cpu-baseline --no-hessian --no-latency --mpc-batch 0 --pmpc-loops 0 --dual-sweep-points 0 --sweep-points 0 --steps 3 --warmup 1 --batch 64"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dual_gpu.py tests/test_dual_hess_gpu.py -m gpu > gpurun_out/pytest_dual.log 2>&1 || { tail -30 gpurun_out/pytest_dual.log; exit 1; }
tail -2 gpurun_out/pytest_dual.log
for lib in new old; do
  if [ $lib = old ]; then cp tools/ab/libawedual_old.so awebox_amd/libawedual.so; fi
  timeout -k 10 300 python -u bench.py $DUAL > gpurun_out/bench_dual_$lib.log 2>&1 || { tail -20 gpurun_out/bench_dual_$lib.log; exit 1; }
  python - "$lib" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/bench_dual_{sys.argv[1]}.log") if l.startswith("{")][-1])["dual"]
print(sys.argv[1], json.dumps({k: d[k] for k in ("value", "ms_per_step")}), json.dumps(d.get("roofline", {}))[:300])
PY
done
cp awebox_amd/libawedual.so tools/ab/libawedual_old_restored.so 2>/dev/null
