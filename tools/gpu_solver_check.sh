cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
bash tools/gpu_dual_ab.sh || exit 1
git_rev=none
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-hessian --no-latency --dual-batch 0 --dual-sweep-points 0 --steps 3 --warmup 1 --batch 64 > gpurun_out/bench_solver.log 2>&1 || { tail -20 gpurun_out/bench_solver.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_solver.log") if l.startswith("{")][-1])
print("sweep", d["sweep"]["value"], d["sweep"]["wall_s"], "mpc", json.dumps({k: d["mpc"]["converged"][k] for k in ("ms_per_step", "realtime_factor", "ipm_iterations_max")}))
PY
