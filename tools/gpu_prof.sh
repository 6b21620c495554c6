set -o pipefail
cd "$GRAFT_REPO_ROOT"
STAGES="prof" BENCH_ARGS="--sweep-points 0" bash tools/gpu_check.sh && \
STAGES="pmc" BENCH_ARGS="--sweep-points 0 --mpc-batch 0 --no-hessian" bash tools/gpu_check.sh
