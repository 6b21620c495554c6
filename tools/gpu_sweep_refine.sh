#!/bin/bash
# AP2 8-point fan sweep with the fused separator path's refinement budget 3 (current) and 10
# (IPOPT's max_refinement_steps) before the dense fallback: iterations, powers, fallbacks, wall.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep_refine
export TMPDIR=/tmp
i=0
for r in 3 10 3 10; do
  i=$((i + 1))
  timeout -k 10 300 python -u tools/sweep_phase_probe.py --arch ap2 --refine $r --out gpurun_out/sweep_refine/run${i}_r$r.json > gpurun_out/sweep_refine/run${i}_r$r.log 2>&1 || exit $?
  tail -n 1 gpurun_out/sweep_refine/run${i}_r$r.log
done
