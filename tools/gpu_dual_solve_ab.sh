#!/bin/bash
# dual-kite sweep (8 points, fan): block-recursion solves by the awelu kernel vs rocSOLVER getrs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dual_solve_ab
export TMPDIR=/tmp
O=gpurun_out/dual_solve_ab
timeout -k 10 400 python -u tools/sweep_phase_probe.py --arch dual --awelu-solve --out $O/awelu.json > $O/awelu.log 2>&1 || exit 1
tail -n 1 $O/awelu.log
timeout -k 10 400 python -u tools/sweep_phase_probe.py --arch dual --out $O/library.json > $O/library.log 2>&1 || exit 1
tail -n 1 $O/library.log
