#!/bin/bash
# KKT kernel change check: awelu A/B (bitwise identity + times) against the round-5 baseline, the
# GPU tests of the KKT kernels and solvers, then the AP2 and dual-kite sweep probes (iterations,
# powers, wall time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/kkt_check
export TMPDIR=/tmp
O=gpurun_out/kkt_check
timeout -k 10 300 python -u tools/awelu_ab.py --base abv/libawelu_r05base.so --reps 10 > $O/ab.log 2>&1 || exit 1
grep -c '"factors_bitwise_equal": false\|"solution_bitwise_equal": false' $O/ab.log && { echo "NOT BITWISE"; }
timeout -k 10 600 python -u -m pytest tests/test_batched_lu.py tests/test_inertia.py tests/test_solver.py tests/test_mpc_solve.py tests/test_regression.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/sweep_phase_probe.py --arch ap2 --out $O/ap2.json > $O/ap2.log 2>&1 || exit 1
tail -n 1 $O/ap2.log
timeout -k 10 400 python -u tools/sweep_phase_probe.py --arch dual --out $O/dual.json > $O/dual.log 2>&1 || exit 1
tail -n 1 $O/dual.log
