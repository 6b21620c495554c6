#!/bin/bash
# Fused interior-point measures: kernel-vs-torch bitwise tests, then the end-to-end A/B
# (converged MPC, AP2 default homotopy) with AWE_IPM_FUSED=0 / 1.
set -o pipefail
O=gpurun_out/fused
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ipm_measures_gpu.py \
    > $O/test.log 2>&1 || { tail -40 $O/test.log; exit 1; }
tail -3 $O/test.log
timeout -k 10 700 python -u tools/ipm_fused_ab.py --out $O/ab.json > $O/ab.log 2>&1 || { tail -40 $O/ab.log; exit 1; }
tail -5 $O/ab.log
