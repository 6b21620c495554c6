#!/bin/bash
# Host profiles (cProfile) of the converged MPC and the AP2 / dual fan sweep shards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
O=gpurun_out/hostprof
mkdir -p $O
timeout -k 10 300 python -u tools/pmpc_profile.py --out $O/pmpc_profile.json > $O/pmpc.log 2>&1 || { tail -30 $O/pmpc.log; exit 1; }
timeout -k 10 300 python -u tools/sweep_cprofile.py --arch ap2 --out $O/sweep_ap2.txt > $O/sweep_ap2.log 2>&1 || { tail -30 $O/sweep_ap2.log; exit 1; }
timeout -k 10 400 python -u tools/sweep_cprofile.py --arch dual --out $O/sweep_dual.txt > $O/sweep_dual.log 2>&1 || { tail -30 $O/sweep_dual.log; exit 1; }
head -3 $O/sweep_ap2.txt $O/sweep_dual.txt
