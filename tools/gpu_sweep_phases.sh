#!/bin/bash
# Sweep block phase records (tools/sweep_phase_probe.py): AP2 8 points unsynchronised and with
# phase timings, the dual-kite 8 points unsynchronised.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep_phases
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/sweep_phase_probe.py --arch ap2 --out gpurun_out/sweep_phases/ap2.json > gpurun_out/sweep_phases/ap2.log 2>&1 &&
timeout -k 10 300 python -u tools/sweep_phase_probe.py --arch ap2 --profile --out gpurun_out/sweep_phases/ap2_prof.json > gpurun_out/sweep_phases/ap2_prof.log 2>&1 &&
timeout -k 10 400 python -u tools/sweep_phase_probe.py --arch dual --out gpurun_out/sweep_phases/dual.json > gpurun_out/sweep_phases/dual.log 2>&1
rc=$?
tail -1 gpurun_out/sweep_phases/*.log
exit $rc
