#!/bin/bash
# Dense vs block-tridiagonal separator solve in the AP2 sweep (same points), with a rocprof
# kernel trace of the btd run.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in dense btd; do
  timeout -k 10 300 python -u -m awebox_amd.sweep --points 4 --separators $s --verbose \
      --out gpurun_out/sweep_ap2_4pts_$s.json > gpurun_out/sweep_sep_$s.log 2>&1 || exit $?
  tail -1 gpurun_out/sweep_sep_$s.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sep -o run --output-format csv -- \
    python -u tools/ipm_profile.py --n-k 40 --iters 20 --separators btd > gpurun_out/prof_sep.log 2>&1 || exit $?
find gpurun_out/prof_sep -name '*_trace.csv' -size +4M -delete
