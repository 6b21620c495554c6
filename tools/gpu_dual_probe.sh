#!/bin/bash
# Config-4 shard (8 points, fan) with the separator through the large-block fused kernels and through
# the block recursion, progress printed as it runs.  A failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dual_probe
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/dual_sweep_probe.py --verbose 2>&1 | tee gpurun_out/dual_probe/fused.log | grep -v "^ *$" | cut -c1-200 || exit 1
timeout -k 10 400 python -u tools/dual_sweep_probe.py --verbose --max-m 48 2>&1 | tee gpurun_out/dual_probe/recursion.log | grep -v "^ *$" | cut -c1-200 || exit 1
