#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/lazy_probe.py --B 128 --runs 4 > gpurun_out/lazy.log 2>&1
rc=$?; echo "=== lazy rc=$rc"; grep run gpurun_out/lazy.log | cut -c1-1200; tail -3 gpurun_out/lazy.log | cut -c1-800
