#!/bin/bash
# lu_batched variants against the round-5 baseline (abv/libawelu_r05base.so): product source, V1 (the
# one-column-per-thread loop kept when no row split applies), V2 (butterfly pivot search)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lu_var
export TMPDIR=/tmp
for v in prod v1 v2; do
  lib=awebox_amd/libawelu.so; [ $v != prod ] && lib=abv/libawelu_$v.so
  timeout -k 10 200 python -u tools/awelu_ab.py --base abv/libawelu_r05base.so --new $lib --reps 10 --lu-only > gpurun_out/lu_var/$v.log 2>&1 || exit 1
  echo "== $v"; grep '"op"' gpurun_out/lu_var/$v.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['batch'],d['n'],d['new_factor_ms'],d['base_factor_ms'],d['factors_bitwise_equal'])"
done
