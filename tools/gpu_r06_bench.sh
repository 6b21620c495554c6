#!/bin/bash
# The default bench on the current sources (one run), and the host profiles of the sweep shards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
O=gpurun_out/bench6
mkdir -p $O
timeout -k 10 700 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c "
import json,sys
d=json.loads(sys.stdin.readline())
print('value', d['value'], 'frac', d['roofline']['frac'])
for k in ('sweep','dual_sweep','mpc'):
    v=d.get(k)
    if isinstance(v,dict): print(k, {kk: v.get(kk) for kk in ('value','wall_s','iterations','period_s','avg_power_W')})
c=d.get('mpc',{}).get('converged') if isinstance(d.get('mpc'),dict) else None
if c: print('pmpc', c.get('ms_per_step'), c.get('realtime_factor'), c.get('ipm_iterations_max'))
"
