#!/bin/bash
# A/B of a solver setting in one GPU session: bench.py's solver blocks (AP2 sweep, config-4 shard in
# fan and chain mode, converged MPC) with AWE_EARLY_INERTIA_MAX_BLOCKS=0 (interval-block inertia
# after the factorisation), at its default (beside it on a side stream up to 512 blocks) and for
# every batch, then the first two again.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # run <tag> <env...>
    local tag=$1; shift
    timeout -k 10 400 env "$@" python -u bench.py --steps 5 --warmup 2 --batch 256 --no-cpu-baseline --no-hessian \
        --no-latency --mpc-batch 32 --dual-batch 0 > "gpurun_out/solver_ab_$tag.log" 2>&1 || exit $?
    python - "$tag" <<'PY'
import json, sys
tag = sys.argv[1]
for l in open(f"gpurun_out/solver_ab_{tag}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        s, ds, m = d.get("sweep") or {}, d.get("dual_sweep") or {}, (d.get("mpc") or {}).get("converged") or {}
        print(tag, "sweep", round(s.get("value", 0), 3), s.get("iterations"), "dual fan", round(ds.get("value", 0), 3),
              "chain", round((ds.get("chain") or {}).get("value", 0), 3), "mpc", round(m.get("ms_per_step", 0), 1),
              round(m.get("realtime_factor", 0), 3), flush=True)
PY
}
if [ -n "$AB_VAR" ]; then           # AB_VAR=NAME: NAME=0 against NAME=1, twice
    run off $AB_VAR=0 && run on $AB_VAR=1 && run off2 $AB_VAR=0 && run on2 $AB_VAR=1
    exit $?
fi
run base AWE_EARLY_INERTIA_MAX_BLOCKS=0
run side AWE_EARLY_INERTIA_MAX_BLOCKS=512
run all AWE_EARLY_INERTIA_MAX_BLOCKS=100000
run base2 AWE_EARLY_INERTIA_MAX_BLOCKS=0
run side2 AWE_EARLY_INERTIA_MAX_BLOCKS=512
