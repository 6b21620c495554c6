"""Config 4 point by point: the sharded runs (8 shards of 8 points, fan and per-shard chain,
profiles/r04/config4/) against the reference-order global chain over all 64 points
(profiles/r05/config4/config4_global_chain.jsonl).  Per point: powers, periods, orbit family (interior
orbit or pinned at the example's t_f bound of 20 s) and the relative power difference; summary: the
points within 0.1 %, the points whose family differs, the largest difference, monotonicity.

    python tools/config4_compare.py > profiles/r05/config4/compare.json
"""
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def shards(path):
    pts = {}
    for line in open(path):
        r = json.loads(line)
        if r.get("summary") or "shard" not in r:
            continue
        for u, p, t, ok in zip(r["u_ref"], r["avg_power_W"], r["period_s"], r["ok"]):
            pts[round(u, 5)] = (p, t, ok, r["shard"])
    return pts


def main():
    g = [json.loads(l) for l in open(os.path.join(ROOT, "profiles", "r05", "config4", "config4_global_chain.jsonl"))][-1]
    fan = shards(os.path.join(ROOT, "profiles", "r04", "config4", "config4_full.jsonl"))
    chain = shards(os.path.join(ROOT, "profiles", "r04", "config4", "config4_chain.jsonl"))
    fam = lambda t: "tf_bound" if t >= 19.99 else "interior"  # noqa: E731
    rows, summ = [], {}
    for i, (u, p, t) in enumerate(zip(g["u_ref"], g["avg_power_W"], g["period_s"])):
        key = round(u, 5)
        row = {"i": i, "u_ref": u, "global": {"P": p, "T": t, "family": fam(t)}}
        for name, d in (("fan", fan), ("shard_chain", chain)):
            if key in d:
                ps, ts, ok, sh = d[key]
                row[name] = {"P": ps, "T": ts, "family": fam(ts), "shard": sh, "ok": ok,
                             "dP_rel": (ps - p) / p, "same_family": fam(ts) == fam(t)}
        rows.append(row)
    for name in ("fan", "shard_chain"):
        d = [r[name] for r in rows if name in r]
        summ[name] = {"points": len(d),
                      "within_0.1pct": sum(abs(x["dP_rel"]) <= 1e-3 for x in d),
                      "family_differs": [r["i"] for r in rows if name in r and not r[name]["same_family"]],
                      "max_abs_dP_rel": max(abs(x["dP_rel"]) for x in d),
                      "worst_point": max(rows, key=lambda r: abs(r.get(name, {}).get("dP_rel", 0.0)))["i"]}
    p = np.array(g["avg_power_W"])
    summ["global_chain"] = {"all_converged": g["all_converged"], "power_monotone": g["power_monotone"],
                            "min_step_W": float(np.diff(p).min()),
                            "dips": [int(i + 1) for i in np.where(np.diff(p) < 0)[0]],
                            "first_tf_bound_point": next(i for i, t in enumerate(g["period_s"]) if t >= 19.99),
                            "wall_s": g["wall_s"], "trials_per_s": g["trials_per_s"]}
    print(json.dumps({"summary": summ, "points": rows}, indent=1))


if __name__ == "__main__":
    main()
