"""Summarise a final-step ensemble trace (tools/final_step_ensemble.py --trace): per iteration the
largest objective difference of the members from member 0 (and, where recorded, the largest
scaled V distance), member 0's inertia correction delta_w, step length and backtracks -- how a
1e-13 difference of the starting point grows along the iteration.

    python tools/divergence_summary.py TRACE.json OUT.json
"""
import json
import sys

import numpy as np


def main():
    d = json.load(open(sys.argv[1]))
    logs = d["logs"]
    n = min(len(l) for l in logs)
    rows = []
    for it in range(n):
        f0 = logs[0][it]["f"]
        df = max(abs(l[it]["f"] - f0) for l in logs[1:]) if len(logs) > 1 else 0.0
        r = {"it": it, "df": df, "mu": logs[0][it]["mu"], "delta_w": logs[0][it]["delta_w"],
             "alpha": logs[0][it]["alpha"], "backtracks": logs[0][it]["backtracks"], "soc": logs[0][it]["soc"]}
        if "dist" in d and it < len(d["dist"]):
            r["dV"] = max(d["dist"][it][1:]) if len(d["dist"][it]) > 1 else 0.0
        if "periods" in d and it < len(d["periods"]):
            r["T"] = d["periods"][it]
        rows.append(r)
    # growth rate of the difference between 1e-12 and 1e-3 (log10 per iteration, least squares)
    key = "dV" if rows and "dV" in rows[0] else "df"
    pts = [(r["it"], np.log10(r[key])) for r in rows if 1e-12 < r[key] < 1e-3]
    rate = float(np.polyfit([p[0] for p in pts], [p[1] for p in pts], 1)[0]) if len(pts) > 3 else None
    nz = [r for r in rows[:60]]
    summary = {"source": sys.argv[1], "members": len(logs), "iterations_compared": n, "growth_measure": key,
               "log10_growth_per_iteration": rate,
               "factor_per_iteration": 10 ** rate if rate is not None else None,
               "first_60": {"inertia_corrected": sum(r["delta_w"] > 0 for r in nz),
                            "alpha_below_1": sum(r["alpha"] < 1.0 for r in nz),
                            "backtracking": sum(r["backtracks"] > 0 for r in nz)},
               "final_periods_s": d.get("final_periods"), "rows": rows}
    json.dump(summary, open(sys.argv[2], "w"), indent=0, default=float)
    print(json.dumps({k: v for k, v in summary.items() if k != "rows"}, default=float))


if __name__ == "__main__":
    main()
