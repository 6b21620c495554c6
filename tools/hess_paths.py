"""Time nlp_hess_l on both Hessian kernels (hyper-dual colour pairs, generated forward-over-reverse)
at the bench's B = 2048 (instance-minor H for the generated path) and at B = 1 (the drop-in
Callback's per-iteration call, host round trip), with a cross-check of the two paths' values.

usage: python tools/hess_paths.py [B]
"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from awebox_amd import evaluator as E, problem as pb  # noqa: E402
from awebox_amd.initial_guess import batch_member, initial_guess  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
consts = pb.build_constants()
lay = pb.NlpLayout(40, 4)
v0 = initial_guess(consts, lay)
V = torch.tensor(np.stack([batch_member(v0, lay, b) for b in range(B)]), device="cuda")
P = torch.tensor(np.stack([pb.pack_p(lay, consts, v0, u_ref=5.0 + 3.0 * b / B) for b in range(B)]), device="cuda")
sig = torch.ones(B, dtype=torch.float64, device="cuda")
lam = torch.tensor(np.random.default_rng(7).standard_normal((B, lay.n_g)), device="cuda")
ev = E.Ap2Evaluator(consts, batch=B)
out = {"batch": B}
res = {}
for path, steps in (("generated", 20), ("hyperdual", 3)):
    ev.hess_path = path
    H = ev.alloc_hess() if path == "generated" else torch.zeros(B, ev.nnz_h, dtype=torch.float64, device="cuda")
    call = (lambda: ev.eval_hess_device_im(V, P, sig, lam, H)) if path == "generated" else \
        (lambda: ev.eval_hess_device(V, P, sig, lam, H))
    call()
    torch.cuda.synchronize()
    kms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        call()
        kms.append(ev.last_hess_ms())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    res[path] = H.contiguous().cpu().numpy() if path == "hyperdual" else H.cpu().numpy()
    out[path] = {"kernel_ms": float(np.median(kms)), "wall_ms": dt * 1e3, "evals_per_s": B / dt,
                 "finite": bool(np.isfinite(res[path]).all())}
d = np.abs(res["generated"] - res["hyperdual"])
scale = np.abs(res["hyperdual"]).max(axis=1, keepdims=True)
out["max_rel_diff"] = float((d / np.maximum(np.abs(res["hyperdual"]), 1e-300 + 1e-11 * scale)).max())
out["max_diff_over_rowmax"] = float((d / scale).max())
# B = 1 host round trip (the drop-in Callback's nlp_hess_l)
ev1 = E.Ap2Evaluator(consts, batch=1)
lam1 = np.random.default_rng(7).standard_normal(lay.n_g)
for path in ("generated", "hyperdual"):
    ev1.hess_path = path
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        ev1.eval_hess(v0.reshape(1, -1), pb.pack_p(lay, consts, v0).reshape(1, -1), 1.0, lam1.reshape(1, -1))
        ts.append(time.perf_counter() - t0)
    out[f"b1_host_ms_{path}"] = float(np.median(ts[5:]) * 1e3)
print(json.dumps(out))
