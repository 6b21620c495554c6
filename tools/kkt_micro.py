"""Micro-benchmark of the structured-KKT building blocks on the GPU (batched LU sizes of the AP2 and
dual-kite problems)."""
import json
import time

import torch


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


out = {}
dev = "cuda"
for name, (nb, n, L) in {"ap2_n40": (40, 268, 120), "dual_n20": (20, 640, 160), "dual_n60": (60, 640, 160)}.items():
    A = torch.randn(nb, n, n, dtype=torch.float64, device=dev) + n * torch.eye(n, dtype=torch.float64, device=dev)
    B = torch.randn(nb, n, L, dtype=torch.float64, device=dev)
    LU, piv = torch.linalg.lu_factor(A)
    out[name + "_lu_factor_ms"] = t(lambda: torch.linalg.lu_factor(A))
    out[name + "_lu_factor_ex_ms"] = t(lambda: torch.linalg.lu_factor_ex(A))
    out[name + "_lu_solve_ms"] = t(lambda: torch.linalg.lu_solve(LU, piv, B))
    out[name + "_inv_ms"] = t(lambda: torch.linalg.inv(A))
    out[name + "_bmm_ms"] = t(lambda: B.transpose(1, 2) @ B)
for nS in (2100, 6300):
    S = torch.randn(nS, nS, dtype=torch.float64, device=dev) + nS * torch.eye(nS, dtype=torch.float64, device=dev)
    out[f"dense_lu_{nS}_ms"] = t(lambda: torch.linalg.lu_factor(S))
idx = torch.randint(0, 20 * 640 * 640, (3_600_000,), device=dev)
v = torch.randn(3_600_000, dtype=torch.float64, device=dev)
Z = torch.zeros(20 * 640 * 640, dtype=torch.float64, device=dev)
out["index_put_acc_3.6M_ms"] = t(lambda: Z.index_put_((idx,), v, accumulate=True))
out["index_put_3.6M_ms"] = t(lambda: Z.index_put_((idx,), v))
print(json.dumps(out, indent=1))
