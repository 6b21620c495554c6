"""Micro-benchmark of the block-tridiagonal kernels (awelu_btd_factor_batched / _solve_batched)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from awebox_amd.batched_lu import btd_factor, btd_solve  # noqa: E402

dev = "cuda"
for b, nb, m, nrhs in [(8, 41, 46, 1), (1, 41, 46, 1), (8, 1, 46, 1), (8, 41, 46, 7), (8, 41, 22, 1), (256, 21, 22, 1)]:
    T = torch.randn(b, nb, 3, m, m, dtype=torch.float64, device=dev)
    T[:, :, 1] += 4 * m * torch.eye(m, dtype=torch.float64, device=dev)
    X = torch.randn(b, nb, m, nrhs, dtype=torch.float64, device=dev)
    F, Dinv = btd_factor(T)
    btd_solve(F, Dinv, X)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        F, Dinv = btd_factor(T)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(5):
        btd_solve(F, Dinv, X)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B={b} nb={nb} m={m} nrhs={nrhs}: factor {(t1 - t0) / 5 * 1e3:.3f} ms, solve {(t2 - t1) / 5 * 1e3:.3f} ms", flush=True)
