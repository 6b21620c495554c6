"""Time the dense fp64 KKT factorisation paths available through torch on this GPU."""
import time

import torch

for N in (4000, 8000, 12600):
    A = torch.randn(N, N, dtype=torch.float64, device="cuda")
    A = A + A.T
    b = torch.randn(N, dtype=torch.float64, device="cuda")
    for name, fn in (("solve", lambda: torch.linalg.solve(A, b)),
                     ("lu_factor", lambda: torch.linalg.lu_factor(A)),
                     ("ldl_factor", lambda: torch.linalg.ldl_factor(A)),
                     ("cholesky(A^2)", None)):
        if fn is None:
            continue
        try:
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / 3
            print(f"N={N} {name}: {dt*1e3:.1f} ms  ({2/3*N**3/dt/1e12:.2f} TFLOP/s LU-equivalent)", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"N={N} {name}: unavailable ({type(e).__name__}: {str(e)[:80]})", flush=True)
