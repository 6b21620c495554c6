"""Micro-benchmark: symmetric eigenvalue counts (inertia) of the KKT blocks on the GPU."""
import time
import torch

dev = "cuda"
for shape in [(40, 268), (320, 268), (41, 46), (328, 46), (1, 1887)]:
    b, n = shape
    A = torch.randn(b, n, n, dtype=torch.float64, device=dev)
    A = A + A.transpose(1, 2)
    torch.linalg.eigvalsh(A)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        ev = torch.linalg.eigvalsh(A)
    torch.cuda.synchronize()
    print(f"eigvalsh {b} x {n}: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms", flush=True)
A = torch.randn(40, 268, 268, dtype=torch.float64, device=dev)
A = A + A.transpose(1, 2)
torch.linalg.lu_factor(A)
torch.cuda.synchronize()
t0 = time.perf_counter()
torch.linalg.lu_factor(A)
torch.cuda.synchronize()
print(f"lu_factor 40 x 268: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from awebox_amd.batched_lu import sym_inertia
for b, n in [(40, 268), (320, 268), (41, 46), (328, 46), (1, 1887)]:
    A = torch.randn(b, n, n, dtype=torch.float64, device=dev)
    A = A + A.transpose(1, 2)
    sym_inertia(A)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        c = sym_inertia(A)
    torch.cuda.synchronize()
    print(f"sym_inertia {b} x {n}: {(time.perf_counter() - t0) / 3 * 1e3:.2f} ms", flush=True)
