"""Phase timing of btd_factor_kernel from an instrumented build (tools/exp_src/btd_timing.hip ->
tools/ab/libawelu_btdtiming.so, wall_clock64 at the stage phases of block 0): load, D -= L W,
Gauss-Jordan, write-out, in microseconds per stage (the wall clock runs at 100 MHz)."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ab", "libawelu_btdtiming.so"))
lib.awelu_btd_factor_batched.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
dev = "cuda"
for b, nb, m in [(8, 41, 46), (64, 21, 22)]:
    T = torch.randn(b, nb, 3, m, m, dtype=torch.float64, device=dev)
    T[:, :, 1] += 4 * m * torch.eye(m, dtype=torch.float64, device=dev)
    Dinv = torch.empty(b, nb, m, m, dtype=torch.float64, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = (ctypes.c_ulonglong * 10)()
    for rep in range(3):
        F = T.clone()
        lib.awelu_btd_factor_batched(nb, m, b, ctypes.c_void_p(F.data_ptr()), ctypes.c_void_p(Dinv.data_ptr()), st)
        torch.cuda.synchronize()
    lib.awelu_btd_timing(out)
    us = [v / 100.0 / nb for v in out[:4]]      # 100 MHz ticks -> us per stage
    mhz = out[8] / out[9] * 100.0 if out[9] else 0.0
    cyc = {k: round(v / (nb * m), 1) for k, v in zip(["publish_col+barrier", "pivot_search", "publish_row+barrier", "update"], out[4:8])}
    print(json.dumps({"batch": b, "nb": nb, "m": m, "us_per_stage": dict(zip(["load", "product", "gauss_jordan", "write"], [round(u, 2) for u in us])),
                      "us_per_gj_column": round(us[2] / m, 3), "shader_clock_mhz": round(mhz, 1),
                      "cycles_per_gj_column": cyc}), flush=True)
