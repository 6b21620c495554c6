"""A/B micro-benchmark of libawelu against a baseline build (--base, e.g. tools/ab/libawelu_r03base.so,
the round-3 sources before the blocked inertia and the batched loads):
  * lu_batched / lu_solve on the interval-block shapes (AP2 268, dual kites 640, the dual separator
    blocks 100): times, and whether factors and solutions are bitwise identical to the baseline;
  * btd_factor / btd_solve on the separator chains (AP2: 41 stages of 46, MPC: 21 of 22): times
    and bitwise identity with the baseline;
  * sym_inertia on the KKT block shapes (268, 640, separator pivot blocks 46, a dense separator
    1887): times, counts against the baseline and against eigenvalue counts.
Prints one JSON line per shape."""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def kkt_batch(b, n, dev, gen):
    """Symmetric indefinite KKT-like blocks [[H, J^T], [J, -1e-9 I]] (70 % of J zero), symmetrically
    permuted: the pivot search meets 1 x 1 and 2 x 2 pivots and interchanges."""
    nc = n // 3
    nx = n - nc
    H = torch.randn(b, nx, nx, dtype=torch.float64, device=dev, generator=gen)
    H = H + H.transpose(1, 2) + torch.diag_embed(3 * torch.rand(b, nx, dtype=torch.float64, device=dev, generator=gen))
    J = torch.randn(b, nc, nx, dtype=torch.float64, device=dev, generator=gen)
    J = J * (torch.rand(b, nc, nx, device=dev, generator=gen) > 0.7)
    K = torch.zeros(b, n, n, dtype=torch.float64, device=dev)
    K[:, :nx, :nx] = H
    K[:, nx:, :nx] = J
    K[:, :nx, nx:] = J.transpose(1, 2)
    K[:, nx:, nx:] = -1e-9 * torch.eye(nc, dtype=torch.float64, device=dev)
    p = torch.randperm(n, device=dev, generator=gen)
    return K[:, p][:, :, p].contiguous()


def run(lib, A, ztol=1e-13):
    W = A.clone()
    c = torch.empty(A.shape[0], 3, dtype=torch.int32, device=A.device)
    rc = lib.awelu_sym_inertia_batched(A.shape[1], A.shape[0], ctypes.c_void_p(W.data_ptr()), ctypes.c_double(ztol),
                                       ctypes.c_void_p(c.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, lib.awelu_last_error()
    return c


def timed(lib, A, reps):
    run(lib, A)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        c = run(lib, A)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3, c


def lu_ab(libs, b, n, nrhs, dev, gen, reps):
    A = torch.randn(b, n, n, dtype=torch.float64, device=dev, generator=gen) + n ** 0.5 * torch.eye(n, dtype=torch.float64, device=dev)
    X0 = torch.randn(b, n, nrhs, dtype=torch.float64, device=dev, generator=gen)
    rec = {"op": "lu", "batch": b, "n": n, "nrhs": nrhs}
    res = {}
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, lib in libs.items():
        LU = A.clone()
        piv = torch.empty(b, n, dtype=torch.int32, device=dev)
        X = X0.clone()
        f = lambda: lib.awelu_factor_batched(n, b, ctypes.c_void_p(LU.data_ptr()), ctypes.c_void_p(piv.data_ptr()), st)
        g = lambda: lib.awelu_solve_batched(n, nrhs, b, ctypes.c_void_p(LU.data_ptr()), ctypes.c_void_p(piv.data_ptr()),
                                            ctypes.c_void_p(X.data_ptr()), st)
        LU.copy_(A); f(); X.copy_(X0); g()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            LU.copy_(A)
            f()
        torch.cuda.synchronize()
        tf = (time.perf_counter() - t0) / reps * 1e3
        t0 = time.perf_counter()
        for _ in range(reps):
            X.copy_(X0)
            g()
        torch.cuda.synchronize()
        ts = (time.perf_counter() - t0) / reps * 1e3
        rec[name + "_factor_ms"] = round(tf, 4)
        rec[name + "_solve_ms"] = round(ts, 4)
        res[name] = (LU.clone(), piv.clone(), X.clone())
    r = torch.linalg.norm(A @ res["new"][2] - X0) / torch.linalg.norm(X0)
    rec["new_rel_residual"] = float(r)
    if "base" in res:
        rec["factors_bitwise_equal"] = bool(torch.equal(res["new"][0], res["base"][0]) and torch.equal(res["new"][1], res["base"][1]))
        rec["solution_bitwise_equal"] = bool(torch.equal(res["new"][2], res["base"][2]))
    return rec


def btd_ab(libs, b, nb, m, nrhs, dev, gen, reps, boost=4.0):
    """boost: multiple of m added to the diagonal blocks' diagonal (0: random pivot rows)."""
    T = torch.randn(b, nb, 3, m, m, dtype=torch.float64, device=dev, generator=gen)
    T[:, :, 1] += boost * m * torch.eye(m, dtype=torch.float64, device=dev)
    X0 = torch.randn(b, nb, m, nrhs, dtype=torch.float64, device=dev, generator=gen)
    rec = {"op": "btd", "batch": b, "nb": nb, "m": m, "nrhs": nrhs, "boost": boost}
    res = {}
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, lib in libs.items():
        F = T.clone()
        Dinv = torch.empty(b, nb, m, m, dtype=torch.float64, device=dev)
        X = X0.clone()
        f = lambda: lib.awelu_btd_factor_batched(nb, m, b, ctypes.c_void_p(F.data_ptr()), ctypes.c_void_p(Dinv.data_ptr()), st)
        g = lambda: lib.awelu_btd_solve_batched(nb, m, nrhs, b, ctypes.c_void_p(F.data_ptr()), ctypes.c_void_p(Dinv.data_ptr()),
                                                ctypes.c_void_p(X.data_ptr()), st)
        F.copy_(T); f(); X.copy_(X0); g()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            F.copy_(T)
            f()
        torch.cuda.synchronize()
        tf = (time.perf_counter() - t0) / reps * 1e3
        t0 = time.perf_counter()
        for _ in range(reps):
            X.copy_(X0)
            g()
        torch.cuda.synchronize()
        ts = (time.perf_counter() - t0) / reps * 1e3
        rec[name + "_factor_ms"] = round(tf, 4)
        rec[name + "_solve_ms"] = round(ts, 4)
        res[name] = (F.clone(), Dinv.clone(), X.clone())
    if "base" in res:
        rec["factors_bitwise_equal"] = bool(torch.equal(res["new"][0], res["base"][0]) and torch.equal(res["new"][1], res["base"][1]))
        rec["solution_bitwise_equal"] = bool(torch.equal(res["new"][2], res["base"][2]))
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", default=os.path.join(ROOT, "tools", "ab", "libawelu_r03base.so"))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--btd-only", action="store_true")
    ap.add_argument("--lu-only", action="store_true")
    ap.add_argument("--new", default=None, help="library under test (default: the product libawelu.so)")
    args = ap.parse_args()
    from awebox_amd.batched_lu import load_library
    libs = {"new": load_library(args.new) if args.new else load_library()}
    if os.path.exists(args.base):
        b = ctypes.CDLL(args.base)
        b.awelu_factor_batched.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        b.awelu_solve_batched.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4
        b.awelu_btd_factor_batched.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
        b.awelu_btd_solve_batched.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p] * 4
        b.awelu_sym_inertia_batched.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_double,
                                                ctypes.c_void_p, ctypes.c_void_p]
        b.awelu_last_error.restype = ctypes.c_char_p
        libs["base"] = b
    dev = "cuda"
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)
    for b, nb, m, nrhs in ([] if args.lu_only else [(8, 41, 46, 1), (1, 41, 46, 1), (8, 41, 46, 7), (1, 41, 46, 24), (7, 41, 46, 24), (64, 21, 22, 1)]):
        print(json.dumps(btd_ab(libs, b, nb, m, nrhs, dev, gen, args.reps)), flush=True)
    for b, nb, m, nrhs, boost in [(8, 41, 46, 1, 0.0), (64, 21, 22, 1, 0.0), (4, 9, 48, 3, 0.0), (4, 9, 17, 3, 0.0),
                                  (7, 41, 46, 1, 0.05)] if not args.lu_only else []:
        print(json.dumps(btd_ab(libs, b, nb, m, nrhs, dev, gen, args.reps, boost)), flush=True)
    if args.btd_only:
        return
    for b, n, nrhs in [(40, 268, 120), (280, 268, 70), (20, 640, 160), (140, 640, 160), (160, 100, 100), (1, 100, 100),
                       (7, 100, 100), (1280, 126, 44), (5120, 126, 44), (1, 46, 46)]:
        print(json.dumps(lu_ab(libs, b, n, nrhs, dev, gen, args.reps)), flush=True)
    if args.lu_only:
        return
    for b, n in [(20, 640), (140, 640), (40, 268), (320, 268), (40, 160), (40, 200), (1280, 126), (5120, 126), (41, 46), (328, 46), (1344, 22), (1, 1887)]:
        A = kkt_batch(b, n, dev, gen)
        rec = {"op": "inertia", "batch": b, "n": n}
        counts = {}
        for name, lib in libs.items():
            ms, c = timed(lib, A, args.reps)
            rec[name + "_ms"] = round(ms, 4)
            counts[name] = c
        ev = torch.linalg.eigvalsh(A)
        scale = A.abs().amax(dim=(1, 2), keepdim=True).squeeze(-1)
        pos = (ev > 1e-13 * scale).sum(1)
        neg = (ev < -1e-13 * scale).sum(1)
        ref = torch.stack([pos, neg, n - pos - neg], 1).to(torch.int32)
        for name, c in counts.items():
            rec[name + "_eq_eig"] = int((c == ref).all(1).sum())
        if "base" in counts:
            rec["new_eq_base"] = int((counts["new"] == counts["base"]).all(1).sum())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
