"""Phase timing of btd_factor_kernel from an instrumented build of the product source.

    python tools/btd_timing.py --build     # here (CPU): instrument awebox_amd/csrc/batched_lu.hip into
                                           # tools/exp_src/btd_timing.hip, compile tools/ab/libawelu_btdtiming.so
    python tools/btd_timing.py             # on the GPU box: run it

Block 0's thread 0 reads wall_clock64 (100 MHz) at the stage phases -- global loads, D -= L W,
Gauss-Jordan, write-out -- and clock64 (shader cycles) at the Gauss-Jordan column phases: column
publish + barrier, pivot search, pivot-row publish + barrier, update.  Prints us per stage, cycles
per column and the shader clock."""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "awebox_amd", "csrc", "batched_lu.hip")
OUT_SRC = os.path.join(ROOT, "tools", "exp_src", "btd_timing.hip")
OUT_LIB = os.path.join(ROOT, "abv", "libawelu_btdtiming.so")


def _after(s, anchor, text, start=0):
    i = s.index(anchor, start) + len(anchor)
    return s[:i] + text + s[i:], i


def _before(s, anchor, text, start=0):
    i = s.index(anchor, start)
    return s[:i] + text + s[i:], i + len(text)


def instrument(s):
    T = "{{ const unsigned long long t = {clk}(); {acc} += t - {prev}; {prev} = t; }}\n"
    s = s.replace("thread_local std::string g_err;", "thread_local std::string g_err;\n"
                  "__device__ unsigned long long g_btd_timing[10];", 1)
    k0 = s.index("void btd_factor_kernel(")
    s, i = _before(s, "    for (int k = 0; k < nb; ++k) {\n        const double* Lg", (
        "    unsigned long long t_load = 0, t_prod = 0, t_gj = 0, t_out = 0, t_prev = wall_clock64();\n"
        "    unsigned long long c_col = 0, c_piv = 0, c_row = 0, c_upd = 0, c_prev = 0, c_start = clock64(),"
        " w_start = t_prev;\n"), k0)
    s, i = _before(s, "        if (k > 0) {                                          // D -= L_k W_{k-1}",
                   "        " + T.format(clk="wall_clock64", acc="t_load", prev="t_prev"), i)
    s, i = _before(s, "        // Gauss-Jordan with partial pivoting",
                   "        " + T.format(clk="wall_clock64", acc="t_prod", prev="t_prev"), i)
    s, i = _after(s, "                if (c < m) {\n", "                    if (c == 0) c_prev = clock64();\n", i)
    s, i = _before(s, "                    __syncthreads();\n                    double kb",
                   "                    " + T.format(clk="clock64", acc="c_col", prev="c_prev"), i)
    s, i = _after(s, "                    __syncthreads();\n", "                    " + T.format(clk="clock64", acc="c_piv", prev="c_prev"), i)
    s, i = _after(s, "                    const int p = crow[bsel + wb];\n",
                  "                    " + T.format(clk="clock64", acc="c_row", prev="c_prev"), i)
    s, i = _before(s, "                    if (tid == 0) pivrow[c] = p;",
                   T.format(clk="clock64", acc="c_upd", prev="c_prev") + "                    ", i)
    s, i = _before(s, "        // row pivrow[c] holds row c of the result",
                   "        " + T.format(clk="wall_clock64", acc="t_gj", prev="t_prev"), i)
    end = "        __syncthreads();\n    }\n}\n"
    j = s.index(end, i)
    s = s[:j] + ("        __syncthreads();\n        " + T.format(clk="wall_clock64", acc="t_out", prev="t_prev") +
                 "    }\n    if (threadIdx.x == 0 && blockIdx.x == 0) {\n"
                 "        g_btd_timing[0] = t_load; g_btd_timing[1] = t_prod; g_btd_timing[2] = t_gj; g_btd_timing[3] = t_out;\n"
                 "        g_btd_timing[4] = c_col; g_btd_timing[5] = c_piv; g_btd_timing[6] = c_row; g_btd_timing[7] = c_upd;\n"
                 "        g_btd_timing[8] = clock64() - c_start; g_btd_timing[9] = wall_clock64() - w_start;\n"
                 "    }\n}\n") + s[j + len(end):]
    s = s.replace("const char* awelu_last_error(void) { return g_err.c_str(); }",
                  "const char* awelu_last_error(void) { return g_err.c_str(); }\n"
                  "int awelu_btd_timing(unsigned long long* out) {\n"
                  "    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_btd_timing), sizeof(unsigned long long) * 10);\n}", 1)
    return s


def build():
    os.makedirs(os.path.dirname(OUT_SRC), exist_ok=True)
    os.makedirs(os.path.dirname(OUT_LIB), exist_ok=True)
    with open(SRC) as fh:
        src = instrument(fh.read())
    with open(OUT_SRC, "w") as fh:
        fh.write(src)
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                    "-Wno-unused-value", "-Wno-unused-result", OUT_SRC, "-o", OUT_LIB], check=True)
    print(OUT_LIB)


def run():
    import torch
    lib = ctypes.CDLL(OUT_LIB)
    lib.awelu_btd_factor_batched.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    dev = "cuda"
    for b, nb, m in [(8, 41, 46), (64, 21, 22)]:
        T = torch.randn(b, nb, 3, m, m, dtype=torch.float64, device=dev)
        T[:, :, 1] += 4 * m * torch.eye(m, dtype=torch.float64, device=dev)
        Dinv = torch.empty(b, nb, m, m, dtype=torch.float64, device=dev)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        out = (ctypes.c_ulonglong * 10)()
        for _ in range(3):
            F = T.clone()
            lib.awelu_btd_factor_batched(nb, m, b, ctypes.c_void_p(F.data_ptr()), ctypes.c_void_p(Dinv.data_ptr()), st)
            torch.cuda.synchronize()
        lib.awelu_btd_timing(out)
        us = [v / 100.0 / nb for v in out[:4]]
        mhz = out[8] / out[9] * 100.0 if out[9] else 0.0
        cyc = {k: round(v / (nb * m), 1) for k, v in
               zip(["candidate+publish", "barrier", "pivot_choice", "update"], out[4:8])}
        print(json.dumps({"batch": b, "nb": nb, "m": m,
                          "us_per_stage": dict(zip(["load", "product", "gauss_jordan", "write"], [round(u, 2) for u in us])),
                          "us_per_gj_column": round(us[2] / m, 3), "shader_clock_mhz": round(mhz, 1),
                          "cycles_per_gj_column": cyc}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    build() if a.build else run()
