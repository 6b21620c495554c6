// awelu -- batched LU factorisation with partial pivoting of many mid-sized dense fp64 matrices
// (the interval blocks of the structured KKT solve, awebox_amd/ipm.py::StructuredKKT).
//
// Why: the library path (torch.linalg.lu_factor -> rocSOLVER getrf batched) takes ~2.5 ms per
// 640 x 640 matrix on MI355X and scales linearly with the batch (tools/kkt_micro.py), which made
// the KKT factorisation 85 % of a dual-kite interior-point iteration.  Here one workgroup
// factorises one matrix with a right-looking blocked algorithm:
//   * panel of NB = 16 columns staged in LDS (n x 16 doubles, <= 128 KB for n <= 1024), factorised
//     there with partial pivoting (column max by a workgroup reduction, row swap, scale, rank-1
//     update of the panel);
//   * the panel's row interchanges applied to the rest of the row (global memory);
//   * one thread per trailing column: the column's 16 U12 entries by forward substitution with
//     L11 (LDS, broadcast reads), then the trailing update A22 -= L21 U12 of that column with
//     coalesced row-wise accesses (L21 broadcast from LDS, U12 in registers).
// Output convention = LAPACK/torch.linalg.lu_factor: row-major LU (unit L below the diagonal, U on
// and above), 1-based pivots piv[k] = row exchanged with row k at step k; so torch.linalg.lu_solve
// consumes it directly.  A zero pivot is not an error here: the caller's refinement / backward
// error test sees the resulting non-finite values.
#include <hip/hip_runtime.h>

#include <string>

namespace {

constexpr int kNB = 16;
constexpr int kThreads = 256;
constexpr int kMaxN = 1024;

thread_local std::string g_err;

__global__ __launch_bounds__(kThreads) void lu_batched_kernel(int n, double* __restrict__ As, int* __restrict__ pivs) {
    extern __shared__ double panel[];                   // [n][kNB], row-major
    __shared__ double red_v[kThreads];
    __shared__ int red_i[kThreads];
    __shared__ int piv_loc[kNB];
    double* A = As + (size_t)blockIdx.x * n * n;
    int* piv = pivs + (size_t)blockIdx.x * n;
    const int tid = threadIdx.x;

    for (int k0 = 0; k0 < n; k0 += kNB) {
        const int kb = min(kNB, n - k0);
        const int rows = n - k0;
        // ---- stage the panel A[k0:n, k0:k0+kb] ----------------------------------------------
        for (int t = tid; t < rows * kb; t += kThreads) {
            const int r = t / kb, c = t % kb;
            panel[r * kNB + c] = A[(size_t)(k0 + r) * n + k0 + c];
        }
        __syncthreads();
        // ---- factorise the panel with partial pivoting ----------------------------------------
        for (int c = 0; c < kb; ++c) {
            double best = -1.0;
            int bi = c;
            for (int r = c + tid; r < rows; r += kThreads) {
                const double v = fabs(panel[r * kNB + c]);
                if (v > best) { best = v; bi = r; }
            }
            red_v[tid] = best;
            red_i[tid] = bi;
            __syncthreads();
            for (int s = kThreads / 2; s > 0; s >>= 1) {
                if (tid < s) {
                    const double o = red_v[tid + s];
                    const int oi = red_i[tid + s];
                    if (o > red_v[tid] || (o == red_v[tid] && oi < red_i[tid])) { red_v[tid] = o; red_i[tid] = oi; }
                }
                __syncthreads();
            }
            const int p = red_i[0];
            if (tid == 0) piv_loc[c] = p;
            if (p != c && tid < kb) {                        // swap panel rows c and p
                const double a = panel[c * kNB + tid];
                panel[c * kNB + tid] = panel[p * kNB + tid];
                panel[p * kNB + tid] = a;
            }
            __syncthreads();
            const double d = panel[c * kNB + c];
            const double rd = 1.0 / d;
            for (int r = c + 1 + tid; r < rows; r += kThreads) {
                const double l = panel[r * kNB + c] * rd;
                panel[r * kNB + c] = l;
                for (int j = c + 1; j < kb; ++j) panel[r * kNB + j] -= l * panel[c * kNB + j];
            }
            __syncthreads();
        }
        // ---- write the panel back, record pivots, apply the swaps outside the panel ----------------
        for (int t = tid; t < rows * kb; t += kThreads) {
            const int r = t / kb, c = t % kb;
            A[(size_t)(k0 + r) * n + k0 + c] = panel[r * kNB + c];
        }
        if (tid < kb) piv[k0 + tid] = k0 + piv_loc[tid] + 1;
        for (int c = 0; c < kb; ++c) {
            const int p = piv_loc[c];
            if (p == c) continue;
            const size_t ra = (size_t)(k0 + c) * n, rb = (size_t)(k0 + p) * n;
            for (int j = tid; j < n; j += kThreads) {
                if (j >= k0 && j < k0 + kb) continue;
                const double a = A[ra + j];
                A[ra + j] = A[rb + j];
                A[rb + j] = a;
            }
            __syncthreads();
        }
        __syncthreads();
        // ---- U12 (forward substitution with L11) and the trailing update, one column per thread --
        for (int j = k0 + kb + tid; j < n; j += kThreads) {
            double u[kNB];
#pragma unroll
            for (int r = 0; r < kNB; ++r) {
                if (r < kb) {
                    double v = A[(size_t)(k0 + r) * n + j];
                    for (int c = 0; c < r; ++c) v -= panel[r * kNB + c] * u[c];
                    u[r] = v;
                    A[(size_t)(k0 + r) * n + j] = v;
                } else {
                    u[r] = 0.0;
                }
            }
            for (int i = kb; i < rows; ++i) {
                double acc = A[(size_t)(k0 + i) * n + j];
#pragma unroll
                for (int c = 0; c < kNB; ++c) acc -= panel[i * kNB + c] * u[c];
                A[(size_t)(k0 + i) * n + j] = acc;
            }
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" {

const char* awelu_last_error(void) { return g_err.c_str(); }

// In-place LU with partial pivoting of `batch` row-major n x n matrices A[b][n][n] (device
// pointer); piv[b][n] receives 1-based pivots.  Asynchronous on `stream`.
int awelu_factor_batched(int n, int batch, double* A, int* piv, void* stream) {
    if (n < 1 || n > kMaxN || batch < 1 || !A || !piv) {
        g_err = "need 1 <= n <= 1024, batch >= 1 and device pointers";
        return 1;
    }
    const size_t lds = sizeof(double) * (size_t)n * kNB;
    lu_batched_kernel<<<dim3((unsigned)batch), kThreads, lds, (hipStream_t)stream>>>(n, A, piv);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

}  // extern "C"
