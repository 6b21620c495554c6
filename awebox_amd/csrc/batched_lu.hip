// awelu -- batched LU factorisation with partial pivoting of many mid-sized dense fp64 matrices
// (the interval blocks of the structured KKT solve, awebox_amd/ipm.py::StructuredKKT).
//
// Why: the library path (torch.linalg.lu_factor -> rocSOLVER getrf batched) takes ~2.5 ms per
// 640 x 640 matrix on MI355X and scales linearly with the batch (tools/kkt_micro.py), which made
// the KKT factorisation 85 % of a dual-kite interior-point iteration.  Here one workgroup
// factorises one matrix with a right-looking blocked algorithm:
//   * panel of NB = 16 columns staged in LDS (n x 16 doubles, <= 128 KB for n <= 1024), factorised
//     there with partial pivoting (column max by wave shuffles and one exchange of the four wave
//     maxima through LDS, row swap, scale, rank-1 update of the panel: three barriers per column);
//   * the panel's row interchanges applied to the rest of the row (global memory);
//   * one thread per trailing column: the column's 16 U12 entries by forward substitution with
//     L11 (LDS, broadcast reads), then the trailing update A22 -= L21 U12 of that column with
//     coalesced row-wise accesses (L21 broadcast from LDS, U12 in registers).
// Output convention = LAPACK/torch.linalg.lu_factor: row-major LU (unit L below the diagonal, U on
// and above), 1-based pivots piv[k] = row exchanged with row k at step k; so torch.linalg.lu_solve
// consumes it directly.  A zero pivot is not an error here: the caller's refinement / backward
// error test sees the resulting non-finite values.
#include <hip/hip_runtime.h>

#include "../../include/awelu.h"

#include <algorithm>
#include <string>

namespace {

constexpr int kNB = 16;
constexpr int kThreads = 256;
constexpr int kLuSmallN = 128;           // lu_batched_kernel<128> for blocks up to this size ...
constexpr int kLuSmallMinBatch = 1100;   // ... in batches beyond what 4 workgroups per CU hold
constexpr int kMaxN = 1024;

thread_local std::string g_err;

// dst(t) = src(t) for t = tid, tid + kThreads, ... < total with U global loads of a thread in flight
// before its first store: a plain loop waits one memory latency per element (the compiler cannot
// move the next load above a store it cannot disambiguate), which made the LDS staging of the
// factor panels and right-hand sides latency-bound.
template <int U, class Ld, class St>
__device__ __forceinline__ void copy_batched(int total, int tid, int nthreads, Ld ld, St st) {
    for (int t0 = tid; t0 < total; t0 += U * nthreads) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = t0 + u * nthreads;
            v[u] = t < total ? ld(t) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = t0 + u * nthreads;
            if (t < total) st(t, v[u]);
        }
    }
}

// Max over the 64 lanes of a wave by DPP moves (quad permutes, row rotations, row broadcasts: VALU
// latency) instead of a __shfl_xor butterfly (six dependent LDS-permute round trips); the result
// is read from lane 63 and is uniform.  fmax is order-independent, so the value is the butterfly's.
template <int Ctrl>
__device__ __forceinline__ double mov_dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, Ctrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), Ctrl, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double wave_max(double v) {
    v = fmax(v, mov_dpp_f64<0xb1>(v));                        // quad_perm [1,0,3,2]
    v = fmax(v, mov_dpp_f64<0x4e>(v));                        // quad_perm [2,3,0,1]
    v = fmax(v, mov_dpp_f64<0x124>(v));                       // row_ror 4
    v = fmax(v, mov_dpp_f64<0x128>(v));                       // row_ror 8
    v = fmax(v, mov_dpp_f64<0x142>(v));                       // row_bcast 15
    v = fmax(v, mov_dpp_f64<0x143>(v));                       // row_bcast 31
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Min over the 64 lanes of a wave (the same DPP steps on 32-bit integers); uniform result.
__device__ __forceinline__ int wave_min_i32(int v) {
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0xb1, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4e, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x124, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x128, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x142, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x143, 0xf, 0xf, false));
    return __builtin_amdgcn_readlane(v, 63);
}

template <int NT>
__global__ __launch_bounds__(NT) void lu_batched_kernel(int n, double* __restrict__ As, int* __restrict__ pivs) {
    extern __shared__ double panel[];                   // [n][kNB], row-major
    __shared__ double red_v[NT / 64];
    __shared__ int red_i[NT / 64];
    __shared__ int piv_loc[kNB];
    __shared__ int orgmap[kMaxN];                       // row -> original row under the panel's swaps
    __shared__ int perm_pos[2 * kNB], perm_org[2 * kNB]; // the panel's interchanges as one permutation
    double* A = As + (size_t)blockIdx.x * n * n;
    int* piv = pivs + (size_t)blockIdx.x * n;
    const int tid = threadIdx.x;
    for (int i = tid; i < n; i += NT) orgmap[i] = i;

    for (int k0 = 0; k0 < n; k0 += kNB) {
        const int kb = min(kNB, n - k0);
        const int rows = n - k0;
        // ---- stage the panel A[k0:n, k0:k0+kb] ----------------------------------------------
        copy_batched<8>(rows * kb, tid, NT,
                        [&](int t) { return A[(size_t)(k0 + t / kb) * n + k0 + t % kb]; },
                        [&](int t, double v) { panel[(t / kb) * kNB + t % kb] = v; });
        __syncthreads();
        // ---- factorise the panel with partial pivoting ----------------------------------------
        for (int c = 0; c < kb; ++c) {
            double best = -1.0;
            int bi = c;
            for (int r = c + tid; r < rows; r += NT) {
                const double v = fabs(panel[r * kNB + c]);
                if (v > best) { best = v; bi = r; }
            }
            {   // the wave's (largest value, lowest row holding it): a DPP max of the values, then a
                // DPP min of the rows of the lanes holding it -- the pair the (value, index)
                // butterfly found, without its twelve dependent LDS permutes (best is never NaN:
                // NaN does not pass v > best, a lane without rows keeps -1)
                const double mx = wave_max(best);
                bi = wave_min_i32(best == mx ? bi : 0x7fffffff);
                best = mx;
            }
            if ((tid & 63) == 0) {
                red_v[tid >> 6] = best;
                red_i[tid >> 6] = bi;
            }
            __syncthreads();
            best = red_v[0];
            bi = red_i[0];
            for (int w = 1; w < NT / 64; ++w) {         // the 4 wave results, same order everywhere
                if (red_v[w] > best || (red_v[w] == best && red_i[w] < bi)) { best = red_v[w]; bi = red_i[w]; }
            }
            const int p = bi;
            if (tid == 0) {
                piv_loc[c] = p;
                const int o = orgmap[k0 + c];                // the same interchange on the row map
                orgmap[k0 + c] = orgmap[k0 + p];
                orgmap[k0 + p] = o;
            }
            if (p != c && tid < kb) {                        // swap panel rows c and p
                const double a = panel[c * kNB + tid];
                panel[c * kNB + tid] = panel[p * kNB + tid];
                panel[p * kNB + tid] = a;
            }
            __syncthreads();
            const double d = panel[c * kNB + c];
            const double rd = 1.0 / d;
            for (int r = c + 1 + tid; r < rows; r += NT) {
                const double l = panel[r * kNB + c] * rd;
                panel[r * kNB + c] = l;
                for (int j = c + 1; j < kb; ++j) panel[r * kNB + j] -= l * panel[c * kNB + j];
            }
            __syncthreads();
        }
        // ---- write the panel back, record pivots; the kb sequential interchanges as one permutation
        //      of the rows they touch (positions k0 + c and k0 + piv_loc[c]; a position listed twice
        //      moves the same value twice), applied with all loads of a column before its stores --
        for (int t = tid; t < rows * kb; t += NT) {
            const int r = t / kb, c = t % kb;
            A[(size_t)(k0 + r) * n + k0 + c] = panel[r * kNB + c];
        }
        if (tid < kb) piv[k0 + tid] = k0 + piv_loc[tid] + 1;
        if (tid < 2 * kNB) {
            const int pos = tid < kb ? k0 + tid : (tid - kNB < kb && tid >= kNB ? k0 + piv_loc[tid - kNB] : k0);
            perm_pos[tid] = pos;
            perm_org[tid] = orgmap[pos];
        }
        __syncthreads();
        if (tid < 2 * kNB) orgmap[perm_pos[tid]] = perm_pos[tid];   // back to the identity
        for (int j = tid; j < n; j += NT) {            // interchanges outside the panel: each
            if (j >= k0 && j < k0 + kb) continue;            // thread owns its columns
            double v[2 * kNB];
#pragma unroll
            for (int e = 0; e < 2 * kNB; ++e) v[e] = A[(size_t)perm_org[e] * n + j];
#pragma unroll
            for (int e = 0; e < 2 * kNB; ++e) A[(size_t)perm_pos[e] * n + j] = v[e];
        }
        __syncthreads();
        // ---- U12 (forward substitution with L11) and the trailing update, one column per thread:
        //      the column's kb U12 rows loaded together, then the trailing rows in groups of kRowU
        //      whose loads are issued one group ahead (a memory latency per group, not per row).
        //      Fewer trailing columns than threads / 2 (the last panels; every panel of the MPC's
        //      126-row blocks): H = threads / columns row chunks per column, one (column, chunk) per
        //      thread, each chunk's thread repeating the column's substitution (the same operations per
        //      entry, so the factors are bitwise those of one thread per column); chunk 0 repeats it
        //      once more after the panel's last barrier, when every chunk has read U12, and stores it --
        constexpr int kRowU = 8;
        auto subst = [&](int j, double (&u)[kNB]) {
#pragma unroll
            for (int r = 0; r < kNB; ++r) u[r] = r < kb ? A[(size_t)(k0 + r) * n + j] : 0.0;
#pragma unroll
            for (int r = 0; r < kNB; ++r) {
                if (r < kb) {
                    double v = u[r];
                    for (int c = 0; c < r; ++c) v -= panel[r * kNB + c] * u[c];
                    u[r] = v;
                }
            }
        };
        auto put_u = [&](int j, const double (&u)[kNB]) {
#pragma unroll
            for (int r = 0; r < kNB; ++r)
                if (r < kb) A[(size_t)(k0 + r) * n + j] = u[r];
        };
        auto trail = [&](int j, int r0, int r1, const double (&u)[kNB]) {
            double nxt[kRowU];
#pragma unroll
            for (int q = 0; q < kRowU; ++q) nxt[q] = r0 + q < r1 ? A[(size_t)(k0 + r0 + q) * n + j] : 0.0;
            for (int i0 = r0; i0 < r1; i0 += kRowU) {
                double acc[kRowU];
#pragma unroll
                for (int q = 0; q < kRowU; ++q) acc[q] = nxt[q];
#pragma unroll
                for (int q = 0; q < kRowU; ++q) {
                    const int i = i0 + kRowU + q;
                    nxt[q] = i < r1 ? A[(size_t)(k0 + i) * n + j] : 0.0;
                }
#pragma unroll
                for (int q = 0; q < kRowU; ++q) {
                    const int i = i0 + q;
                    if (i < r1) {
#pragma unroll
                        for (int c = 0; c < kNB; ++c) acc[q] -= panel[i * kNB + c] * u[c];
                        A[(size_t)(k0 + i) * n + j] = acc[q];
                    }
                }
            }
        };
        const int ncols = n - k0 - kb;
        const int H = ncols > 0 ? max(1, min(4, NT / ncols)) : 1;
        int jd = -1;
        if (H == 1) {
            for (int j = k0 + kb + tid; j < n; j += NT) {
                double u[kNB];
                subst(j, u);
                put_u(j, u);
                trail(j, kb, rows, u);
            }
        } else {
            // H > 1: ncols H <= NT, one (column, row chunk) item per thread.  (This loop form
            // measured 7.8 ms for 20 x 640 against 10.3 ms for the same work as an if on tid;
            // profiles/r05/solver/lu_variants.)
            for (int it = tid; it < ncols * H; it += NT) {
                const int h = it / ncols, j = k0 + kb + (it - h * ncols);
                double u[kNB];
                subst(j, u);
                if (H == 1) {
                    put_u(j, u);
                } else if (h == 0) {
                    jd = j;
                }
                const int len = (rows - kb + H - 1) / H;
                const int r0 = kb + h * len;
                trail(j, r0, min(rows, r0 + len), u);
            }
        }
        __syncthreads();
        if (jd >= 0) {                                       // every chunk has read U12 by now: the
            double u[kNB];                                   // substitution again (same values), stored
            subst(jd, u);
            put_u(jd, u);
        }
        if (H > 1) __syncthreads();                          // L11 (panel) read before the next staging
    }
}

// Solve A X = B with the factors of lu_batched_kernel, for the columns [j0, j0 + w) of the
// row-major right-hand sides X[b][n][ldx] (in place).  One workgroup per matrix; the w columns of
// X live in LDS for the whole solve, and the factors stream through LDS in 16-column panels:
//   forward (unit L):  panel L[k0:n, k0:k0+16]; the 16 x 16 diagonal block by substitution (one
//                      thread per right-hand side, in registers), then every later row updated by a
//                      16-term dot product (threads over rows x cols);
//   backward (U):      panel U[0:k1+16, k1:k1+16], bottom block first, same two phases.
// The library path (rocBLAS trsv for one right-hand side) re-reads the factors per column step
// from HBM: 20 ms for 256 systems of n = 463 against ~0.1 ms here.
__global__ __launch_bounds__(kThreads) void lu_solve_kernel(int n, int ldx, int wchunk,
                                                           const double* __restrict__ LUs,
                                                           const int* __restrict__ pivs,
                                                           double* __restrict__ Xs) {
    extern __shared__ double sm[];
    const int j0 = blockIdx.y * wchunk;                  // this workgroup's right-hand sides
    const int w = min(wchunk, ldx - j0);
    double* panel = sm;                                  // [n][kNB]
    double* X = sm + (size_t)n * kNB;                    // [n][w]
    const double* A = LUs + (size_t)blockIdx.x * n * n;
    const int* piv = pivs + (size_t)blockIdx.x * n;
    double* Xg = Xs + (size_t)blockIdx.x * n * ldx + j0;
    const int tid = threadIdx.x;

    copy_batched<8>(n * w, tid, kThreads, [&](int t) { return Xg[(size_t)(t / w) * ldx + t % w]; },
                    [&](int t, double v) { X[t] = v; });
    __syncthreads();
    for (int j = tid; j < w; j += kThreads) {            // row interchanges, one column per thread
        for (int k = 0; k < n; ++k) {
            const int p = piv[k] - 1;
            if (p != k) {
                const double a = X[k * w + j];
                X[k * w + j] = X[p * w + j];
                X[p * w + j] = a;
            }
        }
    }
    __syncthreads();
    // ---- forward substitution with the unit lower factor --------------------------------------
    for (int k0 = 0; k0 < n; k0 += kNB) {
        const int kb = min(kNB, n - k0), rows = n - k0;
        copy_batched<8>(rows * kb, tid, kThreads, [&](int t) { return A[(size_t)(k0 + t / kb) * n + k0 + t % kb]; },
                        [&](int t, double v) { panel[(t / kb) * kNB + t % kb] = v; });
        __syncthreads();
        // the kb x kb unit-lower diagonal block: one thread per right-hand side, the substitution
        // in registers (per entry the subtractions of the column-by-column form in the same order:
        // bitwise the same, without its kb - 1 barriers)
        for (int j = tid; j < w; j += kThreads) {
            double x[kNB];
#pragma unroll
            for (int r = 0; r < kNB; ++r) x[r] = r < kb ? X[(k0 + r) * w + j] : 0.0;
#pragma unroll
            for (int r = 1; r < kNB; ++r) {
                if (r < kb) {
                    double v = x[r];
#pragma unroll
                    for (int c = 0; c < r; ++c) v -= panel[r * kNB + c] * x[c];
                    x[r] = v;
                }
            }
#pragma unroll
            for (int r = 0; r < kNB; ++r)
                if (r < kb) X[(k0 + r) * w + j] = x[r];
        }
        __syncthreads();
        for (int t = tid; t < (rows - kb) * w; t += kThreads) {
            const int r = kb + t / w, j = t % w;
            double acc = X[(k0 + r) * w + j];
            for (int c = 0; c < kb; ++c) acc -= panel[r * kNB + c] * X[(k0 + c) * w + j];
            X[(k0 + r) * w + j] = acc;
        }
        __syncthreads();
    }
    // ---- backward substitution with the upper factor ------------------------------------------
    for (int k1 = ((n - 1) / kNB) * kNB; k1 >= 0; k1 -= kNB) {
        const int kb = min(kNB, n - k1), rows = k1 + kb;
        copy_batched<8>(rows * kb, tid, kThreads, [&](int t) { return A[(size_t)(t / kb) * n + k1 + t % kb]; },
                        [&](int t, double v) { panel[(t / kb) * kNB + t % kb] = v; });
        __syncthreads();
        // the upper diagonal block, one thread per right-hand side (same order per entry)
        for (int j = tid; j < w; j += kThreads) {
            double x[kNB];
#pragma unroll
            for (int r = 0; r < kNB; ++r) x[r] = r < kb ? X[(k1 + r) * w + j] : 0.0;
#pragma unroll
            for (int c = kNB - 1; c >= 0; --c) {
                if (c < kb) {
                    x[c] /= panel[(k1 + c) * kNB + c];
#pragma unroll
                    for (int r = 0; r < c; ++r) x[r] -= panel[(k1 + r) * kNB + c] * x[c];
                }
            }
#pragma unroll
            for (int r = 0; r < kNB; ++r)
                if (r < kb) X[(k1 + r) * w + j] = x[r];
        }
        __syncthreads();
        for (int t = tid; t < k1 * w; t += kThreads) {
            const int r = t / w, j = t % w;
            double acc = X[r * w + j];
            for (int c = 0; c < kb; ++c) acc -= panel[r * kNB + c] * X[(k1 + c) * w + j];
            X[r * w + j] = acc;
        }
        __syncthreads();
    }
    for (int t = tid; t < n * w; t += kThreads) Xg[(size_t)(t / w) * ldx + t % w] = X[t];
}

constexpr size_t kSolveLds = 144 * 1024;
constexpr long kSolveTargetWgs = 256;                   // one per CU
constexpr long kSolveMinChunk = 16;

// Block-tridiagonal systems, one workgroup per system: nb diagonal blocks of m x m (m <= 48),
// T[b][k][3][m][m] = (sub-diagonal block L_k = (k, k-1), diagonal block D_k, super-diagonal block
// U_k = (k, k+1)).  This is the separator system of the structured KKT in stage order (shooting
// states and continuity multipliers alternate), and the sweep below is its Riccati recursion;
// there are no interchanges between block rows, partial pivoting inside each diagonal block.
//
// btd_factor_kernel:  D'_k = D_k - L_k W_{k-1},  [W_k | D'_k^-1] = D'_k^-1 [U_k | I]
//   by Gauss-Jordan on the augmented block [D'_k | U_k | I] held in registers (a wave per 12 rows;
//   per column each wave publishes its own pivot candidate row and one barrier later every thread
//   picks the same pivot: one barrier per column; the row interchange is folded into the
//   elimination of every other row).  W_k
//   overwrites U_k; D'_k^-1 goes to Dinv[b][k][m][m]; W_{k-1} stays in LDS for the next stage
//   (two augmented blocks and W_{k-1} take 130 KB at m = 48).
//   D'_k itself replaces D_k in T.
// btd_apply_kernel:   Y_k = D'_k^-1 (X_k - L_k Y_{k-1}),  then x_k = Y_k - W_k x_{k+1}: matrix
//   products streamed stage by stage, right-hand sides [j0, j0 + w) of X[b][nb m][ldx].  The
//   explicit inverse alone leaves a backward error of cond(D'_k) eps (the KKT's pivot blocks reach
//   cond ~1e11), so every block solve takes one refinement step with D'_k: Y += D'^-1 (Z - D' Y).
// The factorisation is reused by every solve of an interior-point iteration (iterative
// refinement), and the apply is one launch per solve instead of a library LU's dozens.
// Templated on the workgroup size and the block limit.  A one-wave instantiation <64, 24> for the
// MPC's m = 22 (no barriers between the Gauss-Jordan columns, the same arithmetic) measured slower
// than <256, 48>: 1.28 vs 1.06 ms per 21-stage factorisation at B = 64 (tools/awelu_ab.py), so only
// <256, 48> is instantiated.
constexpr int kBtdMaxM = 48;
constexpr int kBtdMaxRhs = 64;

template <int NT, int MAXM>
__global__ __launch_bounds__(NT) void btd_factor_kernel(int nb, int m, double* __restrict__ Ts,
                                                       double* __restrict__ Dinvs) {
    constexpr int kRG = NT / 64;                              // row groups of the kRG x 64 grid
    // two buffers of the augmented block [D | U | I]: every Gauss-Jordan column reads one and writes
    // the other (row interchange folded into the update), so a column costs one barrier; the
    // second buffer holds L_k while D' = D - L_k W_{k-1} is formed
    __shared__ double R0[MAXM][3 * MAXM + 1];
    __shared__ double R1[MAXM][3 * MAXM + 1];
    __shared__ double Wp[MAXM][MAXM + 1];             // W_{k-1}
    const int tid = threadIdx.x, tj = tid & 63, ti = tid >> 6;
    const size_t mm = (size_t)m * m;
    double* T = Ts + (size_t)blockIdx.x * nb * 3 * mm;
    double* Dinv = Dinvs + (size_t)blockIdx.x * nb * mm;
    const int na = 3 * m;

    for (int k = 0; k < nb; ++k) {
        const double* Lg = T + ((size_t)k * 3 + 0) * mm;
        double* Dg = T + ((size_t)k * 3 + 1) * mm;
        double* Ug = T + ((size_t)k * 3 + 2) * mm;
        const bool last = k == nb - 1;
        {
            // the stage's three blocks: every global load of a thread issued before its first LDS
            // store, so the 3 x 12 row loads overlap instead of paying one memory latency each
            constexpr int R = MAXM / kRG;
            double vd[R], vu[R], vl[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int i = ti + r * kRG;
                const bool in = i < m && tj < m;
                vd[r] = in ? Dg[i * m + tj] : 0.0;
                vu[r] = (in && !last) ? Ug[i * m + tj] : 0.0;
                vl[r] = (in && k > 0) ? Lg[i * m + tj] : 0.0;
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int i = ti + r * kRG;
                if (i < m && tj < m) {
                    R0[i][tj] = vd[r];
                    R0[i][m + tj] = vu[r];
                    R0[i][2 * m + tj] = i == tj ? 1.0 : 0.0;
                    if (k > 0) R1[i][tj] = vl[r];
                }
            }
        }
        __syncthreads();
        if (k > 0) {                                          // D -= L_k W_{k-1}
            // thread (ti, tj): column j = tj (< m <= 48 < 64), rows ti, ti + 4, ...: 12 independent
            // accumulators per thread, so the LDS loads of one c step pipeline
            constexpr int kRows = MAXM / kRG;
            const int j = tj;
            if (j < m) {
                double acc[kRows];
#pragma unroll
                for (int r = 0; r < kRows; ++r) acc[r] = 0.0;
                // rows i >= m (padding, < MAXM) are accumulated too and never written: a guard per
                // row compiled to a branch with its own LDS wait per product
                for (int c = 0; c < m; ++c) {
                    const double wc = Wp[c][j];
#pragma unroll
                    for (int r = 0; r < kRows; ++r) acc[r] += R1[ti + r * kRG][c] * wc;
                }
#pragma unroll
                for (int r = 0; r < kRows; ++r) {
                    const int i = ti + r * kRG;
                    if (i < m) R0[i][j] -= acc[r];
                }
            }
            __syncthreads();
        }
        for (int i = ti; i < m; i += kRG)                     // keep D'_k for the solves' refinement
            for (int j = tj; j < m; j += 64) Dg[i * m + j] = R0[i][j];
        // Gauss-Jordan with partial pivoting, the augmented block held in registers: wave w owns
        // rows kWR w .. kWR w + kWR - 1, lane (rq, cq) = (lane / 16, lane % 16) the kLR x kLC tile
        // (rows kWR w + kLR rq .., columns kLC cq ..) of [D' | U | I].  Per column c every wave
        // finds its own pivot candidate -- the largest |entry| among its unused rows, its lowest
        // such row on ties -- and publishes key (that magnitude; -1: no finite candidate, its
        // lowest unused row instead; -2: no unused row), row and the whole candidate row; after ONE
        // barrier every thread takes the same pivot from the four candidates (largest key, lowest
        // wave on ties: the lowest row holding the column maximum, as the block-wide search of the
        // previous two-barrier form) and reads its kLC pivot-row entries, and its rows' multipliers
        // come from the lane of its row group holding column c (a shuffle before the barrier).
        // The arithmetic per entry is the previous form's: pr = a[p][.] (1 / a[p][c]),
        // a[r][.] -= a[r][c] pr, row p := pr -- factors bitwise equal.  Candidate buffers alternate
        // between columns (c & 1): a wave writes column c + 2's only after every wave has passed
        // column c + 1's barrier, i.e. finished reading column c's.  Rows are not interchanged:
        // row piv[c] ends as row c of [I | W | D'^-1] and is written there.
        static_assert(NT == 256 && MAXM == 48, "tile layout of the Gauss-Jordan loop");
        constexpr int kWR = MAXM / kRG, kLR = kWR / 4, kLC = 3 * MAXM / 16;     // 12 rows, 3 x 9 tiles
        const int rq = tj >> 4, cq = tj & 15;
        const int row0 = ti * kWR + rq * kLR;
        double a[kLR][kLC];
#pragma unroll
        for (int i = 0; i < kLR; ++i)
#pragma unroll
            for (int q = 0; q < kLC; ++q) {
                const int r = row0 + i, j = cq * kLC + q;
                a[i][q] = (r < m && j < na) ? R0[r][j] : 0.0;
            }
        double* cbuf = &R1[0][0];                             // [2][kRG][3 MAXM] candidate rows
        double* ckey = cbuf + 2 * kRG * 3 * MAXM;             // [2][kRG]
        int* crow = reinterpret_cast<int*>(ckey + 2 * kRG);   // [2][kRG]
        int* pivrow = crow + 2 * kRG;                         // pivot row of column c
        const int wr0 = ti * kWR, wr1 = min(m, wr0 + kWR);
        const unsigned long long wmask = wr1 > wr0 ? (((1ull << (wr1 - wr0)) - 1ull) << wr0) : 0ull;
        unsigned long long usedmask = 0ull;                   // rows already pivots (m <= 48, uniform)
        __syncthreads();
        for (int cg = 0; cg * kLC < m; ++cg) {
#pragma unroll
            for (int qc = 0; qc < kLC; ++qc) {
                const int c = cg * kLC + qc;
                if (c < m) {
                    const int bsel = (c & 1) * kRG;
                    // this lane's candidate: its rows' column-c entries (lanes of column group cg)
                    double best = -1.0;
                    int bi = -1;
                    if (cq == cg) {
#pragma unroll
                        for (int i = 0; i < kLR; ++i) {
                            const int r = row0 + i;
                            const double v = fabs(a[i][qc]);
                            if (r < m && !((usedmask >> r) & 1ull) && v > best) { best = v; bi = r; }
                        }
                    }
                    const double mx = wave_max(best);
                    const unsigned long long hit = __ballot(bi >= 0 && best == mx);
                    int kr;
                    double key;
                    if (hit) {
                        kr = __builtin_amdgcn_readlane(bi, __ffsll((long long)hit) - 1);
                        key = mx;
                    } else {
                        const unsigned long long fr = wmask & ~usedmask;
                        kr = fr ? __ffsll((long long)fr) - 1 : -1;
                        key = fr ? -1.0 : -2.0;
                    }
                    // multipliers of this lane's rows: column c from lane (rq, cg)
                    double f[kLR];
#pragma unroll
                    for (int i = 0; i < kLR; ++i) f[i] = __shfl(a[i][qc], (tj & ~15) | cg);
#pragma unroll
                    for (int i = 0; i < kLR; ++i)
                        if (row0 + i == kr) {
#pragma unroll
                            for (int q = 0; q < kLC; ++q) cbuf[(bsel + ti) * 3 * MAXM + cq * kLC + q] = a[i][q];
                        }
                    if (tj == 0) {
                        ckey[bsel + ti] = key;
                        crow[bsel + ti] = kr;
                    }
                    __syncthreads();
                    double kb = ckey[bsel];
                    int wb = 0;
#pragma unroll
                    for (int w = 1; w < kRG; ++w) {
                        const double kw = ckey[bsel + w];
                        if (kw > kb) { kb = kw; wb = w; }
                    }
                    const int p = crow[bsel + wb];
                    usedmask |= 1ull << p;
                    const double* prow = cbuf + (bsel + wb) * 3 * MAXM;
                    const double rp = 1.0 / prow[c];
                    double pr[kLC];
#pragma unroll
                    for (int q = 0; q < kLC; ++q) pr[q] = prow[cq * kLC + q] * rp;
#pragma unroll
                    for (int i = 0; i < kLR; ++i)
#pragma unroll
                        for (int q = 0; q < kLC; ++q) a[i][q] = a[i][q] - f[i] * pr[q];
#pragma unroll
                    for (int i = 0; i < kLR; ++i)
                        if (row0 + i == p) {
#pragma unroll
                            for (int q = 0; q < kLC; ++q) a[i][q] = pr[q];
                        }
                    if (tid == 0) pivrow[c] = p;
                }
            }
        }
        __syncthreads();
        // row pivrow[c] holds row c of the result: scatter back to R0 in order
#pragma unroll
        for (int i = 0; i < kLR; ++i)
#pragma unroll
            for (int q = 0; q < kLC; ++q) {
                const int r = row0 + i, j = cq * kLC + q;
                if (r < m && j < na) R0[r][j] = a[i][q];
            }
        __syncthreads();
        double (*src)[3 * MAXM + 1] = R0;
        const int* rowof = pivrow;
        for (int i = ti; i < m; i += kRG) {
            const int ri = rowof[i];
            for (int j = tj; j < m; j += 64) {
                Wp[i][j] = src[ri][m + j];
                if (!last) Ug[i * m + j] = src[ri][m + j];
                Dinv[(size_t)k * mm + i * m + j] = src[ri][2 * m + j];
            }
        }
        __syncthreads();
    }
}

// Z[i][j] (-)= sum_c M[i][c] Y[c][j] for i < m, j < w: one thread per (i, j) over the whole
// workgroup (consecutive threads take consecutive columns of a row: M[i][c] is a broadcast,
// Y[c][j] conflict-free), the m products summed in order from LDS (independent loads, they
// pipeline).  The previous forms -- a wave per (i, j) with a shuffle-tree sum for few right-hand
// sides (six dependent cross-lane steps per row), one thread per (row group, column) otherwise (12
// rows serially per thread; 4 of 256 threads busy for one column) -- were latency-bound: the
// 41-stage solve took 3.1 ms, 2.2 ms with this mapping for one column.
template <int K, int SIGN, int NT, int MAXM>
__device__ __forceinline__ void btd_chains(double (*M)[MAXM + 1], double (*Yv)[kBtdMaxRhs + 1],
                                           double (*Zv)[kBtdMaxRhs + 1], double (*Out)[kBtdMaxRhs + 1],
                                           int m, int w, int total, int p0, bool init_zero) {
    int ii[K], jj[K];
    double acc[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        const int p = p0 + u * NT;
        ii[u] = p / w;
        jj[u] = p - ii[u] * w;
        acc[u] = 0.0;
    }
#pragma unroll 8
    for (int c = 0; c < m; ++c) {
#pragma unroll
        for (int u = 0; u < K; ++u) acc[u] += M[ii[u]][c] * Yv[c][jj[u]];
    }
#pragma unroll
    for (int u = 0; u < K; ++u) Out[ii[u]][jj[u]] = (init_zero ? 0.0 : Zv[ii[u]][jj[u]]) + SIGN * acc[u];
}

template <int SIGN, int NT, int MAXM>
__device__ __forceinline__ void btd_matmul(double (*M)[MAXM + 1], double (*Yv)[kBtdMaxRhs + 1],
                                           double (*Zv)[kBtdMaxRhs + 1], double (*Out)[kBtdMaxRhs + 1],
                                           int m, int w, int ti, int tj, bool init_zero) {
    // a thread's outputs p, p + NT, .. (several when w > 1: the factorisation's T^-1 E with the
    // border columns) four or two at a time, so their in-order sums run as independent chains
    const int total = m * w;
    int p0 = ti * 64 + tj;
    while (p0 < total) {
        const int left = (total - p0 + NT - 1) / NT;
        if (left >= 4) {
            btd_chains<4, SIGN, NT, MAXM>(M, Yv, Zv, Out, m, w, total, p0, init_zero);
            p0 += 4 * NT;
        } else if (left >= 2) {
            btd_chains<2, SIGN, NT, MAXM>(M, Yv, Zv, Out, m, w, total, p0, init_zero);
            p0 += 2 * NT;
        } else {
            btd_chains<1, SIGN, NT, MAXM>(M, Yv, Zv, Out, m, w, total, p0, init_zero);
            p0 += NT;
        }
    }
}

template <int NT, int MAXM>
__global__ __launch_bounds__(NT) void btd_apply_kernel(int nb, int m, int ldx, int j0_base, int wchunk,
                                                            const double* __restrict__ Ts,
                                                            const double* __restrict__ Dinvs,
                                                            double* __restrict__ Xs) {
    // right-hand sides [j0, j0 + w) of this workgroup: chunk blockIdx.y of width wchunk (every column
    // is computed by the same operations whatever chunk it is in)
    const int j0 = j0_base + (int)blockIdx.y * wchunk;
    const int w = min(wchunk, ldx - j0);
    if (w <= 0) return;
    __shared__ double A[MAXM][MAXM + 1];
    __shared__ double Ai[MAXM][MAXM + 1];
    __shared__ double Dp[MAXM][MAXM + 1];
    __shared__ double Y[MAXM][kBtdMaxRhs + 1];
    __shared__ double Z[MAXM][kBtdMaxRhs + 1];
    __shared__ double Q[MAXM][kBtdMaxRhs + 1];
    constexpr int kRG = NT / 64;
    const int tid = threadIdx.x, tj = tid & 63, ti = tid >> 6;
    const size_t mm = (size_t)m * m;
    const double* T = Ts + (size_t)blockIdx.x * nb * 3 * mm;
    const double* Dinv = Dinvs + (size_t)blockIdx.x * nb * mm;
    double* X = Xs + (size_t)blockIdx.x * nb * m * ldx + j0;
    // a stage's global loads (right-hand sides and up to three blocks, 12 rows each per thread,
    // tj < 64 covers the m <= 48 and w <= 64 columns) are all issued before the first LDS store:
    // one memory latency per stage instead of one per row and block (the chain is latency-bound)
    constexpr int R = MAXM / kRG;

    // stage k + 1's loads are issued right after stage k's LDS stores and its barrier, so they are
    // in flight during stage k's four dependent products instead of starting the next stage
    double vz[R], vl[R], vi[R], vp[R];
    auto load_fwd = [&](int k) {
        const double* Xk = X + (size_t)k * m * ldx;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = ti + r * kRG;
            const bool in = i < m && tj < m;
            vz[r] = (i < m && tj < w) ? Xk[(size_t)i * ldx + tj] : 0.0;
            vl[r] = (in && k > 0) ? T[((size_t)k * 3 + 0) * mm + i * m + tj] : 0.0;
            vi[r] = in ? Dinv[(size_t)k * mm + i * m + tj] : 0.0;
            vp[r] = in ? T[((size_t)k * 3 + 1) * mm + i * m + tj] : 0.0;
        }
    };
    load_fwd(0);
    for (int k = 0; k < nb; ++k) {                            // forward: Y_k
        double* Xk = X + (size_t)k * m * ldx;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = ti + r * kRG;
            if (i < m) {
                if (tj < w) Z[i][tj] = vz[r];
                if (tj < m) { A[i][tj] = vl[r]; Ai[i][tj] = vi[r]; Dp[i][tj] = vp[r]; }
            }
        }
        __syncthreads();
        if (k + 1 < nb) load_fwd(k + 1);
        if (k > 0) {                                          // Z -= L_k Y_{k-1}
            btd_matmul<-1, NT, MAXM>(A, Y, Z, Z, m, w, ti, tj, false);
            __syncthreads();
        }
        btd_matmul<1, NT, MAXM>(Ai, Z, Z, Y, m, w, ti, tj, true);       // Y = D'^-1 Z
        __syncthreads();
        btd_matmul<-1, NT, MAXM>(Dp, Y, Z, Q, m, w, ti, tj, false);     // one refinement step: Q = Z - D' Y
        __syncthreads();
        btd_matmul<1, NT, MAXM>(Ai, Q, Y, Y, m, w, ti, tj, false);      // Y += D'^-1 Q
        __syncthreads();
        for (int i = ti; i < m; i += kRG)
            for (int j = tj; j < w; j += 64) Xk[(size_t)i * ldx + j] = Y[i][j];
    }
    double vu[R];
    auto load_bwd = [&](int k) {
        const double* Xk = X + (size_t)k * m * ldx;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = ti + r * kRG;
            vu[r] = (i < m && tj < m) ? T[((size_t)k * 3 + 2) * mm + i * m + tj] : 0.0;
            vz[r] = (i < m && tj < w) ? Xk[(size_t)i * ldx + tj] : 0.0;
        }
    };
    if (nb >= 2) load_bwd(nb - 2);
    for (int k = nb - 2; k >= 0; --k) {                       // backward: x_k = Y_k - W_k x_{k+1}
        double* Xk = X + (size_t)k * m * ldx;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = ti + r * kRG;
            if (i < m) {
                if (tj < m) A[i][tj] = vu[r];
                if (tj < w) Z[i][tj] = vz[r];
            }
        }
        __syncthreads();
        if (k > 0) load_bwd(k - 1);
        btd_matmul<-1, NT, MAXM>(A, Y, Z, Z, m, w, ti, tj, false);
        __syncthreads();
        for (int i = ti; i < m; i += kRG) {
            for (int j = tj; j < w; j += 64) {
                Y[i][j] = Z[i][j];
                Xk[(size_t)i * ldx + j] = Z[i][j];
            }
        }
        __syncthreads();
    }
}


// Inertia (numbers of positive, negative and zero eigenvalues) of `batch` symmetric n x n matrices
// by Bunch-Kaufman symmetric indefinite elimination (LAPACK's pivoting, alpha = (1 + sqrt 17) / 8),
// Sylvester's law on the block-diagonal factor: a 1 x 1 pivot counts its sign, a 2 x 2 pivot by
// the signs of its determinant and trace.  IPOPT's inertia correction needs exactly these counts of
// the KKT matrix (MA27/MA57 report them); ipm.StructuredKKT adds them over the interval blocks and
// the separator pivot blocks (Haynsworth additivity).  A pivot with max(|a_kk|, colmax) <= ztol *
// max|A| counts as a zero eigenvalue and is skipped.
//
// One workgroup per matrix, in place on A[b] (row-major; the lower triangle is read, the matrix is
// destroyed).  Blocked with delayed updates (the scheme of LAPACK's dlasyf): a panel of up to nb
// pivot columns is eliminated keeping the trailing matrix un-updated in global memory; every column
// the pivot search needs (column k, and column imax when |a_kk| is small) is formed on the fly as
//     S(r, g) = A(r, g) - sum_c W(r, c) L(g, c),     W = L D (the panel's columns, LDS),
// interchanges are applied to the un-updated matrix and to the rows of W; after the panel one pass
// applies the rank-nb update A -= W D^-1 W^T to the trailing lower triangle.  The unblocked
// elimination (dsytf2) re-read and re-wrote the whole trailing triangle per pivot (n^3 / 3 doubles
// of global traffic; 7.4 ms for the dual-kite sweep's 640-row blocks); here that traffic falls by
// the panel width.  The lower triangle is first mirrored into the upper storage, so column c of the
// lower triangle is row c of the array: the column gathers, the interchanges of rows below the
// pivot and the trailing update (a wave per 4 columns, lanes over rows, W from LDS column-major)
// all touch contiguous memory.  tools/bk_blocked_model.py is a host model of exactly this scheme.
template <int NT = kThreads>
__device__ __forceinline__ void block_argmax(double& v, int& i, double* rv, int* ri, int tid) {
    // per wave: a DPP max of the values, then a DPP min of the indices of the lanes holding it
    // (the (value, lowest index) pair of a shuffle butterfly; v is never NaN here)
    const double mx = wave_max(v);
    i = wave_min_i32(v == mx ? i : 0x7fffffff);
    v = mx;
    if ((tid & 63) == 0) { rv[tid >> 6] = v; ri[tid >> 6] = i; }
    __syncthreads();
    v = rv[0];
    i = ri[0];
    for (int w = 1; w < NT / 64; ++w)
        if (rv[w] > v || (rv[w] == v && ri[w] < i)) { v = rv[w]; i = ri[w]; }
    __syncthreads();
}

// Small matrices (the separator pivot blocks, the MPC's 126-row interval blocks): the unblocked
// elimination (dsytf2) -- per pivot a column max, the interchange, and the trailing lower triangle
// updated one row per wave with lanes over the row's columns (row-major, coalesced).  Below ~200
// rows its per-pivot work is cheaper than the panel bookkeeping of the blocked kernel, and the
// trailing triangle is L2-resident.
template <int NT>
__global__ __launch_bounds__(NT) void sym_inertia_unblocked_kernel(int n, double* __restrict__ As, double ztol,
                                                                   int* __restrict__ counts) {
    extern __shared__ double pc[];                      // pivot columns: [2][n]
    __shared__ double rv[NT / 64];
    __shared__ int ri[NT / 64];
    double* A = As + (size_t)blockIdx.x * n * n;
    const int tid = threadIdx.x;
    const int wv = tid >> 6, ln = tid & 63;
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    auto L = [&](int i, int j) -> double& { return i >= j ? A[(size_t)i * n + j] : A[(size_t)j * n + i]; };
    // scale for the zero-pivot test
    double amax = 0.0;
    int dummy = 0;
    for (int t = tid; t < n * n; t += NT) {
        const int i = t / n, j = t - i * n;
        if (j <= i) amax = fmax(amax, fabs(A[t]));
    }
    block_argmax<NT>(amax, dummy, rv, ri, tid);
    const double zlim = ztol * amax;
    int pos = 0, neg = 0, zero = 0;                     // uniform across the workgroup
    int k = 0;
    while (k < n) {
        const double absakk = fabs(L(k, k));
        double colmax = 0.0;
        int imax = k;
        for (int i = k + 1 + tid; i < n; i += NT) {
            const double v = fabs(L(i, k));
            if (v > colmax) { colmax = v; imax = i; }
        }
        block_argmax<NT>(colmax, imax, rv, ri, tid);
        if (fmax(absakk, colmax) <= zlim) {             // zero column: a zero eigenvalue
            ++zero;
            ++k;
            continue;
        }
        int kp = k, kstep = 1;
        if (absakk < alpha * colmax) {
            double rowmax = 0.0;
            int jm = 0;
            for (int j = k + tid; j < n; j += NT)
                if (j != imax) {
                    const double v = fabs(L(imax, j));
                    if (v > rowmax) { rowmax = v; jm = j; }
                }
            block_argmax<NT>(rowmax, jm, rv, ri, tid);
            if (absakk >= alpha * colmax * (colmax / rowmax)) {
                kp = k;
            } else if (fabs(L(imax, imax)) >= alpha * rowmax) {
                kp = imax;
            } else {
                kp = imax;
                kstep = 2;
            }
            // every thread has read L(imax, imax) for the decision above before any thread's
            // interchange below writes it (without this barrier a late wave could decide on the
            // swapped value: the pivot choice, and with it the counts, then depended on timing)
            __syncthreads();
        }
        const int kk = k + kstep - 1;
        if (kp != kk) {                                  // symmetric interchange of kk and kp
            for (int i = kp + 1 + tid; i < n; i += NT) {
                const double a = A[(size_t)i * n + kk];
                A[(size_t)i * n + kk] = A[(size_t)i * n + kp];
                A[(size_t)i * n + kp] = a;
            }
            for (int j = kk + 1 + tid; j < kp; j += NT) {
                const double a = A[(size_t)j * n + kk];
                A[(size_t)j * n + kk] = A[(size_t)kp * n + j];
                A[(size_t)kp * n + j] = a;
            }
            if (tid == 0) {
                const double a = A[(size_t)kk * n + kk];
                A[(size_t)kk * n + kk] = A[(size_t)kp * n + kp];
                A[(size_t)kp * n + kp] = a;
                if (kstep == 2) {
                    const double b = A[(size_t)(k + 1) * n + k];
                    A[(size_t)(k + 1) * n + k] = A[(size_t)kp * n + k];
                    A[(size_t)kp * n + k] = b;
                }
            }
            __syncthreads();
        }
        // stage the pivot column(s) below the pivot block
        const int r0 = k + kstep;
        for (int i = r0 + tid; i < n; i += NT) {
            pc[i] = A[(size_t)i * n + k];
            if (kstep == 2) pc[n + i] = A[(size_t)i * n + k + 1];
        }
        const double d11 = A[(size_t)k * n + k];
        double d21 = 0.0, d22 = 0.0;
        if (kstep == 2) {
            d21 = A[(size_t)(k + 1) * n + k];
            d22 = A[(size_t)(k + 1) * n + k + 1];
        }
        __syncthreads();
        if (kstep == 1) {
            if (d11 > 0.0) ++pos; else if (d11 < 0.0) ++neg; else ++zero;
            const double rd = 1.0 / d11;
            for (int i = r0 + wv; i < n; i += NT / 64) {     // one row per wave, lanes over j <= i
                const double ci = pc[i] * rd;
                double* row = A + (size_t)i * n;
                for (int j = r0 + ln; j <= i; j += 64) row[j] -= ci * pc[j];
            }
        } else {
            const double det = d11 * d22 - d21 * d21;
            if (det < 0.0) { ++pos; ++neg; }
            else if (det > 0.0) { if (d11 + d22 > 0.0) pos += 2; else neg += 2; }
            else { ++zero; if (d11 + d22 > 0.0) ++pos; else if (d11 + d22 < 0.0) ++neg; else ++zero; }
            const double i11 = d22 / det, i22 = d11 / det, i21 = -d21 / det;   // D^-1
            for (int i = r0 + wv; i < n; i += NT / 64) {
                const double ai = pc[i], bi = pc[n + i];
                const double wi1 = i11 * ai + i21 * bi, wi2 = i21 * ai + i22 * bi;
                double* row = A + (size_t)i * n;
                for (int j = r0 + ln; j <= i; j += 64) row[j] -= wi1 * pc[j] + wi2 * pc[n + j];
            }
        }
        __syncthreads();
        k += kstep;
    }
    if (tid == 0) {
        counts[3 * blockIdx.x + 0] = pos;
        counts[3 * blockIdx.x + 1] = neg;
        counts[3 * blockIdx.x + 2] = zero;
    }
}

constexpr int kSyNB = 16;                                 // panel width (W columns in LDS)
constexpr size_t kSyLds = 150 * 1024;
constexpr int kSyBlockedMinN = 200;                      // blocked from here (tools/awelu_ab.py)

// Column g of the current Schur complement, rows [k, n), into W slot dst.  Storage: lower-triangle
// entry (r, c), r >= c, at A[c n + r].
__device__ __forceinline__ void bk_gather(const double* __restrict__ A, double* W, int n, int k, int g, int j,
                                          int dst, const double* ca, const double* cb, const int* cp, int tid) {
    double lg[kSyNB];                                     // L(g, c): wave-uniform
#pragma unroll
    for (int c = 0; c < kSyNB; ++c) lg[c] = c < j ? ca[c] * W[c * n + g] + cb[c] * W[cp[c] * n + g] : 0.0;
    constexpr int U = 4;                                  // the rows' global loads issued together
    for (int rb = k; rb < n; rb += U * kThreads) {        // uniform trip count
        const int r0 = rb + tid;
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = r0 + u * kThreads;
            v[u] = r < n ? (r >= g ? A[(size_t)g * n + r] : A[(size_t)r * n + g]) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = r0 + u * kThreads;
            if (r < n) {
#pragma unroll
                for (int c = 0; c < kSyNB; ++c)
                    if (c < j) v[u] -= W[c * n + r] * lg[c];
                W[dst * n + r] = v[u];
            }
        }
    }
}

__global__ __launch_bounds__(kThreads) void sym_inertia_kernel(int n, int nb, double* __restrict__ As, double ztol,
                                                               int* __restrict__ counts) {
    extern __shared__ double W[];                       // [nb][n], column-major panel W = L D
    __shared__ double rv[kThreads / 64];
    __shared__ int ri[kThreads / 64];
    __shared__ double ca[kSyNB], cb[kSyNB];              // L(s, c) = ca[c] W(s, c) + cb[c] W(s, cp[c])
    __shared__ int cp[kSyNB];
    double* A = As + (size_t)blockIdx.x * n * n;
    const int tid = threadIdx.x;
    const int wv = tid >> 6, ln = tid & 63;
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    // the lower triangle mirrored into the upper storage; its scale for the zero-pivot test
    double amax = 0.0;
    int dummy = 0;
    for (int t = tid; t < n * n; t += kThreads) {
        const int i = t / n, j = t - i * n;
        if (j <= i) {
            const double v = A[t];
            amax = fmax(amax, fabs(v));
            if (j < i) A[(size_t)j * n + i] = v;
        }
    }
    block_argmax(amax, dummy, rv, ri, tid);              // (its barriers also order the mirror)
    const double zlim = ztol * amax;
    int pos = 0, neg = 0, zero = 0;                     // uniform across the workgroup
    int k = 0;
    while (k < n) {
        int j = 0;                                      // panel columns used
        while (k < n && j < nb - 1) {                   // (a 2 x 2 pivot needs two free slots)
            bk_gather(A, W, n, k, k, j, j, ca, cb, cp, tid);
            __syncthreads();
            const double absakk = fabs(W[j * n + k]);
            double colmax = 0.0;
            int imax = k;
            for (int r = k + 1 + tid; r < n; r += kThreads) {
                const double v = fabs(W[j * n + r]);
                if (v > colmax) { colmax = v; imax = r; }
            }
            block_argmax(colmax, imax, rv, ri, tid);
            imax = __builtin_amdgcn_readfirstlane(imax);
            if (__builtin_amdgcn_readfirstlane(fmax(absakk, colmax) <= zlim)) {   // zero column: a zero eigenvalue
                ++zero;
                ++k;
                continue;
            }
            int kp = k, kstep = 1;
            if (__builtin_amdgcn_readfirstlane(absakk < alpha * colmax)) {
                bk_gather(A, W, n, k, imax, j, j + 1, ca, cb, cp, tid);
                __syncthreads();
                double rowmax = 0.0;
                int jm = 0;
                for (int r = k + tid; r < n; r += kThreads)
                    if (r != imax) {
                        const double v = fabs(W[(j + 1) * n + r]);
                        if (v > rowmax) { rowmax = v; jm = r; }
                    }
                block_argmax(rowmax, jm, rv, ri, tid);
                if (absakk >= alpha * colmax * (colmax / rowmax)) {
                    kp = k;
                } else if (fabs(W[(j + 1) * n + imax]) >= alpha * rowmax) {
                    kp = imax;
                } else {
                    kp = imax;
                    kstep = 2;
                }
                kp = __builtin_amdgcn_readfirstlane(kp);     // uniform by construction; made
                kstep = __builtin_amdgcn_readfirstlane(kstep);   // scalar for the compiler
                // every wave has read W(imax, j + 1) for the decision above before the 2 x 2
                // interchange below rewrites it (a late wave would otherwise decide on the swapped
                // value, and the waves could disagree on the pivot)
                __syncthreads();
            }
            const int kk = k + kstep - 1;
            if (kp != kk) {
                // symmetric interchange of kk and kp in the un-updated matrix ...
                for (int i = kp + 1 + tid; i < n; i += kThreads) {
                    const double a = A[(size_t)kk * n + i];
                    A[(size_t)kk * n + i] = A[(size_t)kp * n + i];
                    A[(size_t)kp * n + i] = a;
                }
                for (int jj = kk + 1 + tid; jj < kp; jj += kThreads) {
                    const double a = A[(size_t)kk * n + jj];
                    A[(size_t)kk * n + jj] = A[(size_t)jj * n + kp];
                    A[(size_t)jj * n + kp] = a;
                }
                if (tid == 0) {
                    const double a = A[(size_t)kk * n + kk];
                    A[(size_t)kk * n + kk] = A[(size_t)kp * n + kp];
                    A[(size_t)kp * n + kp] = a;
                }
                // ... in the rows of the panel's earlier columns ...
                for (int c = tid; c < j; c += kThreads) {
                    const double a = W[c * n + kk];
                    W[c * n + kk] = W[c * n + kp];
                    W[c * n + kp] = a;
                }
                // ... and in the pivot column(s) formed above
                if (kstep == 1) {                       // column imax becomes column k
                    for (int r = k + tid; r < n; r += kThreads)
                        W[j * n + r] = W[(j + 1) * n + (r == k ? kp : r == kp ? k : r)];
                } else if (tid < 2) {
                    const int sl = j + tid;
                    const double a = W[sl * n + kk];
                    W[sl * n + kk] = W[sl * n + kp];
                    W[sl * n + kp] = a;
                }
            }
            __syncthreads();
            const double d11 = W[j * n + k];
            if (kstep == 1) {
                if (d11 > 0.0) ++pos; else if (d11 < 0.0) ++neg; else ++zero;
                if (tid == 0) { ca[j] = 1.0 / d11; cb[j] = 0.0; cp[j] = j; }
            } else {
                const double d21 = W[j * n + k + 1], d22 = W[(j + 1) * n + k + 1];
                const double det = d11 * d22 - d21 * d21;
                if (det < 0.0) { ++pos; ++neg; }
                else if (det > 0.0) { if (d11 + d22 > 0.0) pos += 2; else neg += 2; }
                else { ++zero; if (d11 + d22 > 0.0) ++pos; else if (d11 + d22 < 0.0) ++neg; else ++zero; }
                if (tid == 0) {                         // D^-1 = [d22, -d21; -d21, d11] / det
                    ca[j] = d22 / det; cb[j] = -d21 / det; cp[j] = j + 1;
                    ca[j + 1] = d11 / det; cb[j + 1] = -d21 / det; cp[j + 1] = j;
                }
            }
            __syncthreads();
            j += kstep;
            k += kstep;
        }
        if (k < n && j > 0) {
            // trailing update A(r, s) -= sum_c L(s, c) W(r, c), k <= s <= r: a wave takes 4 columns,
            // their L rows in registers, lanes over r (one LDS read of W(r, c) feeds 4 columns)
            constexpr int kCB = 4;
            for (int s0 = k + kCB * wv; s0 < n; s0 += kCB * (kThreads / 64)) {
                double ls[kCB][kSyNB];
#pragma unroll
                for (int q = 0; q < kCB; ++q) {
                    const int s = min(s0 + q, n - 1);
#pragma unroll
                    for (int c = 0; c < kSyNB; ++c)
                        ls[q][c] = c < j ? ca[c] * W[c * n + s] + cb[c] * W[cp[c] * n + s] : 0.0;
                }
                for (int rb = s0; rb < n; rb += 64) {             // wave-uniform trip count
                    const int r = rb + ln;
                    const bool in = r < n;
                    double acc[kCB];
#pragma unroll
                    for (int q = 0; q < kCB; ++q) acc[q] = (in && s0 + q <= r) ? A[(size_t)(s0 + q) * n + r] : 0.0;
                    const int rr = in ? r : n - 1;
#pragma unroll
                    for (int c = 0; c < kSyNB; ++c) {
                        if (c < j) {
                            const double w = W[c * n + rr];
#pragma unroll
                            for (int q = 0; q < kCB; ++q) acc[q] -= ls[q][c] * w;
                        }
                    }
#pragma unroll
                    for (int q = 0; q < kCB; ++q)
                        if (in && s0 + q <= r) A[(size_t)(s0 + q) * n + r] = acc[q];
                }
            }
            __syncthreads();
        }
    }
    if (tid == 0) {
        counts[3 * blockIdx.x + 0] = pos;
        counts[3 * blockIdx.x + 1] = neg;
        counts[3 * blockIdx.x + 2] = zero;
    }
}

}  // namespace

// Fixed-order gather-sums of ipm._ScatterSum (the KKT assembly, the KKT and Jacobian products):
// out[r][dst[u]] += sum over the source list of destination u of v(r, s), v = vals[r][s] or
// vals[r][s] * x[r][cols[s]].  The lists are padded to a power-of-two width w <= 64 and laid out
// in lanes, each list on w consecutive lanes aligned to w (widest first), so one butterfly of
// shuffles with offsets 1, 2, .., w / 2 adds every list as the adjacent-pair tree
// ((v0 + v1) + (v2 + v3)) + ..: the order torch's sum over a row of <= 64 float64 entries uses on
// this GPU (tools/torch_sum_order_probe.py), so this one launch returns bitwise what the gather /
// sum / index-put chain it replaces returned (tests/test_gather_sum_gpu.py).  No contraction: the
// product and the sums round as the separate torch operations did.
__global__ __launch_bounds__(256) void gather_sum_kernel(int L, const int* __restrict__ lsrc,
                                                         const unsigned char* __restrict__ lw,
                                                         const int* __restrict__ ldst, const double* __restrict__ vals,
                                                         long long ldv, const double* __restrict__ x,
                                                         const int* __restrict__ cols, long long ldx,
                                                         double* __restrict__ out, long long ldo) {
#pragma clang fp contract(off)
    const int l = blockIdx.x * 256 + threadIdx.x;
    const long long r = blockIdx.y;
    const int li = l < L ? l : L - 1;                         // every lane takes part in the shuffles
    const int s = lsrc[li];
    const int w = lw[li];
    double v = 0.0;
    if (l < L && s >= 0) {
        v = vals[r * ldv + s];
        if (x) v = v * x[r * ldx + cols[s]];
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_xor(v, o);
        if (o < w) v = v + u;
    }
    const int d = ldst[li];
    if (l < L && d >= 0) out[r * ldo + d] = out[r * ldo + d] + v;
}

// The lists wider than 64 of the same gather-sums (the few long destination lists, e.g. t_f's
// column of J): one workgroup per (list, row), the list's sources summed in awelu_row_sum's order over
// its power-of-two width (thread t adds entries t, t + 256, .. from 0.0, padding entries as 0.0, then
// the adjacent-pair tree), then added to the destination -- bitwise what ipm._ScatterSum's torch path
// (gather, det.row_sum, indexed add) computes, in one launch for all wide lists.
__global__ __launch_bounds__(256) void gather_sum_wide_kernel(const int* __restrict__ wsrc, const int* __restrict__ woff,
                                                              const int* __restrict__ ww, const int* __restrict__ wdst,
                                                              const double* __restrict__ vals, long long ldv,
                                                              const double* __restrict__ x, const int* __restrict__ cols,
                                                              long long ldx, double* __restrict__ out, long long ldo) {
#pragma clang fp contract(off)
    __shared__ double part[4];
    const int l = blockIdx.x, t = threadIdx.x;
    const long long r = blockIdx.y;
    const int* src = wsrc + woff[l];
    const int W = ww[l];
    double acc = 0.0;
    for (int j = t; j < W; j += 256) {
        const int sj = src[j];
        double v = 0.0;
        if (sj >= 0) {
            v = vals[r * ldv + sj];
            if (x) v = v * x[r * ldx + cols[sj]];
        }
        acc = acc + v;
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) acc = acc + __shfl_xor(acc, o);
    if ((t & 63) == 0) part[t >> 6] = acc;
    __syncthreads();
    if (t == 0) {
        const double sum = (part[0] + part[1]) + (part[2] + part[3]);
        double* o = out + r * ldo + wdst[l];
        *o = *o + sum;
    }
}

// ---- Batch-invariant reductions and products (awebox_amd/det.py) --------------------------------
// The interior-point solver's per-instance algebra on [B, n] tensors must round the same way
// whatever B is: a problem solved alone and the same problem inside a batch of 128 (or inside a
// sweep shard of 8, 4, 2 or 1 points) must follow the same iterates.  torch's
// row reductions pick a strategy by the tensor's shape, and rocBLAS picks a GEMM kernel by the batch
// count, so their last bits change with B.  These kernels fix one order per output that depends only
// on the row length (row_sum) or the inner dimension (bmm), never on the number of rows or matrices,
// and that det.py restates with elementwise torch operations on any device (the CPU harness and the
// bitwise tests).

// out[r] = sum_j x[r * ldx + j], j < n: thread t (of 256) adds x[t], x[t + 256], ... in sequence from
// 0.0; the 256 partial sums are then added as the adjacent-pair tree ((p0 + p1) + (p2 + p3)) + ..
// (xor butterfly inside each wave, the four wave sums through LDS).
constexpr int kRowSumThreads = 256;

__global__ __launch_bounds__(kRowSumThreads) void row_sum_kernel(long long n, const double* __restrict__ x,
                                                                 long long ldx, double* __restrict__ out) {
    __shared__ double part[kRowSumThreads / 64];
    const long long r = blockIdx.x;
    const int t = threadIdx.x;
    const double* xr = x + r * ldx;
    double acc = 0.0;
    long long j = t;
    // four independent loads in flight per step; the additions stay in sequence
    for (; j + 3 * kRowSumThreads < n; j += 4 * kRowSumThreads) {
        const double a = xr[j], b = xr[j + kRowSumThreads], c = xr[j + 2 * kRowSumThreads],
                     d = xr[j + 3 * kRowSumThreads];
        acc = acc + a;
        acc = acc + b;
        acc = acc + c;
        acc = acc + d;
    }
    for (; j < n; j += kRowSumThreads) acc = acc + xr[j];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) acc = acc + __shfl_xor(acc, o);
    if ((t & 63) == 0) part[t >> 6] = acc;
    __syncthreads();
    if (t == 0) out[r] = (part[0] + part[1]) + (part[2] + part[3]);
}

// C[b] = A[b] B[b] (M x K times K x N), strided operands (a transposed view is a pair of strides):
// every output entry is acc = 0; acc = acc + a_ik b_kj for k = 0, 1, .., K - 1, product and sum
// rounded separately (no contraction), so the bits do not depend on the tile shape chosen below or
// on the batch.  Workgroup: a TM x TN output tile (TY x TX threads, RM x RN entries each) of one
// matrix; the K dimension streams through LDS in chunks of KC.
template <int TX, int TY, int RM, int RN, int KC>
__global__ __launch_bounds__(TX * TY) void bmm_kernel(int M, int N, int K, const double* __restrict__ A, long long sAb,
                                                      long long sAm, long long sAk, const double* __restrict__ Bm,
                                                      long long sBb, long long sBk, long long sBn,
                                                      double* __restrict__ C, long long sCb, long long sCm,
                                                      long long sCn, int tiles_n) {
#pragma clang fp contract(off)
    constexpr int NT = TX * TY, TM = TY * RM, TN = TX * RN;
    __shared__ double As[KC][TM + 1];
    __shared__ double Bs[KC][TN + 1];
    const long long b = blockIdx.x;
    const int tm = blockIdx.y / tiles_n, tn = blockIdx.y % tiles_n;
    const int m0 = tm * TM, n0 = tn * TN;
    const double* Ab = A + b * sAb;
    const double* Bb = Bm + b * sBb;
    const int tid = threadIdx.x, tx = tid % TX, ty = tid / TX;
    double acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = 0.0;
    const bool a_mfast = sAm == 1;                       // load A along its contiguous dimension
    const bool b_nfast = sBn == 1;
    for (int k0 = 0; k0 < K; k0 += KC) {
        for (int e = tid; e < TM * KC; e += NT) {
            const int mm = a_mfast ? e % TM : e / KC, kk = a_mfast ? e / TM : e % KC;
            const int gm = m0 + mm, gk = k0 + kk;
            As[kk][mm] = (gm < M && gk < K) ? Ab[gm * sAm + gk * sAk] : 0.0;
        }
        for (int e = tid; e < TN * KC; e += NT) {
            const int nn = b_nfast ? e % TN : e / KC, kk = b_nfast ? e / TN : e % KC;
            const int gn = n0 + nn, gk = k0 + kk;
            Bs[kk][nn] = (gn < N && gk < K) ? Bb[gk * sBk + gn * sBn] : 0.0;
        }
        __syncthreads();
        const int kc = min(KC, K - k0);                  // padded k would add 0 * 0 = +0: skipped
        for (int kk = 0; kk < kc; ++kk) {
            double a[RM], bv[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i) a[i] = As[kk][ty + i * TY];
#pragma unroll
            for (int j = 0; j < RN; ++j) bv[j] = Bs[kk][tx + j * TX];
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j) acc[i][j] = acc[i][j] + a[i] * bv[j];
        }
        __syncthreads();
    }
    double* Cb = C + b * sCb;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
            const int gm = m0 + ty + i * TY, gn = n0 + tx + j * TX;
            if (gm < M && gn < N) Cb[gm * sCm + gn * sCn] = acc[i][j];
        }
}

// ---- Interior-point measures (awebox_amd/ipm.py, solve_batch) -------------------------------------
// One workgroup per instance computes, in one pass over its vectors, what the solver's loop head and
// line search otherwise assemble from ~130 torch operations per iteration: IPOPT's scaled optimality
// error and its parts (dual, primal, complementarity; the unscaled tests; the barrier problem's error
// at the current mu) and the merit pair theta = ||c||_1, phi = the barrier function.  Every value is
// the torch composition's (ipm.errors_torch / ipm.barrier_phi_torch): the same operations per entry,
// rounded separately (no contraction), each sum in row_sum_kernel's order (thread t adds entries t,
// t + 256, .. from 0.0, then the adjacent-pair tree), maxima with NaN propagation like torch's amax,
// a division by a host scalar as torch performs it (a product with the host reciprocal).
constexpr int kIpmThreads = 256;

__device__ __forceinline__ double nan_max(double a, double b) { return (a != a || a > b) ? a : b; }
__device__ __forceinline__ double clamp_lo(double v, double lo) { return (v != v) ? v : (v < lo ? lo : v); }

__global__ __launch_bounds__(kIpmThreads) void ipm_measures_kernel(AweluIpmMeasures a) {
#pragma clang fp contract(off)
    constexpr int NW = kIpmThreads / 64;
    __shared__ double part[16][NW];
    const int b = blockIdx.x, t = threadIdx.x;
    const size_t oy = (size_t)b * a.ny, om = (size_t)b * a.m, oi = (size_t)b * a.mI, on = (size_t)b * a.n;
    const bool head = a.mode == 0;
    const double mu_h = a.mu[b];
    const double kd_mu = mu_h * a.kappa_d;
    // sums: 0 |zl|, 1 |zu|, 2 log gaps (lower), 3 (upper), 4 lower-only gaps, 5 upper-only gaps, 6 |c|,
    // 7 |lam|; maxima: 0 |dual|, 1 |damped dual|, 2 |compl| at mu_target, 3 at mu, 4 unscaled |dual|,
    // 5 |c|, 6 unscaled equality |c|, 7 inequality-row bound violation
    double s[8], mx[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) s[q] = mx[q] = 0.0;
    for (int i = t; i < a.ny; i += kIpmThreads) {
        const double yv = a.y[oy + i];
        const bool hl = a.hl[oy + i] != 0, hu = a.hu[oy + i] != 0;
        const double dl = hl ? yv - a.yl[oy + i] : 1.0;
        const double du = hu ? a.yu[oy + i] - yv : 1.0;
        const double lo = a.lo_only[i], hi = a.hi_only[i];
        s[2] = s[2] + (hl ? log(dl) : 0.0);
        s[3] = s[3] + (hu ? log(du) : 0.0);
        s[4] = s[4] + lo * dl;
        s[5] = s[5] + hi * du;
        if (head) {
            const double zl = a.zl[oy + i], zu = a.zu[oy + i];
            s[0] = s[0] + fabs(zl);
            s[1] = s[1] + fabs(zu);
            const double r = a.jt_lam[oy + i];
            const double g = i < a.n ? a.grad[on + i] + r : 0.0 + (r - a.lam[om + a.ineq[i - a.n]]);
            const double d = (g - zl) + zu;
            const double dd = d + kd_mu * (lo - hi);
            mx[0] = nan_max(mx[0], fabs(d));
            mx[1] = nan_max(mx[1], fabs(dd));
            const double clt = hl ? dl * zl - a.mu_target : 0.0, cut = hu ? du * zu - a.mu_target : 0.0;
            const double clh = hl ? dl * zl - mu_h : 0.0, cuh = hu ? du * zu - mu_h : 0.0;
            mx[2] = nan_max(mx[2], nan_max(fabs(clt), fabs(cut)));
            mx[3] = nan_max(mx[3], nan_max(fabs(clh), fabs(cuh)));
            mx[4] = nan_max(mx[4], i < a.n ? fabs(d) : fabs(d * a.cs_slack[oi + (i - a.n)]));
        }
    }
    for (int j = t; j < a.m; j += kIpmThreads) {
        const double cj = a.c[om + j];
        s[6] = s[6] + fabs(cj);
        mx[5] = nan_max(mx[5], fabs(cj));
        if (head) {
            s[7] = s[7] + fabs(a.lam[om + j]);
            mx[6] = nan_max(mx[6], a.eq_row[j] ? fabs(cj / a.c_scale[om + j]) : 0.0);
        }
    }
    if (head)
        for (int k = t; k < a.mI; k += kIpmThreads) {
            const double gI = (a.c[om + a.ineq[k]] + a.y[oy + a.n + k]) / a.cs_slack[oi + k];
            const double gu = a.gu0[k], gl = a.gl0[k];
            const double v = nan_max(isfinite(gu) ? gI - gu : 0.0, isfinite(gl) ? gl - gI : 0.0);
            mx[7] = nan_max(mx[7], clamp_lo(v, 0.0));
        }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        double v = s[q], w = mx[q];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            v = v + __shfl_xor(v, o);
            w = nan_max(w, __shfl_xor(w, o));
        }
        if ((t & 63) == 0) {
            part[q][t >> 6] = v;
            part[8 + q][t >> 6] = w;
        }
    }
    __syncthreads();
    if (t != 0) return;
    double S[8], A[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        S[q] = (part[q][0] + part[q][1]) + (part[q][2] + part[q][3]);
        A[q] = nan_max(nan_max(part[8 + q][0], part[8 + q][1]), nan_max(part[8 + q][2], part[8 + q][3]));
    }
    const double theta = S[6];
    const double phi = (a.f[b] - mu_h * (S[2] + S[3])) + kd_mu * (S[4] + S[5]);
    double* out = a.out + b;
    const long long B = a.B;
    if (!head) {
        out[0] = theta;
        out[B] = phi;
        return;
    }
    const double zsum = S[0] + S[1];
    const double s_d = clamp_lo((S[7] + zsum) * a.inv_mnb, a.s_max) * a.inv_smax;
    const double s_c = clamp_lo(zsum * a.inv_nb, a.s_max) * a.inv_smax;
    const double e_pr = A[5];
    const double e_d = A[0] / s_d, e_c = A[2] / s_c;
    const double osc = a.obj_scale[b];
    out[0] = nan_max(nan_max(e_d, e_pr), e_c);
    out[B] = e_d;
    out[2 * B] = e_pr;
    out[3 * B] = e_c;
    out[4 * B] = A[4] / osc;
    out[5 * B] = nan_max(A[6], A[7]);
    out[6 * B] = A[2] / osc;
    out[7 * B] = nan_max(nan_max(A[1] / s_d, e_pr), A[3] / s_c);
    out[8 * B] = theta;
    out[9 * B] = phi;
}

// The Newton system's vectors at an iterate (ipm.solve_batch, before the factorisation): the bound
// gaps dl, du, the barrier diagonal Sigma, grad phi and the right-hand side [-(grad phi + A^T lam); -c],
// every entry as the torch composition computes it (Measures.newton_torch).  A thread per entry of
// [ny | m] and instance.
__global__ __launch_bounds__(256) void ipm_newton_kernel(AweluIpmNewton a) {
#pragma clang fp contract(off)
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.ny + a.m) return;
    const size_t oy = (size_t)b * a.ny;
    if (i >= a.ny) {
        const int j = i - a.ny;
        a.rhs[(size_t)b * (a.ny + a.m) + a.ny + j] = -a.c[(size_t)b * a.m + j];
        return;
    }
    const double mu = a.mu[b];
    const double yv = a.y[oy + i];
    const bool hl = a.hl[oy + i] != 0, hu = a.hu[oy + i] != 0;
    const double dl = hl ? yv - a.yl[oy + i] : 1.0;
    const double du = hu ? a.yu[oy + i] - yv : 1.0;
    const double sig = (hl ? a.zl[oy + i] / dl : 0.0) + (hu ? a.zu[oy + i] / du : 0.0);
    const double g = i < a.n ? a.grad[(size_t)b * a.n + i] : 0.0;
    const double gp = ((g - (hl ? mu / dl : 0.0)) + (hu ? mu / du : 0.0)) + (mu * a.kappa_d) * (a.lo_only[i] - a.hi_only[i]);
    const double r = a.jt_lam[oy + i];
    const double at = i < a.n ? r : r - a.lam[(size_t)b * a.m + a.ineq[i - a.n]];
    a.dl[oy + i] = dl;
    a.du[oy + i] = du;
    a.sigma[oy + i] = sig;
    a.grad_phi[oy + i] = gp;
    a.rhs[(size_t)b * (a.ny + a.m) + i] = -(gp + at);
}

__device__ __forceinline__ double nan_min(double a, double b) { return (a != a || a < b) ? a : b; }

// The accepted step (ipm.solve_batch after the line search): the bound multipliers' Newton step
// dz = mu / gap - z -/+ z / gap dy at the Newton system's gaps (dl_old, du_old), its fraction-to-the-boundary length
// alpha_z = min(1, min -tau z / dz) (a workgroup per instance: first pass and a block minimum), then
// y <- y_new where accepted, lam += alpha dlam, z += alpha_z dz, and IPOPT's kappa_sigma safeguard
// z <- clamp(z, mu / (kappa_sigma gap), kappa_sigma mu / gap) at the new gaps; every entry as the
// torch composition (Measures.step_torch).  any_acc = 0: no instance stepped (only the safeguard).
__global__ __launch_bounds__(kIpmThreads) void ipm_step_kernel(AweluIpmStep a) {
#pragma clang fp contract(off)
    constexpr int NW = kIpmThreads / 64;
    __shared__ double part[NW];
    const int b = blockIdx.x, t = threadIdx.x;
    const size_t oy = (size_t)b * a.ny;
    const double mu = a.mu[b];
    const bool acc = a.acc[b] != 0;
    double az = 0.0;
    if (a.any_acc) {
        const double tau = a.tau[b];
        double mn = INFINITY;
        for (int i = t; i < a.ny; i += kIpmThreads) {
            const bool hl = a.hl[oy + i] != 0, hu = a.hu[oy + i] != 0;
            const double dl = a.dl_old[oy + i], du = a.du_old[oy + i];
            const double zl = a.zl[oy + i], zu = a.zu[oy + i], dy = a.dy[oy + i];
            const double dzl = hl ? (mu / dl - zl) - (zl / dl) * dy : 0.0;
            const double dzu = hu ? (mu / du - zu) + (zu / du) * dy : 0.0;
            mn = nan_min(mn, (hl && dzl < 0.0) ? (-tau * zl) / dzl : INFINITY);
            mn = nan_min(mn, (hu && dzu < 0.0) ? (-tau * zu) / dzu : INFINITY);
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) mn = nan_min(mn, __shfl_xor(mn, o));
        if ((t & 63) == 0) part[t >> 6] = mn;
        __syncthreads();
        mn = part[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) mn = nan_min(mn, part[w]);
        const double az_b = nan_min(mn, 1.0);
        az = acc ? az_b : 0.0;
        if (t == 0) a.alpha_z[b] = az_b;
    } else if (t == 0) {
        a.alpha_z[b] = 0.0;
    }
    const double al = acc ? a.alpha[b] : 0.0;
    for (int i = t; i < a.ny; i += kIpmThreads) {
        const double yold = a.y[oy + i];
        const bool hl = a.hl[oy + i] != 0, hu = a.hu[oy + i] != 0;
        double zl = a.zl[oy + i], zu = a.zu[oy + i], yv = yold;
        if (a.any_acc) {
            const double dl = a.dl_old[oy + i], du = a.du_old[oy + i];
            const double dy = a.dy[oy + i];
            const double dzl = hl ? (mu / dl - zl) - (zl / dl) * dy : 0.0;
            const double dzu = hu ? (mu / du - zu) + (zu / du) * dy : 0.0;
            yv = acc ? a.y_new[oy + i] : yold;
            zl = zl + az * dzl;
            zu = zu + az * dzu;
        }
        const double dl = hl ? yv - a.yl[oy + i] : 1.0;
        const double du = hu ? a.yu[oy + i] - yv : 1.0;
        const double ks_mu = mu * a.kappa_sigma;
        if (hl) zl = (zl != zl) ? zl : fmin(fmax(zl, mu / (dl * a.kappa_sigma)), ks_mu / dl);
        if (hu) zu = (zu != zu) ? zu : fmin(fmax(zu, mu / (du * a.kappa_sigma)), ks_mu / du);
        a.y_out[oy + i] = yv;
        a.zl_out[oy + i] = zl;
        a.zu_out[oy + i] = zu;
    }
    if (a.any_acc)
        for (int j = t; j < a.m; j += kIpmThreads) {
            const size_t k = (size_t)b * a.m + j;
            a.lam_out[k] = a.lam[k] + al * a.dlam[k];
        }
}

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
    // small blocks in large batches (the MPC's 1,280 interval blocks of 126 rows): two waves per
    // matrix keep every block resident at once (8 workgroups per CU instead of 4: one round of the
    // grid instead of two); the factors are the same bits (per entry the same operations)
    if (n <= kLuSmallN && batch >= kLuSmallMinBatch)
        lu_batched_kernel<128><<<dim3((unsigned)batch), 128, lds, (hipStream_t)stream>>>(n, A, piv);
    else
        lu_batched_kernel<kThreads><<<dim3((unsigned)batch), kThreads, lds, (hipStream_t)stream>>>(n, A, piv);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// X <- A^-1 X for `batch` systems with the factors (LU, piv) of awelu_factor_batched; X[b][n][nrhs]
// row-major (device pointer), solved in place.  Asynchronous on `stream`.
int awelu_solve_batched(int n, int nrhs, int batch, const double* LU, const int* piv, double* X, void* stream) {
    if (n < 1 || n > kMaxN || nrhs < 1 || batch < 1 || !LU || !piv || !X) {
        g_err = "need 1 <= n <= 1024, nrhs >= 1, batch >= 1 and device pointers";
        return 1;
    }
    const long cap = (long)(kSolveLds / sizeof(double)) / n - kNB;   // right-hand sides per pass
    if (cap < 1) {
        g_err = "n too large for the LDS-resident solve";
        return 1;
    }
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)lu_solve_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSolveLds);
        attr = true;
    }
    // one workgroup per (matrix, chunk of right-hand sides), all in one launch: enough
    // workgroups to fill the CUs for small batches (>= 16 columns per chunk: every chunk streams
    // the whole factor), at most `cap` columns (LDS)
    const long want = std::max<long>(1, (kSolveTargetWgs + batch - 1) / batch);
    long w = std::max<long>(kSolveMinChunk, (nrhs + want - 1) / want);
    w = std::min<long>(w, cap);
    const long nchunks = (nrhs + w - 1) / w;
    w = (nrhs + nchunks - 1) / nchunks;                   // balanced chunk widths
    const size_t lds = sizeof(double) * (size_t)n * (kNB + w);
    lu_solve_kernel<<<dim3((unsigned)batch, (unsigned)nchunks), kThreads, lds, (hipStream_t)stream>>>(n, nrhs, (int)w, LU,
                                                                                                     piv, X);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// Block-tridiagonal factorisation: T[b][nb][3][m][m] (sub-, main, super-diagonal block of each
// block row; the sub-diagonal block of row 0 and the super-diagonal block of row nb-1 are
// ignored), m <= 48.  In place: the super-diagonal blocks become W_k = D'_k^-1 U_k; Dinv[b][nb][m][m]
// receives the inverted pivot blocks D'_k^-1.
int awelu_btd_factor_batched(int nb, int m, int batch, double* T, double* Dinv, void* stream) {
    if (nb < 1 || m < 1 || m > kBtdMaxM || batch < 1 || !T || !Dinv) {
        g_err = "need nb >= 1, 1 <= m <= 48, batch >= 1 and device pointers";
        return 1;
    }
    btd_factor_kernel<kThreads, kBtdMaxM><<<dim3((unsigned)batch), kThreads, 0, (hipStream_t)stream>>>(nb, m, T, Dinv);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// X[b] <- T[b]^-1 X[b] with the factors of awelu_btd_factor_batched; X[b][nb m][nrhs] row-major,
// solved in place (64 right-hand sides per pass).
int awelu_btd_solve_batched(int nb, int m, int nrhs, int batch, const double* T, const double* Dinv, double* X,
                            void* stream) {
    if (nb < 1 || m < 1 || m > kBtdMaxM || nrhs < 1 || batch < 1 || !T || !Dinv || !X) {
        g_err = "need nb >= 1, 1 <= m <= 48, nrhs >= 1, batch >= 1 and device pointers";
        return 1;
    }
    // the columns are independent chains: split them over enough workgroups to occupy the chip when
    // the batch is small (the AP2 factorisation's T^-1 E, 24 columns of one chain, ran as one
    // workgroup: 1.2 ms, against 0.47 ms for a single column)
    const int chunks = std::min(nrhs, std::max((nrhs + kBtdMaxRhs - 1) / kBtdMaxRhs, (256 + batch - 1) / batch));
    const int w = (nrhs + chunks - 1) / chunks;
    const int launched = (nrhs + w - 1) / w;
    if (launched > 65535) {
        g_err = "too many right-hand-side chunks";
        return 1;
    }
    btd_apply_kernel<kThreads, kBtdMaxM><<<dim3((unsigned)batch, (unsigned)launched), kThreads, 0, (hipStream_t)stream>>>(
        nb, m, nrhs, 0, w, T, Dinv, X);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// Inertia of `batch` symmetric n x n matrices A[b][n][n] (lower triangle read, A destroyed):
// counts[b][3] = (positive, negative, zero) eigenvalue counts.  Asynchronous on `stream`.
int awelu_sym_inertia_batched(int n, int batch, double* A, double ztol, int* counts, void* stream) {
    const int nb = std::min<long>(kSyNB, (long)(kSyLds / sizeof(double)) / std::max(n, 1));
    if (n < 1 || nb < 4 || batch < 1 || !A || !counts) {
        g_err = "need 1 <= n <= 4800 (a panel of >= 4 columns in LDS), batch >= 1 and device pointers";
        return 1;
    }
    static bool attr = false;
    if (!attr) {
        hipFuncSetAttribute((const void*)sym_inertia_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSyLds);
        attr = true;
    }
    // (a <128> instantiation, two waves per matrix as in lu_batched_kernel, measured slower on the
    // MPC's 1,280 x 126: 1.66 vs 1.27 ms; profiles/r05/solver/mpc_check/ab.log)
    if (n < kSyBlockedMinN)
        sym_inertia_unblocked_kernel<kThreads><<<dim3((unsigned)batch), kThreads, sizeof(double) * 2 * (size_t)n,
                                                 (hipStream_t)stream>>>(n, A, ztol, counts);
    else
        sym_inertia_kernel<<<dim3((unsigned)batch), kThreads, sizeof(double) * (size_t)nb * n, (hipStream_t)stream>>>(
            n, nb, A, ztol, counts);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// Gather-sums for `rows` rows (see gather_sum_kernel): L lanes of (source, width, destination);
// x and cols NULL for plain sums.  Asynchronous on `stream`.
int awelu_gather_sum(int L, int rows, const int* lsrc, const unsigned char* lw, const int* ldst, const double* vals,
                     long long ldv, const double* x, const int* cols, long long ldx, double* out, long long ldo,
                     void* stream) {
    if (L < 0 || rows < 0 || rows > 65535 || (L > 0 && (!lsrc || !lw || !ldst || !vals || !out)) || (x && !cols)) {
        g_err = "need L >= 0, 0 <= rows <= 65535 and device pointers (cols with x)";
        return 1;
    }
    if (L == 0 || rows == 0) return 0;
    gather_sum_kernel<<<dim3((unsigned)((L + 255) / 256), (unsigned)rows), 256, 0, (hipStream_t)stream>>>(
        L, lsrc, lw, ldst, vals, ldv, x, cols, ldx, out, ldo);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// out[r] = sum of x[r][0 .. n) in row_sum_kernel's fixed order, r < rows (x row stride ldx >= n).
int awelu_row_sum(long long rows, long long n, const double* x, long long ldx, double* out, void* stream) {
    if (rows < 0 || rows > 0x7fffffffLL || n < 0 || ldx < n || (rows > 0 && (!x || !out))) {
        g_err = "need 0 <= rows < 2^31, n >= 0, ldx >= n and device pointers";
        return 1;
    }
    if (rows == 0) return 0;
    row_sum_kernel<<<dim3((unsigned)rows), kRowSumThreads, 0, (hipStream_t)stream>>>(n, x, ldx, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// C[b] = A[b] B[b] for b < batch: M x K times K x N with element strides (sAm, sAk), (sBk, sBn),
// (sCm, sCn) and batch strides sAb, sBb, sCb (a transposed operand is a swapped stride pair).  C must
// not overlap A or B.  Every entry is summed over k in sequence (bmm_kernel): the result is the same
// for every batch and every tile shape.
int awelu_bmm(int batch, int M, int N, int K, const double* A, long long sAb, long long sAm, long long sAk,
              const double* B, long long sBb, long long sBk, long long sBn, double* C, long long sCb, long long sCm,
              long long sCn, void* stream) {
    if (batch < 0 || M < 0 || N < 0 || K < 0 || (batch > 0 && M > 0 && N > 0 && (!A || !B || !C))) {
        g_err = "need non-negative sizes and device pointers";
        return 1;
    }
    if (batch == 0 || M == 0 || N == 0) return 0;
    const hipStream_t s = (hipStream_t)stream;
    // the tile shape follows the output's shape only (never the batch): wide outputs 64 x 64
    // (4 x 4 per thread), narrow ones 128 x 8 (2 x 2), single columns 256 x 1
    auto tiles = [](int total, int t) { return (total + t - 1) / t; };
    long long grid_y;
    if (N >= 24) {
        const int tn = tiles(N, 64);
        grid_y = (long long)tiles(M, 64) * tn;
        if (grid_y <= 65535)
            bmm_kernel<16, 16, 4, 4, 16><<<dim3((unsigned)batch, (unsigned)grid_y), 256, 0, s>>>(
                M, N, K, A, sAb, sAm, sAk, B, sBb, sBk, sBn, C, sCb, sCm, sCn, tn);
    } else if (N > 1) {
        const int tn = tiles(N, 8);
        grid_y = (long long)tiles(M, 128) * tn;
        if (grid_y <= 65535)
            bmm_kernel<4, 64, 2, 2, 16><<<dim3((unsigned)batch, (unsigned)grid_y), 256, 0, s>>>(
                M, N, K, A, sAb, sAm, sAk, B, sBb, sBk, sBn, C, sCb, sCm, sCn, tn);
    } else {
        grid_y = tiles(M, 256);
        if (grid_y <= 65535)
            bmm_kernel<1, 256, 1, 1, 32><<<dim3((unsigned)batch, (unsigned)grid_y), 256, 0, s>>>(
                M, N, K, A, sAb, sAm, sAk, B, sBb, sBk, sBn, C, sCb, sCm, sCn, 1);
    }
    if (grid_y > 65535) {
        g_err = "output too large for one launch";
        return 1;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// The interior-point measures (ipm_measures_kernel) of a->B instances: a->mode 0 writes the loop
// head's ten rows out[row][b], mode 1 the merit pair (theta, phi).
int awelu_ipm_measures(const AweluIpmMeasures* a, void* stream) {
    if (!a || a->B < 0 || a->ny < 0 || a->n < 0 || a->n > a->ny || a->m < 0 || a->mI < 0 ||
        a->n + a->mI != a->ny || (a->mode != 0 && a->mode != 1) || !a->out || !a->y || !a->yl || !a->yu ||
        !a->hl || !a->hu || !a->lo_only || !a->hi_only || !a->f || !a->mu || (a->m > 0 && !a->c)) {
        g_err = "awelu_ipm_measures: need ny = n + mI, mode 0 or 1 and device pointers";
        return 1;
    }
    if (a->mode == 0 && (!a->grad || !a->jt_lam || !a->zl || !a->zu || !a->obj_scale ||
                         (a->m > 0 && (!a->lam || !a->c_scale || !a->eq_row)) ||
                         (a->mI > 0 && (!a->ineq || !a->cs_slack || !a->gl0 || !a->gu0)))) {
        g_err = "awelu_ipm_measures: mode 0 needs the gradient, J^T lam, multipliers and scalings";
        return 1;
    }
    if (a->B == 0) return 0;
    ipm_measures_kernel<<<dim3((unsigned)a->B), kIpmThreads, 0, (hipStream_t)stream>>>(*a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// The Newton system's vectors (ipm_newton_kernel) of a->B instances.
int awelu_ipm_newton(const AweluIpmNewton* a, void* stream) {
    if (!a || a->B < 0 || a->B > 65535 || a->n < 0 || a->mI < 0 || a->m < 0 || a->ny != a->n + a->mI ||
        !a->y || !a->yl || !a->yu || !a->hl || !a->hu || !a->zl || !a->zu || !a->lo_only || !a->hi_only ||
        !a->jt_lam || !a->mu || !a->dl || !a->du || !a->sigma || !a->grad_phi || !a->rhs ||
        (a->n > 0 && !a->grad) || (a->m > 0 && (!a->c || !a->lam)) || (a->mI > 0 && !a->ineq)) {
        g_err = "awelu_ipm_newton: need ny = n + mI, B <= 65535 and device pointers";
        return 1;
    }
    if (a->B == 0 || a->ny + a->m == 0) return 0;
    ipm_newton_kernel<<<dim3((unsigned)((a->ny + a->m + 255) / 256), (unsigned)a->B), 256, 0, (hipStream_t)stream>>>(*a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// The accepted step and the kappa_sigma safeguard (ipm_step_kernel) of a->B instances.
int awelu_ipm_step(const AweluIpmStep* a, void* stream) {
    if (!a || a->B < 0 || a->ny < 0 || a->m < 0 || !a->y || !a->yl || !a->yu || !a->hl || !a->hu || !a->zl ||
        !a->zu || !a->mu || !a->acc || !a->y_out || !a->zl_out || !a->zu_out || !a->alpha_z ||
        (a->any_acc && (!a->y_new || !a->dy || !a->dl_old || !a->du_old || !a->tau || !a->alpha || (a->m > 0 && (!a->lam || !a->dlam || !a->lam_out))))) {
        g_err = "awelu_ipm_step: need device pointers";
        return 1;
    }
    if (a->B == 0) return 0;
    ipm_step_kernel<<<dim3((unsigned)a->B), kIpmThreads, 0, (hipStream_t)stream>>>(*a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

// The wide lists of the gather-sums (gather_sum_wide_kernel): nl lists, list l's sources
// wsrc[woff[l] .. woff[l] + ww[l]) (-1 = padding), added to out[r * ldo + wdst[l]] for r < rows.
int awelu_gather_sum_wide(int nl, int rows, const int* wsrc, const int* woff, const int* ww, const int* wdst,
                          const double* vals, long long ldv, const double* x, const int* cols, long long ldx,
                          double* out, long long ldo, void* stream) {
    if (nl < 0 || rows < 0 || rows > 65535 || (nl > 0 && (!wsrc || !woff || !ww || !wdst || !vals || !out)) ||
        (x && !cols)) {
        g_err = "need nl >= 0, 0 <= rows <= 65535 and device pointers (cols with x)";
        return 1;
    }
    if (nl == 0 || rows == 0) return 0;
    gather_sum_wide_kernel<<<dim3((unsigned)nl, (unsigned)rows), 256, 0, (hipStream_t)stream>>>(
        wsrc, woff, ww, wdst, vals, ldv, x, cols, ldx, out, ldo);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        g_err = hipGetErrorString(e);
        return 2;
    }
    return 0;
}

}  // extern "C"
