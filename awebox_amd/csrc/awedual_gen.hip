// awedual_gen -- the generated instance-minor evaluation path of the dual-kite NLP (config 3:
// examples/dual_kites_power_curve.py, direct collocation radau, phase_fix 'single_reelout').
//
// One lane per NLP instance (the AP2 evaluator's instance-minor design, awegpu.hip §4d of DESIGN.md,
// applied to the 126-variable, two-kite node):
//   dual_gen_in (im::transpose_in_kernel): V, P -> VT[i * ld + b], PT[i * ld + b]
//   dual_gen_node_kernel: Radau tiles (instance block, interval, role) and shooting tiles (instance
//     block, four intervals, role) in one launch; a wavefront evaluates one node for 64 instances in
//     the straight-line code generated from dual_node (dual_nodejac.gen.hpp).  A node's outputs are
//     split into four wavefront roles (the rows of kite 2, the rows of kite 3, node 1's translation
//     rows along two halves of their directions) that recompute the values they need, so that each
//     keeps about one kite's working set in registers; each tangent slot goes straight to its J_g
//     entries (1, or the d polynomial columns of a Radau xdot direction scaled by C[r][n] / (h t_f))
//     through the node's destination row staged in LDS; the Radau node's power and side slips and the
//     directional derivatives of its beta and power cost terms go to `objb` (instance-minor).
//   dual_gen_interval_kernel: one lane per instance, four wavefronts per (instance block, interval):
//     the tracking and regularisation terms of the interval's Radau nodes (objective.py:45-544) with
//     the node kernel's beta / power derivatives, the gradient of the interval's columns, the
//     continuity rows (collocation.py:319-336) and the interval's partial sums.
//   dual_gen_finalize_kernel: one lane per instance: the partials in interval order, the power cost
//     over the phase-fixed period, time and homotopy costs, the global gradient entries, the
//     periodicity and t_f-bound rows (as dual_finalize_kernel).
// J_g and grad f leave instance-minor (jac[e * ldj + b]), every store one 512-byte row; g stays per
// instance (g[b * n_g + i]) as the solver reads it.  No float atomics: results are deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/awedual.h"
#include "../../include/awegpu.h"
#include "awedual_gen.hpp"
#include "dual_nodejac.gen.hpp"
#include "dual_tables.hpp"
#include "im_layout.hpp"

namespace dgen {
namespace {

using namespace dlt;

#define DGEN_TRY(expr)                                                                 \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) {                                                        \
            err = std::string(#expr) + ": " + hipGetErrorString(_e);                   \
            return AWE_ERR_HIP;                                                        \
        }                                                                              \
    } while (0)

constexpr int kMaxTan = 1024;
static_assert(awe_dgen::kNTan[0] <= kMaxTan && awe_dgen::kNTan[1] <= kMaxTan, "slot table too small");
constexpr int kRoles = awe_dgen::kRoles;
constexpr int kObjRows = 3 + awe_dgen::kNDbp;   // per Radau node: power, beta_2, beta_3, dbp[kNDbp]
constexpr int kCO = 2 * ADL_NX + ADL_NU + ADL_NZ;   // x, u, xdot, z of an interval
constexpr int kNodeWaves = 4;
// the collocation degree the kernels are instantiated for (the configs' d = 4: each instantiation of
// the node kernel compiles ~35k generated statements; other d use the colour kernel of awedual.hip)
constexpr int kGenD = 4;

// destination count of every tangent slot (1, or d for the xdot directions of a Radau node) and its
// first entry in the node's destination row; compile-time on the device (the generated code's slot
// numbers are constants), built with the run-time d on the host
struct SlotTab {
    int first[2][kMaxTan];
    int cnt[2][kMaxTan];
    int total[2];
    __host__ __device__ constexpr SlotTab(int d) : first(), cnt(), total() {
        for (int kind = 0; kind < 2; ++kind) {
            int dir_of[kMaxTan] = {};
            for (int s = 0; s < kMaxTan; ++s) dir_of[s] = -1;
            for (int r = 0; r < kRowPower; ++r)
                for (int l = 0; l < kDirs; ++l)
                    if (awe_dgen::kTanIdx[kind][r][l] >= 0) dir_of[awe_dgen::kTanIdx[kind][r][l]] = l;
            int f = 0;
            for (int s = 0; s < awe_dgen::kNTan[kind]; ++s) {
                const bool xd = kind == 1 && dir_of[s] >= ADL_NX && dir_of[s] < 2 * ADL_NX;
                first[kind][s] = f;
                cnt[kind][s] = xd ? d : 1;
                f += cnt[kind][s];
            }
            total[kind] = f;
        }
    }
};
template <int D>
constexpr SlotTab kSlots{D};

struct Args {
    awt::DevColl coll;
    int n_k, batch, n_v, n_g, n_p, stride, v_int0, rows, nib, dstride, nkr, single, n_thv;
    unsigned ld8;                // bytes between VT / PT / objb / part rows
    unsigned ldj8;               // bytes between J_g / grad rows
    double kconst[kMaxConst];    // constant J_g values (continuity, periodicity, t_f bounds)
};

__device__ __forceinline__ int interval_tf(const Args& a, int k) { return a.single ? (k < a.nkr ? 1 : 2) : 1; }

// the phase-fixed period of V or P.p.ref (ocp_outputs.py:118-140), from an instance-minor buffer
__device__ __forceinline__ double period(const double* X, const Args& a, unsigned lb) {
    if (!a.single) return im::at(X, 1u, a.ld8, lb);
    return im::at(X, 1u, a.ld8, lb) * a.nkr / a.n_k + im::at(X, 2u, a.ld8, lb) * (a.n_k - a.nkr) / a.n_k;
}

// theta_v entry t of the node variables [diam_t, t_f(k), l_s, diam_s] (single_reelout: theta_v =
// [diam_t, t_f0, t_f1, l_s, diam_s])
__device__ __forceinline__ int node_theta_col(const Args& a, int t, int tfi) {
    if (t == 1) return tfi;
    return a.single ? (t == 0 ? 0 : t + 1) : t;
}

// node variable i of node n (0: shooting) of interval k (first column c0) from VT; xdot at a Radau
// node from the collocation polynomial (collocation.py:202-258), in the colour kernel's order
template <int D>
struct NodeIn {
    const double* v;
    unsigned ld8, lb;
    int c0, n, tfi, thcol[4], gcol;
    double ihtf;
    const double* C;
    __device__ __forceinline__ double at(int col) const { return im::at(v, (unsigned)col, ld8, lb); }
    __device__ __forceinline__ double X(int r, int s) const {
        return at(r == 0 ? c0 + s : c0 + kCO + (r - 1) * (ADL_NX + ADL_NZ) + s);
    }
    __device__ __forceinline__ double operator()(int i) const {
        constexpr int NN = D + 1;
        if (i < ADL_NX) return X(n, i);
        if (i < 2 * ADL_NX) {
            const int s = i - ADL_NX;
            if (n == 0) return at(c0 + ADL_NX + ADL_NU + s);
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < NN; ++r) acc += C[r * NN + n] * X(r, s);
            return acc * ihtf;
        }
        if (i < 2 * ADL_NX + ADL_NU) return at(c0 + ADL_NX + (i - 2 * ADL_NX));
        if (i < kCO) {
            const int z = i - (2 * ADL_NX + ADL_NU);
            return n == 0 ? at(c0 + 2 * ADL_NX + ADL_NU + z) : at(c0 + kCO + (n - 1) * (ADL_NX + ADL_NZ) + ADL_NX + z);
        }
        if (i < ADL_NW) return at(thcol[i - kCO]);
        return at(gcol);                                          // phi.gamma
    }
};

// theta0 of the lane's instance: th[i] at PT row (n_v + NW + 20 + i)
struct ThIn {
    const double* p;
    unsigned row0, ld8, lb;
    __device__ __forceinline__ double operator[](int i) const { return im::at(p, row0 + (unsigned)i, ld8, lb); }
};

// tan[s] = v  ->  the J_g entries of slot s (dt: the node's destination row in LDS, byte offsets)
template <int D, int KIND>
struct JSink {
    double* jac;
    unsigned lb;
    const unsigned* dt;
    const double* xs;
    struct Ref {
        const JSink* s;
        int slot;
        __device__ __forceinline__ void operator=(double v) const { s->put(slot, v); }
    };
    __device__ __forceinline__ Ref operator[](int slot) const { return Ref{this, slot}; }
    __device__ __forceinline__ void put(int slot, double v) const {
        const int f = kSlots<D>.first[KIND][slot], c = kSlots<D>.cnt[KIND][slot];
        if (c == 1) {
            __builtin_nontemporal_store(v, &im::at_byte(jac, dt[f] + lb));
            return;
        }
#pragma unroll
        for (int q = 0; q < D; ++q) __builtin_nontemporal_store(xs[q] * v, &im::at_byte(jac, dt[f + q] + lb));
    }
};

// rows r0 + i of an instance-minor buffer
struct ImRef {
    double* p;
    unsigned r0, ld8, lb;
    __device__ __forceinline__ double& operator[](int i) const { return im::at(p, r0 + (unsigned)i, ld8, lb); }
};

// calls f(std::integral_constant<int, r>) for the role r == role of the generated code.  Each branch
// opens with a distinct empty asm statement: the roles' bodies all begin by loading the same node
// inputs and theta0 entries, and without the marker the compiler hoists those loads above the branch,
// where ~220 doubles then stay live through every role (3,000 VGPRs spilled to scratch)
// diagnostics: -DDGEN_ONLY_ROLE=r (with -DDGEN_RADAU_ONLY) compiles one role of the Radau node alone,
// to read its register use and scratch size (-Rpass-analysis=kernel-resource-usage)
#ifndef DGEN_ONLY_ROLE
#define DGEN_ONLY_ROLE -1
#endif
template <int I = 0, class F>
__device__ __forceinline__ void for_role(int role, const F& f) {
    if constexpr (DGEN_ONLY_ROLE >= 0 && I == 0) {
        (void)role;
        f(std::integral_constant<int, DGEN_ONLY_ROLE>{});
    } else if constexpr (I < kRoles) {
        if (role == I) {
            asm volatile(";; dual node role %0" ::"n"(I));
            f(std::integral_constant<int, I>{});
        } else {
            for_role<I + 1>(role, f);
        }
    }
}

template <int D>
__device__ __forceinline__ NodeIn<D> node_in(const double* VT, const Args& a, unsigned lb, int k, int n, double ihtf,
                                             int tfi) {
    NodeIn<D> in{VT, a.ld8, lb, a.v_int0 + k * a.stride, n, tfi, {}, a.n_thv, ihtf, a.coll.C};
#pragma unroll
    for (int t = 0; t < 4; ++t) in.thcol[t] = node_theta_col(a, t, tfi);
    return in;
}

template <int D>
__device__ __forceinline__ void radau_tile(int t, unsigned* ldt, const double* __restrict__ VT,
                                           const double* __restrict__ PT, const double* __restrict__ cst,
                                           const unsigned* __restrict__ dtab, double* __restrict__ g,
                                           double* __restrict__ jac, double* __restrict__ objb, const Args& a) {
    constexpr int NN = D + 1;
    constexpr int W = D < kNodeWaves ? D : kNodeWaves;
    constexpr int T1 = kSlots<D>.total[1];
    const int role = t % kRoles, tk = t / kRoles;
    const int ib = tk / a.n_k, k = tk - ib * a.n_k;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int m = 1; m < NN; ++m)
        im::stage_offsets<64 * kNodeWaves>(ldt + (m - 1) * T1, dtab + (size_t)(k * NN + m) * a.dstride, T1, a.ldj8,
                                           tid);
    __syncthreads();
    const int b = ib * 64 + lane;
    if (wave >= W || b >= a.batch) return;
    const unsigned lb = 8u * (unsigned)b, ld8 = a.ld8;
    const double* C = a.coll.C;
    const int tfi = interval_tf(a, k);
    const double tf = im::at(VT, (unsigned)tfi, ld8, lb);
    const double ihtf = (double)a.n_k / tf;
    const double T = period(VT, a, lb);
    const double psi = im::at(VT, (unsigned)(a.n_thv + kPhiPsi), ld8, lb);
    const unsigned cost = (unsigned)(a.n_v + ADL_NW);
    const double cb = im::at(PT, cost + kCostBeta, ld8, lb) / cst[ADL_C_NORM_BETA];
    const double cp = im::at(PT, cost + kCostPower, ld8, lb);
    const ThIn th{PT, (unsigned)(a.n_v + ADL_NW + 20), ld8, lb};
    double* gb = g + (size_t)b * a.n_g + (size_t)k * a.rows + ADL_N_EQ + ADL_N_INEQ;
    for (int n = 1 + wave; n < NN; n += W) {
        const int j = n - 1;
        const double wq = a.coll.w[j];
        double xs[D];                                 // C[r][n] / (h t_f) of the columns X_r, r != n
#pragma unroll
        for (int q = 0; q < D; ++q) xs[q] = C[(q < n ? q : q + 1) * NN + n] * ihtf;
        const NodeIn<D> in = node_in<D>(VT, a, lb, k, n, ihtf, tfi);
        JSink<D, 1> js{jac, lb, ldt + (n - 1) * T1, xs};
        const unsigned orow = (unsigned)((k * D + j) * kObjRows);
        ImRef obv{objb, orow, ld8, lb}, dbp{objb, orow + 3, ld8, lb};
        // the node's beta and power cost terms: ex2 beta_k^2 (wq c_beta / norm) and ex3 p, the
        // (1 - psi) power cost -c_P (t_f / N) wq / T of the colour kernel
        const double ex2 = wq * cb;
        const double ex3 = (1.0 - psi) * (-cp) * (tf / a.n_k) * wq / T;
        const double cxx = C[n * NN + n] * ihtf, itf = 1.0 / tf;
        for_role(role, [&](auto r) {
            awe_dgen::dual_node_radau<1, decltype(r)::value>(in, cxx, itf, ex2, ex3, th, cst, gb + j * ADL_N_EQ, js,
                                                              dbp, obv);
        });
    }
}

template <int D>
__device__ __forceinline__ void shoot_tile(int t, unsigned* ldt, const double* __restrict__ VT,
                                           const double* __restrict__ PT, const double* __restrict__ cst,
                                           const unsigned* __restrict__ dtab, const unsigned* __restrict__ ctab,
                                           const int* __restrict__ coff, double* __restrict__ g,
                                           double* __restrict__ jac, const Args& a) {
    constexpr int NN = D + 1;
    constexpr int T0 = kSlots<D>.total[0];
    const int nk4 = (a.n_k + kNodeWaves - 1) / kNodeWaves;
    const int role = t % kRoles, tk = t / kRoles;
    const int ib = tk / nk4, k0 = (tk - ib * nk4) * kNodeWaves;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int w = 0; w < kNodeWaves && k0 + w < a.n_k; ++w)
        im::stage_offsets<64 * kNodeWaves>(ldt + w * T0, dtab + (size_t)((k0 + w) * NN) * a.dstride, T0, a.ldj8, tid);
    __syncthreads();
    const int k = k0 + wave;
    const int b = ib * 64 + lane;
    if (k >= a.n_k || b >= a.batch) return;
    const unsigned lb = 8u * (unsigned)b, ld8 = a.ld8;
    const int tfi = interval_tf(a, k);
    const double ihtf = (double)a.n_k / im::at(VT, (unsigned)tfi, ld8, lb);
    const NodeIn<D> in = node_in<D>(VT, a, lb, k, 0, ihtf, tfi);
    const ThIn th{PT, (unsigned)(a.n_v + ADL_NW + 20), ld8, lb};
    JSink<D, 0> js{jac, lb, ldt + wave * T0, nullptr};
    double* gb = g + (size_t)b * a.n_g + (size_t)k * a.rows;
    for_role(role, [&](auto r) { awe_dgen::dual_node_shoot<1, decltype(r)::value>(in, th, cst, gb, js); });
    if (role != 0) return;
    // the interval's constant J_g entries (continuity; periodicity and t_f bounds in the last one)
    for (int q = coff[k]; q < coff[k + 1]; ++q) {
        const unsigned e = ctab[q];
        __builtin_nontemporal_store(a.kconst[e >> 24], &im::at(jac, e & 0xffffffu, a.ldj8, lb));
    }
}

template <int D>
__global__ __launch_bounds__(64 * kNodeWaves) __attribute__((amdgpu_waves_per_eu(1)))
void dual_gen_node_kernel(const double* __restrict__ VT, const double* __restrict__ PT,
                          const double* __restrict__ cst, const unsigned* __restrict__ dtab,
                          const unsigned* __restrict__ ctab, const int* __restrict__ coff, double* __restrict__ g,
                          double* __restrict__ jac, double* __restrict__ objb, Args a) {
    constexpr int T0 = kSlots<D>.total[0], T1 = kSlots<D>.total[1];
    constexpr int NLDT = D * T1 > kNodeWaves * T0 ? D * T1 : kNodeWaves * T0;
    __shared__ unsigned ldt[NLDT];
    const int nr = a.nib * a.n_k * kRoles;
    const int ns = a.nib * ((a.n_k + kNodeWaves - 1) / kNodeWaves) * kRoles;
    const int t = im::xcd_tile(nr + ns);
    if (t >= nr + ns) return;
    if (t < nr) radau_tile<D>(t, ldt, VT, PT, cst, dtab, g, jac, objb, a);
#ifndef DGEN_RADAU_ONLY
    else shoot_tile<D>(t - nr, ldt, VT, PT, cst, dtab, ctab, coff, g, jac, a);
#endif
}

// sum of the node's dbp entries along direction dir (compile-time dir: folds to the matching rows)
__device__ __forceinline__ double dbp_along(int dir, const ImRef& ob) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < awe_dgen::kNDbp; ++q)
        if (awe_dgen::kDbpDir[q] == dir) s += ob[3 + q];
    return s;
}

// effective objective weight of node variable i (objective.py:45-544; the t_f entry has none,
// objective.py:132): we and, for the tracked variables, psi we
__device__ __forceinline__ double weight(const double* PT, const double* cst, const Args& a, unsigned lb, int i,
                                         bool& track) {
    int ci;
    double nrm;
    track = false;
    if (i < ADL_NX || (i >= 119 && i < 122)) { ci = kCostTracking; nrm = cst[ADL_C_NORM_TRACKING]; track = true; }
    else if (i < 2 * ADL_NX) { ci = kCostXdotRegularisation; nrm = cst[ADL_C_NORM_XDOT_REG]; }
    else if (i < 119) {
        const int u = i - 100;
        const bool fict = (u % 9) < 6 && u < 18;
        ci = fict ? kCostFictitious : kCostURegularisation;
        nrm = cst[fict ? ADL_C_NORM_FICTITIOUS : ADL_C_NORM_U_REG];
    } else { ci = kCostThetaRegularisation; nrm = cst[ADL_C_NORM_THETA_REG]; }
    if (i == awe::dl::kTf) return 0.0;
    return im::at(PT, (unsigned)(a.n_v + i), a.ld8, lb) * im::at(PT, (unsigned)(a.n_v + ADL_NW + ci), a.ld8, lb) / nrm;
}

// The interval kernel: one lane per instance, kIntWaves wavefronts per (instance block, interval);
// wavefront w takes the state components i = w mod kIntWaves (directions i and 50 + i at every Radau
// node), then a share of the controls, and wavefront 0 the algebraic variables, theta and the sums.
constexpr int kIntWaves = 4;
template <int D>
__global__ __launch_bounds__(64 * kIntWaves) void dual_gen_interval_kernel(
        const double* __restrict__ VT, const double* __restrict__ PT, const double* __restrict__ cst,
        const double* __restrict__ objb, double* __restrict__ g, double* __restrict__ grad,
        double* __restrict__ part, Args a) {
    constexpr int NN = D + 1;
    constexpr int W = kIntWaves;
    __shared__ double red[W][3][D][64];           // per wave: tracking, other, t_f-direction sums
    const int total = a.nib * a.n_k;
    const int t = im::xcd_tile(total);
    if (t >= total) return;
    const int ib = t / a.n_k, k = t - ib * a.n_k;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int b = ib * 64 + lane;
    const bool act = b < a.batch;
    const int bb = act ? b : ib * 64;             // idle lanes read instance ib 64 and store nothing
    const unsigned ld8 = a.ld8, lb = 8u * (unsigned)bb;
    const int c0 = a.v_int0 + k * a.stride;
    auto V = [&](int col) { return im::at(VT, (unsigned)col, ld8, lb); };
    auto Pp = [&](int row) { return im::at(PT, (unsigned)row, ld8, lb); };
    const double* C = a.coll.C;
    const int tfi = interval_tf(a, k);
    const double tf = V(tfi);
    const double ihtf = (double)a.n_k / tf;
    const double psi = V(a.n_thv + kPhiPsi);
    auto X = [&](int r, int i) { return V(r == 0 ? c0 + i : c0 + kCO + (r - 1) * (ADL_NX + ADL_NZ) + i); };
    auto Xref = [&](int j, int i) { return Pp(c0 + kCO + j * (ADL_NX + ADL_NZ) + i); };   // p.ref at node j + 1
    auto ob = [&](int j) { return ImRef{const_cast<double*>(objb), (unsigned)((k * D + j) * kObjRows), ld8, lb}; };
    struct GRef { double* p; __device__ void operator=(double v) const { __builtin_nontemporal_store(v, p); } };
    auto GR = [&](int col) { return GRef{&im::at(grad, (unsigned)(c0 + col), a.ldj8, lb)}; };
    double tr[D], ot[D], otf[D];
#pragma unroll
    for (int j = 0; j < D; ++j) tr[j] = ot[j] = otf[j] = 0.0;
    double* gc = g + (size_t)bb * a.n_g + (size_t)k * a.rows + ADL_N_EQ + ADL_N_INEQ + D * ADL_N_EQ;
    // state components: tracking of x, regularisation of xdot, their gradient through the polynomial,
    // the t_f-direction terms -2 wq w xdot^2 / t_f, and the continuity row
#pragma unroll
    for (int i0 = 0; i0 < ADL_NX; i0 += W) {
        const int i = i0 + wave;
        if (i >= ADL_NX) break;
        double Xr[NN];
#pragma unroll
        for (int r = 0; r < NN; ++r) Xr[r] = X(r, i);
        bool trk_x, trk_xd;
        const double we_x = weight(PT, cst, a, lb, i, trk_x), we_xd = weight(PT, cst, a, lb, ADL_NX + i, trk_xd);
        const double wtr_x = psi * we_x, wtr_xd = we_xd;        // x tracked, xdot regularised
        double ox[D], oxd[D];
#pragma unroll
        for (int n = 1; n < NN; ++n) {
            const int j = n - 1;
            const double wq = a.coll.w[j];
            double s = 0.0;
#pragma unroll
            for (int r = 0; r < NN; ++r) s += C[r * NN + n] * Xr[r];
            const double xd = s * ihtf;
            const double cxx = C[n * NN + n] * ihtf;
            const double e = Xr[n] - Xref(j, i);
            const ImRef o = ob(j);
            ox[j] = 2.0 * wq * (wtr_x * e + wtr_xd * xd * cxx) + dbp_along(i, o);
            oxd[j] = 2.0 * wq * wtr_xd * xd + dbp_along(ADL_NX + i, o);
            tr[j] += wq * we_x * e * e;
            ot[j] += wq * we_xd * xd * xd;
            otf[j] -= 2.0 * wq * wtr_xd * xd * xd / tf;
        }
        double cs = 0.0;                                            // continuity, the colour kernel's sum
#pragma unroll
        for (int rr = 0; rr < NN; ++rr) cs += a.coll.D[rr] * Xr[rr];
        const double xnext = V(c0 + a.stride + i);
        if (act) {
            double gs = 0.0;                                        // x[k]: polynomial path only
#pragma unroll
            for (int m = 1; m < NN; ++m) gs += oxd[m - 1] * C[0 * NN + m] * ihtf;
            GR(i) = gs;
#pragma unroll
            for (int n = 1; n < NN; ++n) {                          // coll x of node n
                double s = ox[n - 1];
#pragma unroll
                for (int m = 1; m < NN; ++m)
                    if (m != n) s += oxd[m - 1] * C[n * NN + m] * ihtf;
                GR(kCO + (n - 1) * (ADL_NX + ADL_NZ) + i) = s;
            }
            gc[i] = xnext - cs;
        }
    }
    // controls (zero-order hold): regularisation and fictitious controls
    for (int u = wave; u < ADL_NU; u += W) {
        const int dir = 2 * ADL_NX + u;
        bool trk;
        const double we = weight(PT, cst, a, lb, dir, trk);
        const double e = V(c0 + ADL_NX + u) - Pp(c0 + ADL_NX + u);
        double gs = 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            const double wq = a.coll.w[j];
            double o = 2.0 * wq * we * e;
#pragma unroll
            for (int q = 0; q < awe_dgen::kNDbp; ++q)
                if (awe_dgen::kDbpDir[q] == dir) o += ob(j)[3 + q];
            gs += o;
            ot[j] += wq * we * e * e;
        }
        if (act) GR(ADL_NX + u) = gs;
    }
    for (int c = ADL_NX + ADL_NU + wave; c < kCO; c += W)
        if (act) GR(c) = 0.0;                                       // xdot[k], z[k]
    if (k == a.n_k - 1)
        for (int i = wave; i < ADL_NX; i += W)
            if (act) __builtin_nontemporal_store(0.0, &im::at(grad, (unsigned)(c0 + a.stride + i), a.ldj8, lb));
#pragma unroll
    for (int j = 0; j < D; ++j) {
        red[wave][0][j][lane] = tr[j];
        red[wave][1][j][lane] = ot[j];
        red[wave][2][j][lane] = otf[j];
    }
    __syncthreads();
    if (wave != 0) return;
    // algebraic variables (tracked), theta (regularised), beta and power terms, the partial sums
    double TR = 0.0, OT = 0.0, A = 0.0, pd[4] = {0.0, 0.0, 0.0, 0.0};
    const double cb = Pp(a.n_v + ADL_NW + kCostBeta) / cst[ADL_C_NORM_BETA];
#pragma unroll
    for (int n = 1; n < NN; ++n) {
        const int j = n - 1;
        const double wq = a.coll.w[j];
        const ImRef o = ob(j);
        double trj = 0.0, otj = 0.0, otfj = 0.0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            trj += red[w][0][j][lane];
            otj += red[w][1][j][lane];
            otfj += red[w][2][j][lane];
        }
#pragma unroll
        for (int z = 0; z < ADL_NZ; ++z) {
            const int dir = 2 * ADL_NX + ADL_NU + z;
            bool trk;
            const double we = weight(PT, cst, a, lb, dir, trk);
            const int col = kCO + j * (ADL_NX + ADL_NZ) + ADL_NX + z;
            const double e = V(c0 + col) - Pp(c0 + col);
            if (act) GR(col) = 2.0 * wq * (psi * we) * e + dbp_along(dir, o);
            trj += wq * we * e * e;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {                               // diam_t, t_f(k), l_s, diam_s
            const int dir = kCO + q;
            bool trk;
            const double we = weight(PT, cst, a, lb, dir, trk);
            const int col = node_theta_col(a, q, tfi);
            const double e = V(col) - Pp(col);
            pd[q] += 2.0 * wq * we * e + dbp_along(dir, o) + (q == 1 ? otfj : 0.0);
            otj += wq * we * e * e;
        }
        otj += wq * cb * (o[1] * o[1] + o[2] * o[2]);
        TR += trj;
        OT += otj;
        A += wq * o[0] / a.n_k;
    }
    if (!act) return;
    const ImRef pp{part, (unsigned)(k * kNPart), ld8, lb};
    pp[0] = TR;
    pp[1] = OT;
    pp[2] = A;
#pragma unroll
    for (int q = 0; q < 4; ++q) pp[3 + q] = pd[q];
    pp[7] = 0.0;
}

// one lane per instance: partials in interval order, power cost over the phase-fixed period, time
// and homotopy costs, the global gradient entries, the periodicity and t_f-bound rows
__global__ __launch_bounds__(64) void dual_gen_finalize_kernel(const double* __restrict__ VT,
                                                              const double* __restrict__ PT,
                                                              const double* __restrict__ cst,
                                                              const double* __restrict__ part, double* __restrict__ f,
                                                              double* __restrict__ g, double* __restrict__ grad,
                                                              int d, Args a) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= a.batch) return;
    const unsigned lb = 8u * (unsigned)b, ld8 = a.ld8;
    auto V = [&](int col) { return im::at(VT, (unsigned)col, ld8, lb); };
    auto Pp = [&](int row) { return im::at(PT, (unsigned)row, ld8, lb); };
    auto GR = [&](int col) -> double& { return im::at(grad, (unsigned)col, a.ldj8, lb); };
    const int cost = a.n_v + ADL_NW;
    const int nthv = a.n_thv;
    double tr = 0.0, ot = 0.0, e_end = 0.0, A0 = 0.0, A1 = 0.0, pdt = 0.0, pls = 0.0, pds = 0.0;
    double ptf0 = 0.0, ptf1 = 0.0;
    const double tf0 = V(1), tf1 = a.single ? V(2) : V(1);
    constexpr int U = 4;                       // intervals whose partials are loaded together
    for (int k0 = 0; k0 < a.n_k; k0 += U) {
        double q[U][7];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < 7; ++e)
                q[u][e] = im::at(part, (unsigned)(min(k0 + u, a.n_k - 1) * kNPart + e), ld8, lb);
#pragma unroll
        for (int u = 0; u < U; ++u) {          // summed in interval order
            const int k = k0 + u;
            if (k >= a.n_k) break;
            const bool ph1 = a.single && k >= a.nkr;
            tr += q[u][0];
            ot += q[u][1];
            e_end += (ph1 ? tf1 : tf0) * q[u][2];
            if (ph1) { A1 += q[u][2]; ptf1 += q[u][4]; } else { A0 += q[u][2]; ptf0 += q[u][4]; }
            pdt += q[u][3]; pls += q[u][5]; pds += q[u][6];
        }
    }
    const double T = period(VT, a, lb);
    const double Tref = period(PT, a, lb);
    const double psi = V(nthv + kPhiPsi);
    const double cp = Pp(cost + kCostPower), ct = Pp(cost + kCostTf);
    const double f_power = -cp * e_end / T;
    double fv = psi * tr + (1.0 - psi) * f_power + ot + ct * (T - Tref) * (T - Tref);
    for (int i = 0; i < 7; ++i) fv += Pp(cost + kPhiCost[i]) * V(nthv + i);
    f[b] = fv;
    const double n0 = a.single ? (double)a.nkr / a.n_k : 1.0, n1 = a.single ? (double)(a.n_k - a.nkr) / a.n_k : 0.0;
    GR(0) = pdt;
    GR(1) = ptf0 + (1.0 - psi) * (-cp) * (A0 * T - e_end * n0) / (T * T) + 2.0 * ct * (T - Tref) * n0;
    if (a.single) {
        GR(2) = ptf1 + (1.0 - psi) * (-cp) * (A1 * T - e_end * n1) / (T * T) + 2.0 * ct * (T - Tref) * n1;
        GR(3) = pls;
        GR(4) = pds;
    } else {
        GR(2) = pls;
        GR(3) = pds;
    }
    for (int i = 0; i < 7; ++i) GR(nthv + i) = Pp(cost + kPhiCost[i]) + (i == kPhiPsi ? tr - f_power : 0.0);
    GR(nthv + 7) = 0.0;
    GR(nthv + 8) = 0.0;
    double* gb = g + (size_t)b * a.n_g;
    const int gp = a.n_k * a.rows;
    if (a.single) {
        const double frac = cst[ADL_C_PHASE_FIX_REELOUT];
        gb[gp + ADL_NX] = (T - cst[ADL_C_TF_UB]) / frac;
        gb[gp + ADL_NX + 1] = (cst[ADL_C_TF_LB] - T) / frac;
    }
    const int x0 = a.v_int0;
    const int xT = a.v_int0 + (a.n_k - 1) * a.stride + kCO + (d - 1) * (ADL_NX + ADL_NZ);
    for (int i = 0; i < ADL_NX; ++i) gb[gp + i] = V(x0 + kPeriodicOrder[i]) - V(xT + kPeriodicOrder[i]);
}

}  // namespace

struct Plan {
    Args a{};
    int d = 0;
    size_t ld = 0, nnz = 0;
    unsigned *d_dtab = nullptr, *d_ctab = nullptr;
    int* d_coff = nullptr;
    double *d_VT = nullptr, *d_PT = nullptr, *d_objb = nullptr, *d_part = nullptr;
    hipEvent_t ev[5] = {};
    bool timed = false;
};

void destroy(Plan* p) {
    if (!p) return;
    for (void* q : {(void*)p->d_dtab, (void*)p->d_ctab, (void*)p->d_coff, (void*)p->d_VT, (void*)p->d_PT,
                    (void*)p->d_objb, (void*)p->d_part})
        if (q) (void)hipFree(q);
    for (auto& e : p->ev)
        if (e) (void)hipEventDestroy(e);
    delete p;
}

// destination tables from the gather list of build_tables: per (interval k, node n) a row of CCS
// positions in kSlots order (slot s of the node's generated code, then its d polynomial columns for a
// Radau xdot direction), and per interval the constant entries (position | value index << 24)
int create(const Tables& T, const std::vector<double>& consts, int batch, Plan** out, std::string& why,
           std::string& err) {
    *out = nullptr;
    const Layout& L = T.lay;
    const int n_k = L.n_k, d = L.d, NN = d + 1;
    if ((int)consts[ADL_C_N_ELEMENTS] != awe_dgen::kNElements) {
        why = "the generated node code has " + std::to_string(awe_dgen::kNElements) + " tether elements, the constants " +
              std::to_string((int)consts[ADL_C_N_ELEMENTS]);
        return AWE_OK;
    }
    for (int i = 0; i < 54; ++i)
        if ((int)consts[ADL_C_SD_LEN + i] != awe_dgen::kSdLen[i]) {
            why = "the generated node code was built for other stability-derivative table lengths";
            return AWE_OK;
        }
    if (d != kGenD) {
        why = "the generated dual-kite path is instantiated for d = " + std::to_string(kGenD);
        return AWE_OK;
    }
    if (T.row.size() >= (1u << 24)) { why = "J_g too large for the constant table"; return AWE_OK; }
    // node-relative tangent index of the colour tables -> (row, direction)
    const ColorTabs& ct = T.ct;
    std::vector<std::pair<int, int>> rev[2];
    for (int kind = 0; kind < 2; ++kind) {
        rev[kind].assign(ct.tsize[kind], {-1, -1});
        for (int dir = 0; dir < kDirs; ++dir) {
            const int c = ct.col[kind][dir];
            if (c < 0) continue;
            Mask m;
            m.lo = ct.cm_lo[kind][c];
            m.hi = ct.cm_hi[kind][c];
            for (int r = 0; r < kRowPower; ++r)
                if (T.dmask[kind][dir].has(r)) rev[kind][ct.off[kind][c] + m.below(r)] = {r, dir};
        }
    }
    const SlotTab st(d);
    const int dstride = std::max(st.total[0], st.total[1]);
    std::vector<unsigned> dtab((size_t)n_k * NN * dstride, 0xffffffffu);
    std::vector<unsigned> ctab;
    std::vector<int> coff(n_k + 1, 0);
    auto fail_int = [&](const char* m) { err = m; return AWE_ERR_ARG; };
    for (int k = 0; k < n_k; ++k) {
        for (int e = T.goff[k]; e < T.goff[k + 1]; ++e) {
            const unsigned pos = (unsigned)T.gslot[e];
            const uint32_t cd = T.gcode[e];
            const uint32_t kind = cd >> 29;
            const int rr = (cd >> 25) & 15, nn = (cd >> 21) & 15, src = (int)(cd & ((1u << 21) - 1u));
            if (kind == kKindConst) {
                ctab.push_back(pos | ((unsigned)src << 24));
                continue;
            }
            // src = toff(n) + node-relative index; the poly code carries n, the plain one is found by range
            int n = kind == kKindTangPoly ? nn : -1;
            if (n < 0) n = src < ct.tsize[0] ? 0 : 1 + (src - ct.tsize[0]) / ct.tsize[1];
            const int kd = n > 0 ? 1 : 0;
            const int loc = n == 0 ? src : src - ct.tsize[0] - (n - 1) * ct.tsize[1];
            const auto [r, dir] = rev[kd][loc];
            if (r < 0) return fail_int("internal: gather entry without a (row, direction)");
            const int s = awe_dgen::kTanIdx[kd][r][dir];
            if (s < 0) return fail_int("internal: J_g entry without a generated tangent");
            int q = 0;
            if (kind == kKindTangPoly) q = rr < n ? rr : rr - 1;
            if (q >= st.cnt[kd][s]) return fail_int("internal: destination count of a generated tangent");
            unsigned& slot = dtab[(size_t)(k * NN + n) * dstride + st.first[kd][s] + q];
            if (slot != 0xffffffffu) return fail_int("internal: two J_g entries for one generated destination");
            slot = pos;
        }
        coff[k + 1] = (int)ctab.size();
        for (int n = 0; n < NN; ++n)
            for (int i = 0; i < st.total[n > 0 ? 1 : 0]; ++i)
                if (dtab[(size_t)(k * NN + n) * dstride + i] == 0xffffffffu)
                    return fail_int("internal: generated destination without a J_g entry");
    }
    if (ctab.empty()) ctab.push_back(0);
    for (auto& x : dtab) if (x == 0xffffffffu) x = 0;   // padding of the shorter node kind
    auto* p = new Plan();
    Args& a = p->a;
    for (int j = 0; j < NN; ++j) {
        for (int r = 0; r < NN; ++r) a.coll.C[j * NN + r] = T.coll.C[j][r];
        a.coll.D[j] = T.coll.D[j];
    }
    for (int j = 0; j < d; ++j) a.coll.w[j] = T.coll.w[j];
    a.n_k = n_k;
    a.batch = batch;
    a.n_v = L.n_v;
    a.n_g = L.n_g;
    a.n_p = L.n_p;
    a.stride = L.stride;
    a.v_int0 = L.v_int0;
    a.rows = L.rows;
    a.nib = (batch + 63) / 64;
    a.dstride = dstride;
    a.nkr = L.nk_reelout;
    a.single = L.single;
    a.n_thv = L.n_thv;
    for (size_t i = 0; i < T.kconst.size() && i < (size_t)kMaxConst; ++i) a.kconst[i] = T.kconst[i];
    p->d = d;
    p->ld = (size_t)batch;
    p->nnz = T.row.size();
    a.ld8 = (unsigned)(8 * p->ld);
    const size_t rows_in = std::max((size_t)L.n_v, (size_t)L.n_p);
    if (rows_in * p->ld * 8 >= ((size_t)1 << 32)) {
        destroy(p);
        why = "instance-minor inputs would exceed 4 GiB";
        return AWE_OK;
    }
    auto up = [&](auto*& dst, const auto& v) -> int {
        DGEN_TRY(hipMalloc((void**)&dst, sizeof(v[0]) * v.size()));
        DGEN_TRY(hipMemcpy(dst, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice));
        return AWE_OK;
    };
    int rc = up(p->d_dtab, dtab);
    if (!rc) rc = up(p->d_ctab, ctab);
    if (!rc) rc = up(p->d_coff, coff);
    auto alloc = [&](double*& dst, size_t n) -> int {
        DGEN_TRY(hipMalloc((void**)&dst, sizeof(double) * n));
        return AWE_OK;
    };
    if (!rc) rc = alloc(p->d_VT, p->ld * L.n_v);
    if (!rc) rc = alloc(p->d_PT, p->ld * L.n_p);
    if (!rc) rc = alloc(p->d_objb, p->ld * (size_t)n_k * d * kObjRows);
    if (!rc) rc = alloc(p->d_part, p->ld * (size_t)n_k * kNPart);
    for (auto& e : p->ev)
        if (!rc && hipEventCreate(&e) != hipSuccess) { err = "hipEventCreate"; rc = AWE_ERR_HIP; }
    if (rc) {
        destroy(p);
        return rc;
    }
    *out = p;
    return AWE_OK;
}

int eval(Plan* p, const double* cst, const double* V, const double* P, double* f, double* g, double* grad_f,
         double* jac, size_t ldj, hipStream_t s, std::string& err) {
    Args a = p->a;
    const int B = a.batch;
    if (ldj < (size_t)B) { err = "ld must be >= batch"; return AWE_ERR_ARG; }
    if (std::max(p->nnz, (size_t)a.n_v) * ldj * 8 >= ((size_t)1 << 32)) {
        err = "instance-minor J_g must stay below 4 GiB";
        return AWE_ERR_ARG;
    }
    a.ldj8 = (unsigned)(8 * ldj);
    DGEN_TRY(hipEventRecord(p->ev[0], s));
    const dim3 tgrid((unsigned)((a.n_v + a.n_p + 63) / 64), (unsigned)a.nib);
    im::transpose_in_kernel<<<tgrid, 256, 0, s>>>(V, P, p->d_VT, p->d_PT, B, a.n_v, a.n_p, (int)p->ld);
    DGEN_TRY(hipGetLastError());
    DGEN_TRY(hipEventRecord(p->ev[1], s));
    const int nk4 = (a.n_k + kNodeWaves - 1) / kNodeWaves;
    const dim3 ngrid((unsigned)im::xcd_grid(a.nib * (a.n_k + nk4) * kRoles));
    const dim3 igrid((unsigned)im::xcd_grid(a.nib * a.n_k));
#define DGEN_LAUNCH(DD)                                                                                            \
    dual_gen_node_kernel<DD><<<ngrid, 64 * kNodeWaves, 0, s>>>(p->d_VT, p->d_PT, cst, p->d_dtab, p->d_ctab,         \
                                                              p->d_coff, g, jac, p->d_objb, a);                    \
    if (hipGetLastError() != hipSuccess) { err = "dual_gen_node_kernel launch"; return AWE_ERR_HIP; }              \
    DGEN_TRY(hipEventRecord(p->ev[2], s));                                                                         \
    dual_gen_interval_kernel<DD><<<igrid, 64 * kIntWaves, 0, s>>>(p->d_VT, p->d_PT, cst, p->d_objb, g, grad_f,      \
                                                                  p->d_part, a)
    switch (p->d) {
        case kGenD: DGEN_LAUNCH(kGenD); break;
        default: err = "unsupported d"; return AWE_ERR_ARG;
    }
#undef DGEN_LAUNCH
    DGEN_TRY(hipGetLastError());
    DGEN_TRY(hipEventRecord(p->ev[3], s));
    dual_gen_finalize_kernel<<<dim3((unsigned)a.nib), 64, 0, s>>>(p->d_VT, p->d_PT, cst, p->d_part, f, g, grad_f, p->d,
                                                                  a);
    DGEN_TRY(hipGetLastError());
    DGEN_TRY(hipEventRecord(p->ev[4], s));
    p->timed = true;
    return AWE_OK;
}

int last_ms(Plan* p, float ms[4], std::string& err) {
    if (!p || !p->timed) { err = "no timed instance-minor evaluation yet"; return AWE_ERR_ARG; }
    DGEN_TRY(hipEventSynchronize(p->ev[4]));
    for (int i = 0; i < 4; ++i) DGEN_TRY(hipEventElapsedTime(&ms[i], p->ev[i], p->ev[i + 1]));
    return AWE_OK;
}

}  // namespace dgen
