// awedual -- MI355X (gfx950) evaluator for the awebox multi-kite power-cycle NLP (config 3: two
// 6-DOF AP2 kites on secondary tethers, architecture {1: 0, 2: 1, 3: 1}, direct collocation
// radau, zoh, phase_fix 'single_reelout'; examples/dual_kites_power_curve.py).
//
// Replaces the CasADi-expanded SX evaluation of f, g, grad f and J_g that IPOPT reaches through
// nlpsol (awebox/opti/preparation.py:366-400).
//
// Execution model (the AP2 evaluator's design, awegpu.hip, scaled to the 126-variable node):
//   * one workgroup per (NLP instance, shooting interval), 256 threads;
//   * the interval's slice of V and of P.p.ref plus the effective objective weights are staged
//     in LDS with coalesced loads;
//   * model pass, compressed forward mode: the 127 seed directions of a node are coloured on the
//     host into <= 64 groups with disjoint row sets (37 at the shooting node, 39 at a Radau node);
//     one thread per (node, colour) evaluates dual_node in dual arithmetic along its colour (the
//     193 tasks at d = 4 are packed into 4 wavefronts), recovering every node Jacobian block.  The
//     collocation chain rule
//     xdot = C X / (h t_f(k)) is folded into the seeds (dual_tables.hpp);
//   * rows stream from the lanes into a compressed LDS tangent buffer (branch-free sink);
//   * objective pass: one thread per (Radau node, direction) forms the directional derivative
//     of the regularisation, beta and power terms; per V column they are summed in a fixed order;
//   * write-out: g rows and grad f columns of the interval are contiguous stores; J_g values come
//     from a host-built gather list (one entry per CCS slot: tangent index, polynomial scale or
//     constant); a one-workgroup-per-instance finalize kernel reduces the interval partials in a
//     fixed order (power cost over the phase-fixed period, time cost, homotopy) and writes the
//     global gradient entries, the periodicity and t_f-bound rows.  No float atomics.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/awedual.h"
#include "../../include/awegpu.h"
#include "dual_model.hpp"
#include "dual_tables.hpp"
#include "dual_hess_tables.hpp"
#include "awedual_gen.hpp"

namespace {

using namespace dlt;

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define ADL_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess)                                                          \
            return fail(AWE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)


struct DArgs {
    const double* V;
    const double* P;
    const double* cst;
    awt::DevColl coll;
    const ColorTabs* ct;
    const int* goff;
    const int* gslot;
    const uint32_t* gcode;
    double kconst[kMaxConst];
    double* f;
    double* g;
    double* grad;
    double* jac;
    double* part;         // [B][n_k][kNPart]
    int n_k, d, n_v, n_g, n_p, nnz, stride, v_int0, nkr, single, n_thv, tang_total;
};

__device__ __forceinline__ double time_period(const double* V, const DArgs& a) {
    if (!a.single) return V[1];
    return V[1] * a.nkr / a.n_k + V[2] * (a.n_k - a.nkr) / a.n_k;   // ocp_outputs.py:118-140
}

// node variable i along lane's colour
struct DLaneIn {
    const double* w;
    const int8_t* col;
    int lane;
    double cxx;          // C[n][n] / (h tf) at a Radau node, 0 at the shooting node
    double tfl;          // -1/tf if this lane carries the t_f colour of a Radau node, else 0
    __device__ __forceinline__ awe::Dual operator()(int i) const {
        double t = (col[i] == lane) ? 1.0 : 0.0;
        if (i >= ADL_NX && i < 2 * ADL_NX) {
            if (col[i - ADL_NX] == lane) t += cxx;
            t += tfl * w[i];
        }
        return awe::Dual(w[i], t);
    }
};

struct DSink {
    double* tp;          // node tangent base + colour offset
    double* gv;          // node values [kGvalStride]
    double* dump;        // this lane's private dump slot
    uint64_t lo, hi;
    bool c0;
    __device__ __forceinline__ void emit(int r, const awe::Dual& v) {
        *(c0 ? gv + r : dump) = v.v;
        bool on;
        int idx;
        if (r < 64) {
            on = (lo >> r) & 1u;
            idx = __popcll(lo & ((1ull << r) - 1ull));
        } else {
            on = (hi >> (r - 64)) & 1u;
            idx = __popcll(lo) + __popcll(hi & ((1ull << (r - 64)) - 1ull));
        }
        *(on ? tp + idx : dump) = v.d;
    }
    __device__ __forceinline__ void eq_row(int r, const awe::Dual& v) { emit(r, v); }
    __device__ __forceinline__ void ineq_row(int r, const awe::Dual& v) { emit(ADL_N_EQ + r, v); }
    __device__ __forceinline__ void power(const awe::Dual& v) { emit(kRowPower, v); }
    __device__ __forceinline__ void beta(int k, const awe::Dual& v) { emit(kRowBeta0 + k, v); }
};

// Preaccumulated sub-model layout per node: main drag [3 values | 3 x 7 partials], then per kite
// the secondary drag [6 values (up, lo) | 6 x 13 partials]; partials w.r.t. the SI inputs
// (q10, dq10, diam_t) and (q10, dq10, q_k, dq_k, diam_s).
constexpr int kPreMain = 3 + 3 * 7;
constexpr int kPreSec = 6 + 6 * 13;
constexpr int kPreStride = kPreMain + 2 * kPreSec;    // 192
constexpr int kPreThreads = 7 + 2 * 13;               // one input direction per thread

// Stage-A atmosphere of every tether element of a node: (uw, d uw/dz, rho, d rho/dz) at the
// element midpoint height, [segment 0..2][element] (the transcendental part of the drag model).
constexpr int kMaxElements = 8;
struct PreAtmosphere {
    const double* atm;   // this node's block [3][kMaxElements][4]
    __device__ __forceinline__ void operator()(int seg, int e, const awe::Dual& zz, const double*, awe::Dual& uw,
                                               awe::Dual& rho) const {
        const double* p = atm + (seg * kMaxElements + e) * 4;
        uw = awe::Dual(p[0], p[1] * zz.d);
        rho = awe::Dual(p[2], p[3] * zz.d);
    }
};

struct DualPreSubmodels {
    const double* pre;   // this node's block
    template <class T>
    __device__ __forceinline__ void kite_atmosphere(const T& qz, const double* th, T& uw, T& rho) const {
        uw = awe::wind_speed(qz, th);
        rho = awe::isa_density(qz, th);
    }
    __device__ __forceinline__ void main_drag(const awe::Dual* q, const awe::Dual* v, const awe::Dual& diam,
                                              const double*, const double*, awe::Dual up[3]) const {
        const double t[7] = {q[0].d, q[1].d, q[2].d, v[0].d, v[1].d, v[2].d, diam.d};
        for (int i = 0; i < 3; ++i) {
            double d = 0.0;
            for (int j = 0; j < 7; ++j) d += pre[3 + i * 7 + j] * t[j];
            up[i] = awe::Dual(pre[i], d);
        }
    }
    __device__ __forceinline__ void sec_drag(int k, const awe::Dual* qb, const awe::Dual* vb, const awe::Dual* qt,
                                             const awe::Dual* vt, const awe::Dual& diam, const double*, const double*,
                                             awe::Dual up[3], awe::Dual lo[3]) const {
        const double* p = pre + kPreMain + k * kPreSec;
        const double t[13] = {qb[0].d, qb[1].d, qb[2].d, vb[0].d, vb[1].d, vb[2].d, qt[0].d, qt[1].d, qt[2].d,
                              vt[0].d, vt[1].d, vt[2].d, diam.d};
        for (int i = 0; i < 6; ++i) {
            double d = 0.0;
            for (int j = 0; j < 13; ++j) d += p[6 + i * 13 + j] * t[j];
            (i < 3 ? up[i] : lo[i - 3]) = awe::Dual(p[i], d);
        }
    }
};

// Workgroup size: the (node, colour) tasks of the model pass (37 + d x 39 at d = 4) are packed
// into 4 wavefronts instead of one wavefront per node, so that two workgroups fit a CU at the
// kernel's register budget (256 VGPRs = 2 waves per SIMD: 8 waves per CU).
constexpr int kBlock = 256;

#ifndef ADL_MIN_BLOCKS
#define ADL_MIN_BLOCKS 2    // __launch_bounds__ minimum waves per SIMD: two workgroups per CU
#endif

// LDS image of the first-order front (staging, node values, sub-models, model pass), shared by
// the first-order kernel and the Hessian kernel
template <int D>
struct FrontLds {
    static constexpr int NN = D + 1;
    static constexpr int STRIDE = 2 * ADL_NX + ADL_NU + ADL_NZ + D * (ADL_NX + ADL_NZ);
    static constexpr int NLOC = ADL_NTHV + 7 + STRIDE + ADL_NX;
    double vloc[NLOC];                 // theta_v, phi, x[k], u, xdot, z, coll.., x[k+1]
    double rloc[ADL_NTHV + STRIDE];    // p.ref: theta_v, interval slice
    double wtr[ADL_NW];                // effective weights (x psi for tracking)
    double wef[ADL_NW];                // effective weights
    double wn[NN][128];                // node values (scaled), [126] = phi.gamma
    double rn[D][ADL_NW];              // reference values at the Radau nodes
    double gval[NN][kGvalStride];
    double dumpbuf[kBlock];
    int8_t colb[2][128];
    double pre[NN][kPreStride];        // preaccumulated tether drags
    double atmo[NN][3 * kMaxElements * 4];
};

// Interval geometry the passes after the front share
struct FrontGeo {
    int tfi;          // index of the interval's t_f in theta_v
    double tf, ihtf;  // t_f(k), n_k / t_f(k)
    double psi;
};

// Stages the interval, forms the node values, preaccumulates the tether drags and runs the
// compressed forward-mode model pass (node tangents into `tang`, node values into s.gval).
template <int D>
__device__ __forceinline__ FrontGeo dual_front(const DArgs& a, FrontLds<D>& s, double* tang, int b, int k, int tid) {
    constexpr int NN = D + 1;
    constexpr int NT = kBlock;
    constexpr int STRIDE = FrontLds<D>::STRIDE;
    constexpr int NLOC = FrontLds<D>::NLOC;
    auto& vloc = s.vloc;
    auto& rloc = s.rloc;
    auto& wtr = s.wtr;
    auto& wef = s.wef;
    auto& wn = s.wn;
    auto& rn = s.rn;
    auto& gval = s.gval;
    auto& dumpbuf = s.dumpbuf;
    auto& colb = s.colb;
    auto& pre = s.pre;
    auto& atmo = s.atmo;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const int nthv = a.n_thv;
    const int base = a.v_int0 + k * STRIDE;
    // ---- stage -------------------------------------------------------------------------
    // every load of a thread's share issued before its LDS stores, unconditionally (a guarded load
    // per element is a branch, and the compiler then waits for each load before the next)
    {
        constexpr int NR = ADL_NTHV + STRIDE;
        constexpr int U = (NLOC + NR + NT - 1) / NT;
        double r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = tid + u * NT;
            const double* src;
            if (i < NLOC) {
                src = i < ADL_NTHV ? V + (i < nthv ? i : 0)
                    : i < ADL_NTHV + 7 ? V + nthv + (i - ADL_NTHV) : V + base + (i - ADL_NTHV - 7);
            } else {
                const int q = i < NLOC + NR ? i - NLOC : 0;
                src = q < ADL_NTHV ? P + (q < nthv ? q : 0) : P + base + (q - ADL_NTHV);
            }
            r[u] = *src;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = tid + u * NT;
            if (i < NLOC) vloc[i] = (i < ADL_NTHV && i >= nthv) ? 0.0 : r[u];
            else if (i < NLOC + NR) {
                const int q = i - NLOC;
                rloc[q] = (q < ADL_NTHV && q >= nthv) ? 0.0 : r[u];
            }
        }
    }
    for (int i = tid; i < 256; i += NT) colb[i >> 7][i & 127] = a.ct->col[i >> 7][i & 127];
    __syncthreads();                                    // psi below reads the staged image
    const double* wts = P + a.n_v;
    const double* cost = P + a.n_v + ADL_NW;
    const double* th = P + a.n_v + ADL_NW + 20;
    const double psi = vloc[ADL_NTHV + kPhiPsi];
    for (int i = tid; i < ADL_NW; i += NT) {
        int ci;
        double nrm;
        bool track = false;
        if (i < ADL_NX || (i >= 119 && i < 122)) { ci = kCostTracking; nrm = a.cst[ADL_C_NORM_TRACKING]; track = true; }
        else if (i < 2 * ADL_NX) { ci = kCostXdotRegularisation; nrm = a.cst[ADL_C_NORM_XDOT_REG]; }
        else if (i < 119) {
            const int u = i - 100;
            const bool fict = (u % 9) < 6 && u < 18;
            ci = fict ? kCostFictitious : kCostURegularisation;
            nrm = a.cst[fict ? ADL_C_NORM_FICTITIOUS : ADL_C_NORM_U_REG];
        } else { ci = kCostThetaRegularisation; nrm = a.cst[ADL_C_NORM_THETA_REG]; }
        double we = wts[i] * cost[ci] / nrm;
        if (i == awe::dl::kTf) we = 0.0;                      // objective.py:132 (t_f exception)
        wef[i] = we;
        wtr[i] = track ? psi * we : we;
    }
    __syncthreads();

    const int tfi = a.single ? (k < a.nkr ? 1 : 2) : 1;
    const double tf = vloc[tfi];
    const double ihtf = (double)a.n_k / tf;
    const double* C = a.coll.C;
    const double* xk = vloc + ADL_NTHV + 7;
    const double* uk = xk + ADL_NX;
    const double* xdk = uk + ADL_NU;
    const double* zk = xdk + ADL_NX;
    const double* coll = zk + ADL_NZ;
    const double* xk1 = coll + D * (ADL_NX + ADL_NZ);
    auto Xv = [&](int r, int i) -> double { return r == 0 ? xk[i] : coll[(r - 1) * (ADL_NX + ADL_NZ) + i]; };
    auto node_theta = [&](const double* tv, int t) -> double {   // [diam_t, t_f(k), l_s, diam_s]
        if (t == 1) return tv[tfi];
        return a.single ? tv[t == 0 ? 0 : t + 1] : tv[t];
    };

    // ---- node values --------------------------------------------------------------------
    for (int t = tid; t < NN * 128; t += NT) {
        const int n = t >> 7, i = t & 127;
        double val = 0.0;
        if (i < ADL_NX) val = Xv(n, i);
        else if (i < 2 * ADL_NX) {
            if (n == 0) val = xdk[i - ADL_NX];
            else {
                double s = 0.0;
                for (int r = 0; r < NN; ++r) s += C[r * NN + n] * Xv(r, i - ADL_NX);
                val = s * ihtf;
            }
        } else if (i < 2 * ADL_NX + ADL_NU) val = uk[i - 2 * ADL_NX];
        else if (i < 2 * ADL_NX + ADL_NU + ADL_NZ) {
            const int z = i - (2 * ADL_NX + ADL_NU);
            val = n == 0 ? zk[z] : coll[(n - 1) * (ADL_NX + ADL_NZ) + ADL_NX + z];
        } else if (i < ADL_NW) val = node_theta(vloc, i - (2 * ADL_NX + ADL_NU + ADL_NZ));
        else if (i == 126) val = vloc[ADL_NTHV];                 // phi.gamma
        wn[n][i] = val;
    }
    for (int t = tid; t < D * ADL_NW; t += NT) {
        const int j = t / ADL_NW, i = t % ADL_NW;
        const double* rl = rloc + ADL_NTHV;
        double val;
        if (i < ADL_NX) val = rl[2 * ADL_NX + ADL_NU + ADL_NZ + j * (ADL_NX + ADL_NZ) + i];
        else if (i < 2 * ADL_NX) val = 0.0;                       // objective.py:186
        else if (i < 2 * ADL_NX + ADL_NU) val = rl[ADL_NX + (i - 2 * ADL_NX)];
        else if (i < 2 * ADL_NX + ADL_NU + ADL_NZ)
            val = rl[2 * ADL_NX + ADL_NU + ADL_NZ + j * (ADL_NX + ADL_NZ) + ADL_NX + (i - (2 * ADL_NX + ADL_NU))];
        else val = node_theta(rloc, i - (2 * ADL_NX + ADL_NU + ADL_NZ));
        rn[j][i] = val;
    }
    __syncthreads();

    // ---- tether drags once per node -------------------------------------------------------
    // stage A: wind and density (values and height derivatives) at every element midpoint,
    // one (node, segment, element) per thread
    const int n_el = (int)a.cst[ADL_C_N_ELEMENTS];
    {
        const double* sc = a.cst + ADL_C_SCALING;
        for (int t = tid; t < NN * 3 * n_el; t += NT) {
            const int n = t / (3 * n_el), sg = (t / n_el) % 3, e = t % n_el;
            const double* wv = wn[n];
            const double qtz = sg == 0 ? wv[awe::dl::kQ10 + 2] * sc[awe::dl::kQ10 + 2]
                                       : wv[awe::dl::q(sg - 1) + 2] * sc[awe::dl::q(sg - 1) + 2];
            const double qbz = sg == 0 ? 0.0 : wv[awe::dl::kQ10 + 2] * sc[awe::dl::kQ10 + 2];
            const double zz = awe::element_height(e, n_el, qbz, qtz);
            const awe::Dual z(zz, 1.0);
            const awe::Dual uw = awe::wind_speed(z, th), rho = awe::isa_density(z, th);
            double* p = &atmo[n][(sg * kMaxElements + e) * 4];
            p[0] = uw.v; p[1] = uw.d; p[2] = rho.v; p[3] = rho.d;
        }
    }
    __syncthreads();
    // stage B: element algebra in dual arithmetic, one SI input direction per thread
    {
        const double* sc = a.cst + ADL_C_SCALING;
        const awe::DualInlineSubmodels inl;
        for (int t = tid; t < NN * kPreThreads; t += NT) {
            const int n = t / kPreThreads, j = t % kPreThreads;
            const double* wv = wn[n];
            const PreAtmosphere atm{atmo[n]};
            auto S = [&](int i, int seed) { return awe::Dual(wv[i] * sc[i], seed ? 1.0 : 0.0); };
            awe::Dual q1[3], v1[3];
            if (j < 7) {
                for (int i = 0; i < 3; ++i) {
                    q1[i] = S(awe::dl::kQ10 + i, j == i);
                    v1[i] = S(awe::dl::kDQ10 + i, j == 3 + i);
                }
                awe::Dual up[3];
                inl.main_drag(q1, v1, S(awe::dl::kDiamT, j == 6), th, a.cst, up, atm);
                for (int i = 0; i < 3; ++i) {
                    pre[n][3 + i * 7 + j] = up[i].d;
                    if (j == 0) pre[n][i] = up[i].v;
                }
            } else {
                const int k = (j - 7) / 13, jj = (j - 7) % 13;
                awe::Dual qk[3], vk[3];
                for (int i = 0; i < 3; ++i) {
                    q1[i] = S(awe::dl::kQ10 + i, jj == i);
                    v1[i] = S(awe::dl::kDQ10 + i, jj == 3 + i);
                    qk[i] = S(awe::dl::q(k) + i, jj == 6 + i);
                    vk[i] = S(awe::dl::dq(k) + i, jj == 9 + i);
                }
                awe::Dual up[3], lo[3];
                inl.sec_drag(k, q1, v1, qk, vk, S(awe::dl::kDiamS, jj == 12), th, a.cst, up, lo, atm);
                double* p = pre[n] + kPreMain + k * kPreSec;
                for (int i = 0; i < 6; ++i) {
                    const awe::Dual& o = i < 3 ? up[i] : lo[i - 3];
                    p[6 + i * 13 + jj] = o.d;
                    if (jj == 0) p[i] = o.v;
                }
            }
        }
    }
    __syncthreads();

    // ---- model pass: one (node, colour) task per thread, packed across the workgroup ----------
    {
        const int n0c = a.ct->ncol[0], n1c = a.ct->ncol[1];
        int n, lane;
        if (tid < n0c) { n = 0; lane = tid; }
        else { n = 1 + (tid - n0c) / n1c; lane = (tid - n0c) % n1c; }
        const int kind = n > 0;
        if (n < NN) {
            const int toff = n == 0 ? 0 : a.ct->tsize[0] + (n - 1) * a.ct->tsize[1];
            DLaneIn in{wn[n], colb[kind], lane, n > 0 ? C[n * NN + n] * ihtf : 0.0,
                       (n > 0 && colb[1][awe::dl::kTf] == lane) ? -1.0 / tf : 0.0};
            DSink sink{tang + toff + a.ct->off[kind][lane], gval[n], &dumpbuf[tid], a.ct->cm_lo[kind][lane],
                       a.ct->cm_hi[kind][lane], lane == 0};
            awe::Dual gamma(wn[n][126], colb[kind][126] == lane ? 1.0 : 0.0);
            awe::dual_node<awe::Dual>(in, gamma, th, a.cst, sink, n == 0, DualPreSubmodels{pre[n]});
        }
    }
    __syncthreads();

    return FrontGeo{tfi, tf, ihtf, psi};
}

template <int D>
__global__ __launch_bounds__(kBlock, ADL_MIN_BLOCKS) void dual_interval_kernel(DArgs a) {
    constexpr int NN = D + 1;
    constexpr int NT = kBlock;
    constexpr int STRIDE = FrontLds<D>::STRIDE;
    __shared__ FrontLds<D> s;
    __shared__ double obj[D][128];
    __shared__ double fterm[D][128];
    extern __shared__ double tang[];            // [tang_total]
    const int b = blockIdx.x / a.n_k, k = blockIdx.x % a.n_k;
    const int tid = threadIdx.x;
    const FrontGeo geo = dual_front<D>(a, s, tang, b, k, tid);
    auto& wtr = s.wtr;
    auto& wef = s.wef;
    auto& wn = s.wn;
    auto& rn = s.rn;
    auto& gval = s.gval;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* cost = P + a.n_v + ADL_NW;
    const double* C = a.coll.C;
    const double tf = geo.tf, ihtf = geo.ihtf, psi = geo.psi;
    const int base = a.v_int0 + k * STRIDE;
    const double* xk = s.vloc + ADL_NTHV + 7;
    const double* coll = xk + ADL_NX + ADL_NU + ADL_NX + ADL_NZ;
    const double* xk1 = coll + D * (ADL_NX + ADL_NZ);
    auto Xv = [&](int r, int i) -> double { return r == 0 ? xk[i] : coll[(r - 1) * (ADL_NX + ADL_NZ) + i]; };

    // ---- objective: directional derivatives at the Radau nodes (objective.py:45-544) ------
    const double T = time_period(V, a);
    const double cb = cost[kCostBeta] / a.cst[ADL_C_NORM_BETA];
    const double* wq_all = a.coll.w;
    for (int t = tid; t < D * 128; t += NT) {
        const int j = t >> 7, dir = t & 127, n = j + 1;
        const double wq = wq_all[j];
        const double* wv = wn[n];
        const double* rv = rn[j];
        const double cxx = C[n * NN + n] * ihtf;
        double acc = 0.0, fterm_v = 0.0;
        if (dir < ADL_NX) {
            acc = 2.0 * wq * (wtr[dir] * (wv[dir] - rv[dir]) + wtr[ADL_NX + dir] * wv[ADL_NX + dir] * cxx);
        } else if (dir < 2 * ADL_NX) {
            acc = 2.0 * wq * wtr[dir] * wv[dir];
        } else if (dir == awe::dl::kTf) {
            for (int i = 0; i < ADL_NX; ++i) acc -= 2.0 * wq * wtr[ADL_NX + i] * wv[ADL_NX + i] * wv[ADL_NX + i] / tf;
        } else if (dir < ADL_NW) {
            acc = 2.0 * wq * wtr[dir] * (wv[dir] - rv[dir]);
        }
        if (dir < ADL_NW) {
            const double e = wv[dir] - rv[dir];
            fterm_v = wq * wef[dir] * e * e;
        }
        if (dir < 127) {
            const int toff = a.ct->tsize[0] + (n - 1) * a.ct->tsize[1];
            const int tp = a.ct->obj_tang[dir][0];
            if (tp >= 0)
                acc += (1.0 - psi) * (-cost[kCostPower]) * (tf / a.n_k) * wq / T * tang[toff + tp];
            for (int kk = 0; kk < 2; ++kk) {
                const int tb = a.ct->obj_tang[dir][1 + kk];
                if (tb >= 0) acc += 2.0 * wq * cb * gval[n][kRowBeta0 + kk] * tang[toff + tb];
            }
        }
        obj[j][dir] = acc;
        fterm[j][dir] = fterm_v;
    }
    __syncthreads();

    // ---- interval partials (fixed order) ---------------------------------------------------
    if (tid == 0) {
        double tr = 0.0, ot = 0.0, A = 0.0, pd[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j = 0; j < D; ++j) {
            const int n = j + 1;
            const double wq = wq_all[j];
            for (int i = 0; i < ADL_NW; ++i) {
                const bool track = i < ADL_NX || (i >= 119 && i < 122);
                if (track) tr += fterm[j][i]; else ot += fterm[j][i];
            }
            ot += wq * cb * (gval[n][kRowBeta0] * gval[n][kRowBeta0] + gval[n][kRowBeta0 + 1] * gval[n][kRowBeta0 + 1]);
            A += wq * gval[n][kRowPower] / a.n_k;
            for (int q = 0; q < 4; ++q) pd[q] += obj[j][122 + q];
        }
        double* pp = a.part + ((size_t)b * a.n_k + k) * kNPart;
        pp[0] = tr; pp[1] = ot; pp[2] = A;
        for (int q = 0; q < 4; ++q) pp[3 + q] = pd[q];
        pp[7] = 0.0;
    }

    // ---- gradient of the interval's own columns ------------------------------------------------
    double* grad = a.grad + (size_t)b * a.n_v + base;
    for (int c = tid; c < STRIDE; c += NT) {
        double gr = 0.0;
        if (c < ADL_NX) {
            for (int m = 1; m < NN; ++m) gr += obj[m - 1][ADL_NX + c] * C[0 * NN + m] * ihtf;
        } else if (c < ADL_NX + ADL_NU) {
            for (int m = 1; m < NN; ++m) gr += obj[m - 1][2 * ADL_NX + (c - ADL_NX)];
        } else if (c >= 2 * ADL_NX + ADL_NU + ADL_NZ) {
            const int q = c - (2 * ADL_NX + ADL_NU + ADL_NZ);
            const int j = q / (ADL_NX + ADL_NZ), e = q % (ADL_NX + ADL_NZ), n = j + 1;
            if (e < ADL_NX) {
                gr = obj[j][e];
                for (int m = 1; m < NN; ++m)
                    if (m != n) gr += obj[m - 1][ADL_NX + e] * C[n * NN + m] * ihtf;
            } else {
                gr = obj[j][2 * ADL_NX + ADL_NU + (e - ADL_NX)];
            }
        }
        grad[c] = gr;
    }
    if (k == a.n_k - 1)
        for (int c = tid; c < ADL_NX; c += NT) grad[STRIDE + c] = 0.0;    // x[n_k]

    // ---- g rows of the interval --------------------------------------------------------------
    double* g = a.g + (size_t)b * a.n_g;
    constexpr int ROWS = ADL_N_EQ + ADL_N_INEQ + D * ADL_N_EQ + ADL_NX;
    const int row0 = k * ROWS;
    const double* Dc = a.coll.D;
    for (int r = tid; r < ROWS; r += NT) {
        double val;
        if (r < ADL_N_EQ + ADL_N_INEQ) val = gval[0][r];
        else if (r < ADL_N_EQ + ADL_N_INEQ + D * ADL_N_EQ) {
            const int q = r - (ADL_N_EQ + ADL_N_INEQ);
            val = gval[1 + q / ADL_N_EQ][q % ADL_N_EQ];
        } else {
            const int i = r - (ADL_N_EQ + ADL_N_INEQ + D * ADL_N_EQ);
            double s = 0.0;
            for (int rr = 0; rr < NN; ++rr) s += Dc[rr] * Xv(rr, i);
            val = xk1[i] - s;
        }
        g[row0 + r] = val;
    }

    // ---- J_g values through the gather list -------------------------------------------------
    // (the entries' codes and slots are fetched 8 per thread at a time before the stores: a loop that
    // loads them per entry waits for each pair of loads behind the previous entry's store)
    double* jac = a.jac + (size_t)b * a.nnz;
    const int e0 = a.goff[k], e1 = a.goff[k + 1];
    for (int eb = e0 + tid; eb < e1; eb += 8 * NT) {
        uint32_t cd[8];
        int sl[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int e = min(eb + u * NT, e1 - 1);
            cd[u] = a.gcode[e];
            sl[u] = a.gslot[e];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (eb + u * NT >= e1) break;
            const uint32_t kind = cd[u] >> 29;
            const int rr = (cd[u] >> 25) & 15, n = (cd[u] >> 21) & 15, idx = cd[u] & ((1u << 21) - 1u);
            double val;
            if (kind == kKindTang) val = tang[idx];
            else if (kind == kKindTangPoly) val = tang[idx] * (C[rr * NN + n] * ihtf);
            else val = a.kconst[idx];
            __builtin_nontemporal_store(val, &jac[sl[u]]);   // written once (as the AP2 path's J_g)
        }
    }
}

// one workgroup per instance: objective partials in a fixed order, power cost over the
// phase-fixed period, time and homotopy costs, global gradient entries, periodicity and t_f rows
__global__ __launch_bounds__(64) void dual_finalize_kernel(DArgs a) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* cost = P + a.n_v + ADL_NW;
    double* grad = a.grad + (size_t)b * a.n_v;
    double* g = a.g + (size_t)b * a.n_g;
    const int nthv = a.n_thv;
    if (lane == 0) {
        const double* pp = a.part + (size_t)b * a.n_k * kNPart;
        double tr = 0.0, ot = 0.0, e_end = 0.0, A0 = 0.0, A1 = 0.0, pdt = 0.0, pls = 0.0, pds = 0.0;
        double ptf0 = 0.0, ptf1 = 0.0;
        for (int k = 0; k < a.n_k; ++k) {
            const double* q = pp + (size_t)k * kNPart;
            const bool ph1 = a.single && k >= a.nkr;
            const double tfk = V[ph1 ? 2 : 1];
            tr += q[0];
            ot += q[1];
            e_end += tfk * q[2];
            if (ph1) { A1 += q[2]; ptf1 += q[4]; } else { A0 += q[2]; ptf0 += q[4]; }
            pdt += q[3]; pls += q[5]; pds += q[6];
        }
        const double T = time_period(V, a);
        const double Tref = time_period(P, a);
        const double psi = V[nthv + kPhiPsi];
        const double cp = cost[kCostPower], ct = cost[kCostTf];
        const double f_power = -cp * e_end / T;
        double f = psi * tr + (1.0 - psi) * f_power + ot + ct * (T - Tref) * (T - Tref);
        for (int i = 0; i < 7; ++i) f += cost[kPhiCost[i]] * V[nthv + i];
        a.f[b] = f;
        const double n0 = a.single ? (double)a.nkr / a.n_k : 1.0, n1 = a.single ? (double)(a.n_k - a.nkr) / a.n_k : 0.0;
        grad[0] = pdt;
        grad[1] = ptf0 + (1.0 - psi) * (-cp) * (A0 * T - e_end * n0) / (T * T) + 2.0 * ct * (T - Tref) * n0;
        if (a.single) {
            grad[2] = ptf1 + (1.0 - psi) * (-cp) * (A1 * T - e_end * n1) / (T * T) + 2.0 * ct * (T - Tref) * n1;
            grad[3] = pls;
            grad[4] = pds;
        } else {
            grad[2] = pls;
            grad[3] = pds;
        }
        for (int i = 0; i < 7; ++i) grad[nthv + i] = cost[kPhiCost[i]] + (i == kPhiPsi ? tr - f_power : 0.0);
        grad[nthv + 7] = 0.0;
        grad[nthv + 8] = 0.0;
        if (a.single) {
            const double frac = a.cst[ADL_C_PHASE_FIX_REELOUT];
            const int gt = a.n_k * (ADL_N_EQ + ADL_N_INEQ + a.d * ADL_N_EQ + ADL_NX) + ADL_NX;
            g[gt] = (T - a.cst[ADL_C_TF_UB]) / frac;
            g[gt + 1] = (a.cst[ADL_C_TF_LB] - T) / frac;
        }
    }
    // periodicity rows, sorted x names (operation.py:245-266)
    const int gp = a.n_k * (ADL_N_EQ + ADL_N_INEQ + a.d * ADL_N_EQ + ADL_NX);
    const int x0 = a.v_int0;
    const int xT = a.v_int0 + (a.n_k - 1) * a.stride + 2 * ADL_NX + ADL_NU + ADL_NZ + (a.d - 1) * (ADL_NX + ADL_NZ);
    for (int i = lane; i < ADL_NX; i += 64) g[gp + i] = V[x0 + kPeriodicOrder[i]] - V[xT + kPeriodicOrder[i]];
}

// =========================================================================================
// Hessian of the Lagrangian sigma f + lam^T g (nlp_hess_l), exact (dual_hess_tables.hpp)
// =========================================================================================
struct HDArgs {
    DArgs a;                       // V, P, tables and sizes of the first-order kernel
    const DHessTabs* ht;
    const int* tasks;              // colour pairs (c1 | c2 << 8) per node kind
    const short* task_target;      // [task][kHRowStride] direction-pair index of each row
    const int* ent_off;            // [n_k + 1]
    const int* term_off;
    const unsigned* terms;
    const int* slot0;
    const int* nslot;
    const int* gslot;
    const int* gcol;
    const int* grow;
    const double* sigma;           // [batch]
    const double* lam;             // [batch][n_g]
    double* H;                     // [batch][nnz_h] upper-triangular CCS values
    double* gpart;                 // [batch][n_k][ng] interval partials of the global entries
    double* apart;                 // [batch][n_k] interval power integrals A_k
    int hnnz, ng, hd_total;
};

// hyper-dual node variable i: e1 along colour c1, e2 along colour c2 (DLaneIn twice)
struct DLaneHIn {
    const double* w;
    const int8_t* col;
    int c1, c2;
    double cxx, t1, t2;
    __device__ __forceinline__ awe::HDual operator()(int i) const {
        double x = (col[i] == c1) ? 1.0 : 0.0;
        double y = (col[i] == c2) ? 1.0 : 0.0;
        if (i >= ADL_NX && i < 2 * ADL_NX) {
            if (col[i - ADL_NX] == c1) x += cxx;
            if (col[i - ADL_NX] == c2) y += cxx;
            x += t1 * w[i];
            y += t2 * w[i];
        }
        return awe::HDual(w[i], x, y, 0.0);
    }
};

// accumulates mu_r d2F_r/de1de2 into the node's direction-pair Hessian (branch-free); the
// colouring makes each (task, row) own its pair slot, so no two threads meet
struct DLaneHSink {
    double* hd;
    double* dump;
    const double* mu;
    const short* tt;
    __device__ __forceinline__ void emit(int r, const awe::HDual& v) {
        const int idx = tt[r];
        double* adr = idx >= 0 ? hd + idx : dump;
        *adr += mu[r] * v.ab;
    }
    __device__ __forceinline__ void eq_row(int r, const awe::HDual& v) { emit(r, v); }
    __device__ __forceinline__ void ineq_row(int r, const awe::HDual& v) { emit(ADL_N_EQ + r, v); }
    __device__ __forceinline__ void power(const awe::HDual& v) { emit(kRowPower, v); }
    __device__ __forceinline__ void beta(int k, const awe::HDual& v) { emit(kRowBeta0 + k, v); }
};

constexpr int kGStride = ADL_NX + 2;      // G[n][i] i < 50, [50] = sum_i G 2 xdot_i / tf^2

// dynamic LDS of the Hessian kernel in doubles after the tangent buffer
template <int D>
constexpr int hess_dyn_fixed_doubles() {
    return (D + 1) * kHRowStride + (D + 1) * kGStride + 40 + 2 * D * 128;
}

template <int D>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
void dual_hess_kernel(HDArgs ha) {
    const DArgs& a = ha.a;
    constexpr int NN = D + 1;
    constexpr int NT = kBlock;
    __shared__ FrontLds<D> s;
    extern __shared__ double dyn[];
    const int b = blockIdx.x / a.n_k, k = blockIdx.x % a.n_k;
    const int tid = threadIdx.x;
    const DHessTabs* ht = ha.ht;
    const ColorTabs* ct = a.ct;
    double* tang = dyn;
    double* hd = tang + a.tang_total;
    double* mu = hd + ha.hd_total;                 // [NN][kHRowStride]
    double* G = mu + NN * kHRowStride;             // [NN][kGStride]
    double* scl = G + NN * kGStride;               // [1 + NN NN]
    double* tfp = scl + 40;                        // [D][128]
    double* gtp = tfp + D * 128;                   // [D][128]
    for (int i = tid; i < ha.hd_total; i += NT) hd[i] = 0.0;
    const FrontGeo geo = dual_front<D>(a, s, tang, b, k, tid);   // ends with a barrier

    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* cost = P + a.n_v + ADL_NW;
    const double* th = P + a.n_v + ADL_NW + 20;
    const double* lam = ha.lam + (size_t)b * a.n_g;
    const double sigma = ha.sigma[b];
    const double* C = a.coll.C;
    const double* wq_all = a.coll.w;
    const double tf = geo.tf, ihtf = geo.ihtf, psi = geo.psi;
    const double inv_tf = 1.0 / tf;
    const double T = time_period(V, a);
    const double cp = cost[kCostPower];
    const double cb = cost[kCostBeta] / a.cst[ADL_C_NORM_BETA];
    const bool ph1 = a.single && k >= a.nkr;
    const double n_own = a.single ? (ph1 ? (double)(a.n_k - a.nkr) / a.n_k : (double)a.nkr / a.n_k) : 1.0;
    const double n_oth = a.single ? 1.0 - n_own : 0.0;
    constexpr int ROWS = ADL_N_EQ + ADL_N_INEQ + D * ADL_N_EQ + ADL_NX;
    auto toff = [&](int n) { return n == 0 ? 0 : ct->tsize[0] + (n - 1) * ct->tsize[1]; };
    auto hoff = [&](int n) { return n == 0 ? 0 : ht->npairs[0] + (n - 1) * ht->npairs[1]; };

    // ---- row weights: lam for constraint rows, sigma-scaled objective weights -----------------
    for (int t = tid; t < NN * kHRowStride; t += NT) {
        const int n = t / kHRowStride, r = t % kHRowStride;
        double m = 0.0;
        if (n == 0) {
            if (r < kRowPower) m = lam[k * ROWS + r];
        } else {
            const double wq = wq_all[n - 1];
            if (r < ADL_N_EQ) m = lam[k * ROWS + ADL_N_EQ + ADL_N_INEQ + (n - 1) * ADL_N_EQ + r];
            else if (r == kRowPower) m = sigma * (1.0 - psi) * (-cp) * wq * tf / ((double)a.n_k * T);
            else if (r == kRowBeta0 || r == kRowBeta0 + 1) m = sigma * 2.0 * wq * cb * s.gval[n][r];
        }
        mu[t] = m;
    }
    for (int i = tid; i < 1 + NN * NN; i += NT) scl[i] = i == 0 ? 1.0 : C[i - 1] * ihtf;
    __syncthreads();

    // ---- second-order pass: one (node, colour pair) per thread ---------------------------------
    const int nt0 = ht->ntask[0], nt1 = ht->ntask[1];
    for (int t = tid; t < nt0 + D * nt1; t += NT) {
        const int n = t < nt0 ? 0 : 1 + (t - nt0) / nt1;
        const int kind = n > 0 ? 1 : 0;
        const int ti = (kind == 0 ? t : (t - nt0) % nt1) + ht->task_off[kind];
        const int task = ha.tasks[ti];
        const int c1 = task & 0xff, c2 = task >> 8;
        const int ctf = s.colb[1][awe::dl::kTf];
        DLaneHIn in{s.wn[n], s.colb[kind], c1, c2, n > 0 ? C[n * NN + n] * ihtf : 0.0,
                    (n > 0 && c1 == ctf) ? -inv_tf : 0.0, (n > 0 && c2 == ctf) ? -inv_tf : 0.0};
        DLaneHSink sink{hd + hoff(n), &s.dumpbuf[tid], mu + n * kHRowStride, ha.task_target + (size_t)ti * kHRowStride};
        const int8_t cg = s.colb[kind][awe::dl::kGamma];
        const awe::HDual gamma(s.wn[n][awe::dl::kGamma], cg == c1 ? 1.0 : 0.0, cg == c2 ? 1.0 : 0.0, 0.0);
        awe::dual_node<awe::HDual>(in, gamma, th, a.cst, sink, n == 0);
    }
    __syncthreads();

    // ---- objective terms in direction space and the xdot(t_f) map terms (Radau nodes) --------
    for (int t = tid; t < D * 128; t += NT) {
        const int j = t >> 7, p = t & 127, n = j + 1;
        const double wq = wq_all[j];
        const double* w = s.wn[n];
        const double* rv = s.rn[j];
        const double cxx = C[n * NN + n] * ihtf;
        const double* tp = tang + toff(n);
        double* hn = hd + hoff(n);
        auto addp = [&](int q1, int q2, double v) { hn[ht->pidx[1][q1][q2]] += sigma * v; };
        double tfpart = 0.0, gt = 0.0;
        if (p < ADL_NX) {
            const double ai = s.wef[p], bi = s.wef[ADL_NX + p], xd = w[ADL_NX + p];
            addp(p, p, 2.0 * wq * psi * ai + cxx * cxx * 2.0 * wq * bi);
            addp(p, ADL_NX + p, cxx * 2.0 * wq * bi);
            addp(p, awe::dl::kTf, cxx * (-xd * inv_tf) * 2.0 * wq * bi);
            addp(p, kHDirPsi, 2.0 * wq * ai * (w[p] - rv[p]));
        } else if (p < 2 * ADL_NX) {
            const int i = p - ADL_NX;
            const double bi = s.wef[p], xd = w[p];
            addp(p, p, 2.0 * wq * bi);
            addp(p, awe::dl::kTf, (-xd * inv_tf) * 2.0 * wq * bi);
            tfpart = (xd * inv_tf) * (xd * inv_tf) * 2.0 * wq * bi;
            // gradient of the node Lagrangian w.r.t. xdot_i: rows (first-order tangents) + objective
            double gi = sigma * wq * 2.0 * bi * xd;
            const int c = s.colb[1][p];
            if (c >= 0) {
                const uint64_t cl = ct->cm_lo[1][c], chh = ct->cm_hi[1][c];
                const double* tc = tp + ct->off[1][c];
                for (uint64_t mm = ht->dm_lo[1][p]; mm; mm &= mm - 1ull) {
                    const int r = __builtin_ctzll(mm);
                    gi += mu[n * kHRowStride + r] * tc[__popcll(cl & ((1ull << r) - 1ull))];
                }
                for (uint64_t mm = ht->dm_hi[1][p]; mm; mm &= mm - 1ull) {
                    const int r = __builtin_ctzll(mm);
                    gi += mu[n * kHRowStride + 64 + r] * tc[__popcll(cl) + __popcll(chh & ((1ull << r) - 1ull))];
                }
            }
            G[n * kGStride + i] = gi;
            gt = gi * 2.0 * xd * inv_tf * inv_tf;
        } else if (p < 2 * ADL_NX + ADL_NU) {
            addp(p, p, 2.0 * wq * s.wef[p]);
        } else if (p < 2 * ADL_NX + ADL_NU + ADL_NZ) {                  // lambda: tracked
            addp(p, p, 2.0 * wq * psi * s.wef[p]);
            addp(p, kHDirPsi, 2.0 * wq * s.wef[p] * (w[p] - rv[p]));
        } else if (p < ADL_NW) {
            addp(p, p, 2.0 * wq * s.wef[p]);                             // theta (t_f weight is 0)
        }
        if (p < kDirs) {
            const int ip = ct->obj_tang[p][0];
            if (ip >= 0) {                                               // power cost over the period
                const double tpv = tp[ip];
                const double c0 = (-cp) * wq / (double)a.n_k;
                addp(p, kHDirPsi, -c0 * tf / T * tpv);
                addp(p, awe::dl::kTf, (1.0 - psi) * c0 * (1.0 / T - tf * n_own / (T * T)) * tpv);
                if (a.single) addp(p, kHDirTfOther, (1.0 - psi) * c0 * (-tf * n_oth / (T * T)) * tpv);
            }
            for (int kk = 0; kk < 2; ++kk) {                             // beta cost: Gauss-Newton part
                const int ib = ct->obj_tang[p][1 + kk];
                if (ib < 0) continue;
                const double bp = 2.0 * cb * wq * tp[ib];
                for (int q = p; q < kDirs; ++q) {
                    const int iq = ct->obj_tang[q][1 + kk];
                    if (iq >= 0) addp(p, q, bp * tp[iq]);
                }
            }
        }
        tfp[t] = tfpart;
        gtp[t] = gt;
    }
    __syncthreads();
    if (tid < D) {                                                       // fixed-order reductions
        const int n = tid + 1;
        double a1 = 0.0, a2 = 0.0;
        for (int p = 0; p < 128; ++p) { a1 += tfp[tid * 128 + p]; a2 += gtp[tid * 128 + p]; }
        hd[hoff(n) + ht->pidx[1][awe::dl::kTf][awe::dl::kTf]] += sigma * a1;
        G[n * kGStride + ADL_NX] = a2;
    }
    if (tid == 64) {                                                     // power integral A_k
        double A = 0.0;
        for (int j = 0; j < D; ++j) A += wq_all[j] * s.gval[j + 1][kRowPower] / a.n_k;
        ha.apart[(size_t)b * a.n_k + k] = A;
    }
    __syncthreads();

    // ---- V-space entries: local CCS slots (contiguous) and the global-global partials ---------
    const int nloc = ha.nslot[k];
    const int e0 = ha.ent_off[k];
    const double ctf2 = ihtf * inv_tf;
    double* Hb = ha.H + (size_t)b * ha.hnnz + ha.slot0[k];
    double* gp = ha.gpart + ((size_t)b * a.n_k + k) * ha.ng;
    for (int e = tid; e < nloc + ha.ng; e += NT) {
        double v = 0.0;
        for (int t = ha.term_off[e0 + e]; t < ha.term_off[e0 + e + 1]; ++t) {
            const unsigned term = ha.terms[t];
            const int type = term >> 30, n = (term >> 27) & 7;
            if (type == kHTypeA) {
                v += scl[(term >> 7) & 127] * scl[term & 127] * hd[hoff(n) + ((term >> 14) & 8191)];
            } else if (type == kHTypeB) {
                const int i = (term >> 21) & 63, r = (term >> 18) & 7;
                v += G[n * kGStride + i] * (-C[r * NN + n] * ctf2);
            } else {
                v += G[n * kGStride + ADL_NX];
            }
        }
        if (e < nloc) Hb[e] = v;
        else gp[e - nloc] = v;
    }
}

// global-global entries: sum of the interval partials in a fixed order, plus the power cost over
// the phase-fixed period and the time cost, which couple the t_f globals (objective.py,
// ocp_outputs.py:118-140): with E = sum_k tf_k A_k, T = n0 tf0 + n1 tf1,
//   f_p = -c_p E / T,  d2(E/T)/dtf_i dtf_j = -(A_i n_j + A_j n_i) / T^2 + 2 E n_i n_j / T^3
__global__ __launch_bounds__(64) void dual_hess_finalize_kernel(HDArgs ha) {
    const DArgs& a = ha.a;
    const int b = blockIdx.x;
    const int g = threadIdx.x;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* cost = a.P + (size_t)b * a.n_p + a.n_v + ADL_NW;
    for (int q = g; q < ha.ng; q += 64) {
        double v = 0.0;
        for (int k = 0; k < a.n_k; ++k) v += ha.gpart[((size_t)b * a.n_k + k) * ha.ng + q];
        const int col = ha.gcol[q], row = ha.grow[q];
        const int ntf = a.single ? 2 : 1;
        const bool tf_row = row >= 1 && row <= ntf;
        const bool tf_col = col >= 1 && col <= ntf;
        const bool psi_col = col == a.n_thv + kPhiPsi;
        if (tf_row && (tf_col || psi_col)) {
            double A[2] = {0.0, 0.0}, E = 0.0;
            for (int k = 0; k < a.n_k; ++k) {
                const int ph = (a.single && k >= a.nkr) ? 1 : 0;
                const double Ak = ha.apart[(size_t)b * a.n_k + k];
                A[ph] += Ak;
                E += V[1 + ph] * Ak;
            }
            const double nn[2] = {a.single ? (double)a.nkr / a.n_k : 1.0,
                                  a.single ? (double)(a.n_k - a.nkr) / a.n_k : 0.0};
            const double T = time_period(V, a);
            const double psi = V[a.n_thv + kPhiPsi];
            const double cp = cost[kCostPower], ct = cost[kCostTf];
            const double sigma = ha.sigma[b];
            const int i = row - 1;
            if (tf_col) {
                const int j = col - 1;
                const double d2 = -(A[i] * nn[j] + A[j] * nn[i]) / (T * T) + 2.0 * E * nn[i] * nn[j] / (T * T * T);
                v += sigma * ((1.0 - psi) * (-cp) * d2 + 2.0 * ct * nn[i] * nn[j]);
            } else {
                v += sigma * cp * (A[i] / T - E * nn[i] / (T * T));
            }
        }
        ha.H[(size_t)b * ha.hnnz + ha.gslot[q]] = v;
    }
}

template <int D>
int launch_hess(const HDArgs& ha, int batch, size_t dyn, hipStream_t s) {
    // the LDS image (tangents + direction-pair Hessian) exceeds 64 KiB: raise the dynamic limit
    ADL_TRY(hipFuncSetAttribute((const void*)dual_hess_kernel<D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));
    dual_hess_kernel<D><<<dim3((unsigned)(batch * ha.a.n_k)), kBlock, dyn, s>>>(ha);
    return 0;
}

template <int D>
int launch(const DArgs& a, int batch, size_t dyn, hipStream_t s) {
    dual_interval_kernel<D><<<dim3((unsigned)(batch * a.n_k)), kBlock, dyn, s>>>(a);
    return 0;
}

}  // namespace

struct adl_handle_s {
    Tables t;
    int batch = 0;
    std::vector<double> consts;
    double* d_cst = nullptr;
    ColorTabs* d_ct = nullptr;
    int* d_goff = nullptr;
    int* d_gslot = nullptr;
    uint32_t* d_gcode = nullptr;
    double* d_part = nullptr;
    double *d_V = nullptr, *d_P = nullptr, *d_f = nullptr, *d_g = nullptr, *d_grad = nullptr, *d_jac = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool timed = false;
    // Hessian (built on first use)
    DualHessTables* ht = nullptr;
    DHessTabs* d_ht = nullptr;
    int *d_tasks = nullptr, *d_ent_off = nullptr, *d_term_off = nullptr, *d_slot0 = nullptr, *d_nslot = nullptr;
    int *d_hgslot = nullptr, *d_gcol = nullptr, *d_grow = nullptr;
    short* d_task_target = nullptr;
    unsigned* d_terms = nullptr;
    double *d_gpart = nullptr, *d_apart = nullptr;
    double *d_hV = nullptr, *d_hP = nullptr, *d_sigma = nullptr, *d_lam = nullptr, *d_H = nullptr;   // host-entry scratch
    int hd_total = 0;
    size_t hess_dyn = 0;
    hipEvent_t hev[2] = {nullptr, nullptr};
    bool htimed = false;
    // generated instance-minor path (adl_eval_nlp_im, awedual_gen.hip)
    dgen::Plan* gen = nullptr;
    std::string gen_why;
};

static DArgs make_args(adl_handle h, const double* V, const double* P) {
    const Tables& T = h->t;
    const Layout& L = T.lay;
    DArgs a{};
    a.V = V; a.P = P; a.cst = h->d_cst;
    for (int j = 0; j <= L.d; ++j) {
        for (int r = 0; r <= L.d; ++r) a.coll.C[j * (L.d + 1) + r] = T.coll.C[j][r];
        a.coll.D[j] = T.coll.D[j];
    }
    for (int j = 0; j < L.d; ++j) a.coll.w[j] = T.coll.w[j];
    a.ct = h->d_ct; a.goff = h->d_goff; a.gslot = h->d_gslot; a.gcode = h->d_gcode;
    for (size_t q = 0; q < T.kconst.size(); ++q) a.kconst[q] = T.kconst[q];
    a.part = h->d_part;
    a.n_k = L.n_k; a.d = L.d; a.n_v = L.n_v; a.n_g = L.n_g; a.n_p = L.n_p; a.nnz = (int)T.row.size();
    a.stride = L.stride; a.v_int0 = L.v_int0; a.nkr = L.nk_reelout; a.single = L.single; a.n_thv = L.n_thv;
    a.tang_total = T.tang_total;
    return a;
}

static size_t hess_dyn_fixed(int d) {
    switch (d) {
        case 2: return hess_dyn_fixed_doubles<2>();
        case 3: return hess_dyn_fixed_doubles<3>();
        case 4: return hess_dyn_fixed_doubles<4>();
        default: return hess_dyn_fixed_doubles<5>();
    }
}

// builds and uploads the Hessian tables on first use
static int ensure_hess(adl_handle h) {
    if (h->ht) return AWE_OK;
    auto* H = new DualHessTables();
    std::string err;
    if (build_dual_hess_tables(h->t, h->consts.data(), *H, err)) {
        delete H;
        return fail(AWE_ERR_ARG, err);
    }
    const Tables& T = h->t;
    h->hd_total = H->ht.npairs[0] + T.lay.d * H->ht.npairs[1];
    h->hess_dyn = sizeof(double) * ((size_t)T.tang_total + h->hd_total + hess_dyn_fixed(T.lay.d));
    if (h->hess_dyn > 110 * 1024) {
        delete H;
        return fail(AWE_ERR_ARG, "internal: Hessian LDS image exceeds the workgroup budget");
    }
    h->ht = H;
    const size_t nb = (size_t)h->batch, ng = H->gslot.size();
#define ADL_UPLOAD(dst, src, n)                                                      \
    ADL_TRY(hipMalloc((void**)&dst, sizeof(*dst) * (n)));                            \
    ADL_TRY(hipMemcpy(dst, src, sizeof(*dst) * (n), hipMemcpyHostToDevice));
    ADL_UPLOAD(h->d_ht, &H->ht, 1);
    ADL_UPLOAD(h->d_tasks, H->tasks.data(), H->tasks.size());
    ADL_UPLOAD(h->d_task_target, H->task_target.data(), H->task_target.size());
    ADL_UPLOAD(h->d_ent_off, H->ent_off.data(), H->ent_off.size());
    ADL_UPLOAD(h->d_term_off, H->term_off.data(), H->term_off.size());
    ADL_UPLOAD(h->d_terms, H->terms.data(), H->terms.size());
    ADL_UPLOAD(h->d_slot0, H->slot0.data(), H->slot0.size());
    ADL_UPLOAD(h->d_nslot, H->nslot.data(), H->nslot.size());
    ADL_UPLOAD(h->d_hgslot, H->gslot.data(), ng);
    ADL_UPLOAD(h->d_gcol, H->gcol.data(), ng);
    ADL_UPLOAD(h->d_grow, H->grow.data(), ng);
#undef ADL_UPLOAD
    ADL_TRY(hipMalloc((void**)&h->d_gpart, sizeof(double) * nb * T.lay.n_k * std::max<size_t>(ng, 1)));
    ADL_TRY(hipMalloc((void**)&h->d_apart, sizeof(double) * nb * T.lay.n_k));
    for (auto& e : h->hev) ADL_TRY(hipEventCreate(&e));
    return AWE_OK;
}

static int launch_hess_all(adl_handle h, const double* V, const double* P, const double* sigma, const double* lam,
                           double* Hv, hipStream_t s) {
    const DualHessTables& H = *h->ht;
    HDArgs ha{};
    ha.a = make_args(h, V, P);
    ha.ht = h->d_ht; ha.tasks = h->d_tasks; ha.task_target = h->d_task_target;
    ha.ent_off = h->d_ent_off; ha.term_off = h->d_term_off; ha.terms = h->d_terms;
    ha.slot0 = h->d_slot0; ha.nslot = h->d_nslot; ha.gslot = h->d_hgslot; ha.gcol = h->d_gcol; ha.grow = h->d_grow;
    ha.sigma = sigma; ha.lam = lam; ha.H = Hv; ha.gpart = h->d_gpart; ha.apart = h->d_apart;
    ha.hnnz = H.nnz; ha.ng = (int)H.gslot.size(); ha.hd_total = h->hd_total;
    int rc = 0;
    ADL_TRY(hipEventRecord(h->hev[0], s));
    switch (h->t.lay.d) {
        case 2: rc = launch_hess<2>(ha, h->batch, h->hess_dyn, s); break;
        case 3: rc = launch_hess<3>(ha, h->batch, h->hess_dyn, s); break;
        case 4: rc = launch_hess<4>(ha, h->batch, h->hess_dyn, s); break;
        case 5: rc = launch_hess<5>(ha, h->batch, h->hess_dyn, s); break;
        default: return fail(AWE_ERR_ARG, "unsupported d");
    }
    if (rc) return rc;
    ADL_TRY(hipGetLastError());
    dual_hess_finalize_kernel<<<dim3((unsigned)h->batch), 64, 0, s>>>(ha);
    ADL_TRY(hipGetLastError());
    ADL_TRY(hipEventRecord(h->hev[1], s));
    h->htimed = true;
    return AWE_OK;
}

extern "C" {

const char* adl_last_error(void) { return g_err.c_str(); }

int adl_sparsity_jac_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind, int* row) {
    if (!consts || !nnz) return fail(AWE_ERR_ARG, "null argument");
    Tables T;
    std::string err;
    if (build_tables(n_k, d, consts, n_consts, T, err)) return fail(AWE_ERR_ARG, err);
    *nnz = (int)T.row.size();
    if (colind) std::memcpy(colind, T.colind.data(), sizeof(int) * T.colind.size());
    if (row) std::memcpy(row, T.row.data(), sizeof(int) * T.row.size());
    return AWE_OK;
}

int adl_colour_counts(int n_k, int d, const double* consts, int n_consts, int* n_col_shoot, int* n_col_radau,
                      int* tang_shoot, int* tang_radau) {
    if (!consts) return fail(AWE_ERR_ARG, "null argument");
    Tables T;
    std::string err;
    if (build_tables(n_k, d, consts, n_consts, T, err)) return fail(AWE_ERR_ARG, err);
    if (n_col_shoot) *n_col_shoot = T.ct.ncol[0];
    if (n_col_radau) *n_col_radau = T.ct.ncol[1];
    if (tang_shoot) *tang_shoot = T.ct.tsize[0];
    if (tang_radau) *tang_radau = T.ct.tsize[1];
    return AWE_OK;
}

// Diagnostics (CPU, no device): value and full Jacobian of one node of the model, one direction
// at a time in dual arithmetic.  w[ADL_NW + 1] (last = phi.gamma), th[AWE_NTHETA0];
// val[75] = [eq 53, ineq 19, power, beta2, beta3]; jac[75 * 127] row-major.
int adl_node_eval_host(const double* w, const double* th, const double* consts, int n_consts, double* val,
                       double* jac) {
    if (!w || !th || !consts || !val || !jac) return fail(AWE_ERR_ARG, "null argument");
    if (n_consts != ADL_NCONST) return fail(AWE_ERR_ARG, "consts must have ADL_NCONST entries");
    struct In {
        const double* w;
        int dir;
        awe::Dual operator()(int i) const { return awe::Dual(w[i], i == dir ? 1.0 : 0.0); }
    };
    struct Sink {
        awe::Dual rows[kNRows];
        void eq_row(int r, const awe::Dual& v) { rows[r] = v; }
        void ineq_row(int r, const awe::Dual& v) { rows[ADL_N_EQ + r] = v; }
        void power(const awe::Dual& v) { rows[kRowPower] = v; }
        void beta(int k, const awe::Dual& v) { rows[kRowBeta0 + k] = v; }
    };
    for (int dir = 0; dir < kDirs; ++dir) {
        Sink s;
        awe::dual_node<awe::Dual>(In{w, dir}, awe::Dual(w[ADL_NW], dir == ADL_NW ? 1.0 : 0.0), th, consts, s, true);
        for (int r = 0; r < kNRows; ++r) {
            jac[r * kDirs + dir] = s.rows[r].d;
            if (dir == 0) val[r] = s.rows[r].v;
        }
    }
    return AWE_OK;
}

int adl_create(int n_k, int d, const double* consts, int n_consts, int batch, adl_handle* out) {
    if (!consts || !out || batch < 1) return fail(AWE_ERR_ARG, "bad argument");
    if (d < 2 || d > 5) return fail(AWE_ERR_ARG, "the dual-kite kernel is instantiated for 2 <= d <= 5");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(AWE_ERR_NODEVICE, "no HIP device");
    auto* h = new adl_handle_s();
    std::string err;
    if (build_tables(n_k, d, consts, n_consts, h->t, err)) {
        delete h;
        return fail(AWE_ERR_ARG, err);
    }
    const Tables& T = h->t;
    if (T.ct.ncol[0] + d * T.ct.ncol[1] > kBlock) {
        delete h;
        return fail(AWE_ERR_ARG, "more (node, colour) tasks than threads per workgroup");
    }
    if ((int)consts[ADL_C_N_ELEMENTS] > kMaxElements) {
        delete h;
        return fail(AWE_ERR_ARG, "the dual-kite kernel supports at most 8 tether elements per segment");
    }
    if (T.gslot.size() >= (1u << 31) || T.tang_total >= (1 << 21)) {
        delete h;
        return fail(AWE_ERR_ARG, "tables exceed the gather-code range");
    }
    h->batch = batch;
    h->consts.assign(consts, consts + n_consts);
#define ADL_UPLOAD(dst, src, n)                                                      \
    ADL_TRY(hipMalloc((void**)&dst, sizeof(*dst) * (n)));                            \
    ADL_TRY(hipMemcpy(dst, src, sizeof(*dst) * (n), hipMemcpyHostToDevice));
    ADL_UPLOAD(h->d_cst, consts, n_consts);
    ADL_UPLOAD(h->d_ct, &T.ct, 1);
    ADL_UPLOAD(h->d_goff, T.goff.data(), T.goff.size());
    ADL_UPLOAD(h->d_gslot, T.gslot.data(), T.gslot.size());
    ADL_UPLOAD(h->d_gcode, T.gcode.data(), T.gcode.size());
#undef ADL_UPLOAD
    ADL_TRY(hipMalloc((void**)&h->d_part, sizeof(double) * (size_t)batch * n_k * kNPart));
    for (auto& e : h->ev) ADL_TRY(hipEventCreate(&e));
    if (int rc = dgen::create(T, h->consts, batch, &h->gen, h->gen_why, err)) {
        adl_destroy(h);
        return fail(rc, err);
    }
    *out = h;
    return AWE_OK;
}

int adl_destroy(adl_handle h) {
    if (!h) return AWE_OK;
    void* bufs[] = {h->d_cst, h->d_ct, h->d_goff, h->d_gslot, h->d_gcode, h->d_part,
                    h->d_V, h->d_P, h->d_f, h->d_g, h->d_grad, h->d_jac,
                    h->d_ht, h->d_tasks, h->d_ent_off, h->d_term_off, h->d_slot0, h->d_nslot, h->d_hgslot,
                    h->d_gcol, h->d_grow, h->d_task_target, h->d_terms, h->d_gpart, h->d_apart,
                    h->d_hV, h->d_hP, h->d_sigma, h->d_lam, h->d_H};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : h->hev)
        if (e) (void)hipEventDestroy(e);
    delete h->ht;
    dgen::destroy(h->gen);
    delete h;
    return AWE_OK;
}

int adl_gen_status(adl_handle h, int* available) {
    if (!h || !available) return fail(AWE_ERR_ARG, "null argument");
    *available = h->gen ? 1 : 0;
    if (!h->gen) g_err = h->gen_why;
    return AWE_OK;
}

int adl_eval_nlp_im(adl_handle h, const double* V, const double* P, double* f, double* g, double* grad_f, double* jac,
                    size_t ld, void* stream) {
    if (!h || !V || !P || !f || !g || !grad_f || !jac) return fail(AWE_ERR_ARG, "null argument");
    if (!h->gen) return fail(AWE_ERR_ARG, "generated path unavailable: " + h->gen_why);
    std::string err;
    if (int rc = dgen::eval(h->gen, h->d_cst, V, P, f, g, grad_f, jac, ld, (hipStream_t)stream, err))
        return fail(rc, err);
    return AWE_OK;
}

int adl_last_kernel_ms_im(adl_handle h, float* ms_in, float* ms_node, float* ms_interval, float* ms_fin) {
    if (!h || !h->gen) return fail(AWE_ERR_ARG, "no generated path");
    float ms[4];
    std::string err;
    if (int rc = dgen::last_ms(h->gen, ms, err)) return fail(rc, err);
    if (ms_in) *ms_in = ms[0];
    if (ms_node) *ms_node = ms[1];
    if (ms_interval) *ms_interval = ms[2];
    if (ms_fin) *ms_fin = ms[3];
    return AWE_OK;
}

int adl_sizes(adl_handle h, int* n_v, int* n_g, int* n_p, int* nnz) {
    if (!h) return fail(AWE_ERR_ARG, "null handle");
    if (n_v) *n_v = h->t.lay.n_v;
    if (n_g) *n_g = h->t.lay.n_g;
    if (n_p) *n_p = h->t.lay.n_p;
    if (nnz) *nnz = (int)h->t.row.size();
    return AWE_OK;
}

int adl_sparsity_jac(adl_handle h, int* colind, int* row) {
    if (!h || !colind || !row) return fail(AWE_ERR_ARG, "null argument");
    std::memcpy(colind, h->t.colind.data(), sizeof(int) * h->t.colind.size());
    std::memcpy(row, h->t.row.data(), sizeof(int) * h->t.row.size());
    return AWE_OK;
}

int adl_eval_nlp(adl_handle h, const double* V, const double* P, double* f, double* g, double* grad_f, double* jac,
                 void* stream) {
    if (!h || !V || !P || !f || !g || !grad_f || !jac) return fail(AWE_ERR_ARG, "null argument");
    const Tables& T = h->t;
    const Layout& L = T.lay;
    hipStream_t s = (hipStream_t)stream;
    DArgs a = make_args(h, V, P);
    a.f = f; a.g = g; a.grad = grad_f; a.jac = jac;
    const size_t dyn = sizeof(double) * (size_t)T.tang_total;
    ADL_TRY(hipEventRecord(h->ev[0], s));
    switch (L.d) {
        case 2: launch<2>(a, h->batch, dyn, s); break;
        case 3: launch<3>(a, h->batch, dyn, s); break;
        case 4: launch<4>(a, h->batch, dyn, s); break;
        case 5: launch<5>(a, h->batch, dyn, s); break;
        default: return fail(AWE_ERR_ARG, "unsupported d");
    }
    ADL_TRY(hipGetLastError());
    ADL_TRY(hipEventRecord(h->ev[1], s));
    dual_finalize_kernel<<<dim3((unsigned)h->batch), 64, 0, s>>>(a);
    ADL_TRY(hipGetLastError());
    ADL_TRY(hipEventRecord(h->ev[2], s));
    h->timed = true;
    return AWE_OK;
}

int adl_last_kernel_ms(adl_handle h, float* ms_main, float* ms_fin) {
    if (!h || !h->timed) return fail(AWE_ERR_ARG, "no timed evaluation yet");
    ADL_TRY(hipEventSynchronize(h->ev[2]));
    if (ms_main) ADL_TRY(hipEventElapsedTime(ms_main, h->ev[0], h->ev[1]));
    if (ms_fin) ADL_TRY(hipEventElapsedTime(ms_fin, h->ev[1], h->ev[2]));
    return AWE_OK;
}

int adl_eval_nlp_host(adl_handle h, const double* V, const double* P, double* f, double* g, double* grad_f,
                      double* jac) {
    if (!h || !V || !P || !f || !g || !grad_f || !jac) return fail(AWE_ERR_ARG, "null argument");
    const Layout& L = h->t.lay;
    const size_t nb = (size_t)h->batch, nnz = h->t.row.size();
    if (!h->d_V) {
        ADL_TRY(hipMalloc((void**)&h->d_V, sizeof(double) * nb * L.n_v));
        ADL_TRY(hipMalloc((void**)&h->d_P, sizeof(double) * nb * L.n_p));
        ADL_TRY(hipMalloc((void**)&h->d_f, sizeof(double) * nb));
        ADL_TRY(hipMalloc((void**)&h->d_g, sizeof(double) * nb * L.n_g));
        ADL_TRY(hipMalloc((void**)&h->d_grad, sizeof(double) * nb * L.n_v));
        ADL_TRY(hipMalloc((void**)&h->d_jac, sizeof(double) * nb * nnz));
    }
    ADL_TRY(hipMemcpy(h->d_V, V, sizeof(double) * nb * L.n_v, hipMemcpyHostToDevice));
    ADL_TRY(hipMemcpy(h->d_P, P, sizeof(double) * nb * L.n_p, hipMemcpyHostToDevice));
    int rc = adl_eval_nlp(h, h->d_V, h->d_P, h->d_f, h->d_g, h->d_grad, h->d_jac, nullptr);
    if (rc) return rc;
    ADL_TRY(hipDeviceSynchronize());
    ADL_TRY(hipMemcpy(f, h->d_f, sizeof(double) * nb, hipMemcpyDeviceToHost));
    ADL_TRY(hipMemcpy(g, h->d_g, sizeof(double) * nb * L.n_g, hipMemcpyDeviceToHost));
    ADL_TRY(hipMemcpy(grad_f, h->d_grad, sizeof(double) * nb * L.n_v, hipMemcpyDeviceToHost));
    ADL_TRY(hipMemcpy(jac, h->d_jac, sizeof(double) * nb * nnz, hipMemcpyDeviceToHost));
    auto finite = [](const double* x, size_t n) {
        for (size_t i = 0; i < n; ++i)
            if (!std::isfinite(x[i])) return false;
        return true;
    };
    if (!finite(f, nb) || !finite(g, nb * L.n_g) || !finite(grad_f, nb * L.n_v) || !finite(jac, nb * nnz))
        return fail(AWE_ERR_NONFINITE, "non-finite output");
    return AWE_OK;
}

int adl_hess_nnz(adl_handle h, int* nnz_h) {
    if (!h || !nnz_h) return fail(AWE_ERR_ARG, "null argument");
    int rc = ensure_hess(h);
    if (rc) return rc;
    *nnz_h = h->ht->nnz;
    return AWE_OK;
}

int adl_sparsity_hess(adl_handle h, int* colind, int* row) {
    if (!h || !colind || !row) return fail(AWE_ERR_ARG, "null argument");
    int rc = ensure_hess(h);
    if (rc) return rc;
    std::memcpy(colind, h->ht->colind.data(), sizeof(int) * h->ht->colind.size());
    std::memcpy(row, h->ht->row.data(), sizeof(int) * h->ht->row.size());
    return AWE_OK;
}

int adl_sparsity_hess_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind, int* row) {
    if (!consts || !nnz) return fail(AWE_ERR_ARG, "null argument");
    Tables T;
    std::string err;
    if (build_tables(n_k, d, consts, n_consts, T, err)) return fail(AWE_ERR_ARG, err);
    auto* H = new DualHessTables();
    if (build_dual_hess_tables(T, consts, *H, err)) {
        delete H;
        return fail(AWE_ERR_ARG, err);
    }
    *nnz = H->nnz;
    if (colind) std::memcpy(colind, H->colind.data(), sizeof(int) * H->colind.size());
    if (row) std::memcpy(row, H->row.data(), sizeof(int) * H->row.size());
    delete H;
    return AWE_OK;
}

int adl_eval_hess(adl_handle h, const double* V, const double* P, const double* sigma, const double* lam_g,
                  double* H, void* stream) {
    if (!h || !V || !P || !sigma || !lam_g || !H) return fail(AWE_ERR_ARG, "null argument");
    int rc = ensure_hess(h);
    if (rc) return rc;
    return launch_hess_all(h, V, P, sigma, lam_g, H, (hipStream_t)stream);
}

int adl_eval_hess_host(adl_handle h, const double* V, const double* P, const double* sigma, const double* lam_g,
                       double* H) {
    if (!h || !V || !P || !sigma || !lam_g || !H) return fail(AWE_ERR_ARG, "null argument");
    int rc = ensure_hess(h);
    if (rc) return rc;
    const Layout& L = h->t.lay;
    const size_t nb = (size_t)h->batch, hn = (size_t)h->ht->nnz;
    if (!h->d_H) {
        ADL_TRY(hipMalloc((void**)&h->d_hV, sizeof(double) * nb * L.n_v));
        ADL_TRY(hipMalloc((void**)&h->d_hP, sizeof(double) * nb * L.n_p));
        ADL_TRY(hipMalloc((void**)&h->d_sigma, sizeof(double) * nb));
        ADL_TRY(hipMalloc((void**)&h->d_lam, sizeof(double) * nb * L.n_g));
        ADL_TRY(hipMalloc((void**)&h->d_H, sizeof(double) * nb * hn));
    }
    ADL_TRY(hipMemcpy(h->d_hV, V, sizeof(double) * nb * L.n_v, hipMemcpyHostToDevice));
    ADL_TRY(hipMemcpy(h->d_hP, P, sizeof(double) * nb * L.n_p, hipMemcpyHostToDevice));
    ADL_TRY(hipMemcpy(h->d_sigma, sigma, sizeof(double) * nb, hipMemcpyHostToDevice));
    ADL_TRY(hipMemcpy(h->d_lam, lam_g, sizeof(double) * nb * L.n_g, hipMemcpyHostToDevice));
    rc = launch_hess_all(h, h->d_hV, h->d_hP, h->d_sigma, h->d_lam, h->d_H, nullptr);
    if (rc) return rc;
    ADL_TRY(hipDeviceSynchronize());
    ADL_TRY(hipMemcpy(H, h->d_H, sizeof(double) * nb * hn, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nb * hn; ++i)
        if (!std::isfinite(H[i])) return fail(AWE_ERR_NONFINITE, "non-finite value in the Hessian");
    return AWE_OK;
}

int adl_last_hess_ms(adl_handle h, float* ms) {
    if (!h || !h->htimed || !ms) return fail(AWE_ERR_ARG, "no timed Hessian launch yet");
    ADL_TRY(hipEventSynchronize(h->hev[1]));
    ADL_TRY(hipEventElapsedTime(ms, h->hev[0], h->hev[1]));
    return AWE_OK;
}

}  // extern "C"
