// awegpu -- MI355X (gfx950) evaluator for the awebox AP2 direct-collocation NLP.
//
// Replaces, for the AP2 configuration, the CasADi-expanded SX evaluation that IPOPT calls
// through nlpsol (awebox/opti/preparation.py:366-400): f, g, grad f and the CCS values of J_g.
//
// Execution model:
//   * one workgroup per (NLP instance, shooting interval); W = ceil((d+1)/2) wavefronts;
//   * the interval's slice of V is staged in LDS with coalesced loads;
//   * model pass: every half-wavefront (32 lanes) evaluates ONE node (the shooting node or one
//     Radau node) of the hand-written model in forward-mode dual arithmetic.  The node's
//     Jacobian block is obtained by *compressed* forward mode: the 61 seed directions are
//     grouped into <= 32 colours whose row sets are disjoint (greedy Curtis-Powell-Reid
//     colouring computed on the host from the structural dependencies of the same model), so
//     32 lanes recover the whole block and one wavefront evaluates two nodes at once;
//   * seed directions live in V-space where that is free: at a Radau node the direction of
//     state i seeds x_i AND xdot_i = C[jj,jj]/(h tf); the direction of xdot_i feeds the other
//     d columns of the collocation polynomial; one direction carries d/d t_f of every xdot_i
//     (collocation.py:202-258).  The chain rule through xdot = C X / (h tf) costs no extra pass;
//   * the sub-models that depend on very few variables (tether drag: q, dq, diam_t; kite-height
//     wind and density: q_z) are preaccumulated once per node, one (element, direction) per
//     thread, and enter the model pass as values plus partial derivatives;
//   * objective pass (one lane per direction): directional derivatives of the objective terms
//     of each Radau node (objective.py), summed per V column in a fixed order;
//   * write-out: the interval's g rows and grad f columns are contiguous stores; the CCS values
//     of J_g are produced by a host-built gather list with one entry per CCS slot of the
//     interval (tangent-buffer index, polynomial scale), so the J stores are contiguous and
//     coalesced; the few global gradient entries are reduced deterministically by a small
//     finalize kernel (no float atomics anywhere).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/awegpu.h"
#include "ap2_model.hpp"
#include "ap2_tables.hpp"

namespace {

using namespace awt;

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess)                                                          \
            return fail(AWE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)




// ---------------------------------------------------------------------------------------
// device side
// ---------------------------------------------------------------------------------------


struct KArgs {
    const double* V;
    const double* P;
    const double* cst;
    DevColl coll;                // by value: uniform loads from the kernel-argument segment
    const ColorTabs* ct;
    const int* seg;              // [n_k][kSegs][3] global CCS slot, length, offset in the list
    const unsigned* glist;       // per CCS slot: tangent index | scale index << 16
    const int* glist_off;        // [n_k] first list entry of each interval
    double* g;
    double* jac;
    double* grad;
    double* partial;             // [batch][n_k][kNPartial]
    double* f;
    int n_k, d, n_v, n_g, n_p, nnz, batch;
    int stride, rows, v_int0;
    int tang_total;              // tangent buffer entries; tang[tang_total] holds 1.0
    int nscale;                  // 1 + (d+1)^2 polynomial scales + constant entries
    double kconst[kMaxConst];    // values of constant J entries (continuity, periodicity)
    int nconst;
    int want_derivs;
};

// node variable i of one lane's colour: value from LDS, tangent from the colour's seeds
struct LaneIn {
    const double* w;             // LDS: 59 node values (scaled)
    unsigned long long seedA;
    unsigned int seedXD;
    double cxx;                  // C[jj][jj] / (h tf) at a Radau node, 0 at the shooting node
    double tfs;                  // -1/tf for the t_f colour at a Radau node, else 0
    // seed bit -> 0.0 / 1.0 by a bit-field extract and one conversion (i is a compile-time
    // constant after inlining) instead of a 64-bit test and two selects per input read: -1 % kernel
    // time at B = 2048 (tools/ap2_variants.py, profiles/r02/ap2_variants.log); the same form on the
    // xdot seeds measured slower (register spills)
    __device__ __forceinline__ static double bit(unsigned long long m, int i) {
        return (double)(unsigned)((m >> i) & 1ull);
    }
    __device__ __forceinline__ awe::Dual operator()(int i) const {
        double t = bit(seedA, i);
        if (i >= AWE_NX && i < 2 * AWE_NX) {
            const int j = i - AWE_NX;
            if ((seedA >> j) & 1ull) t += cxx;
            if ((seedXD >> j) & 1u) t += 1.0;
            t += tfs * w[i];
        }
        return awe::Dual(w[i], t);
    }
};

// streams one node's rows into the compressed LDS tangent buffer (and values into gval)
// (branch-free: stores a lane does not own go to its private dump slot)
struct NodeSink {
    double* tp;
    double* gv;
    double* dump;
    unsigned long long cm;
    bool c0;
    __device__ __forceinline__ void emit(int r, const awe::Dual& v) {
        double* ga = c0 ? gv + r : dump;
        *ga = v.v;
        const bool on = (cm >> r) & 1ull;
        double* ta = on ? tp + __popcll(cm & ((1ull << r) - 1ull)) : dump;
        *ta = v.d;
    }
    __device__ __forceinline__ void eq_row(int r, const awe::Dual& v) { emit(r, v); }
    __device__ __forceinline__ void ineq_row(int r, const awe::Dual& v) { emit(AWE_N_EQ + r, v); }
    __device__ __forceinline__ void power(const awe::Dual& v) { emit(kRowPower, v); }
    __device__ __forceinline__ void beta(const awe::Dual& v) { emit(kRowBeta, v); }
};

// Preaccumulated sub-models (InlineSubmodels in ap2_model.hpp): values and partial derivatives
// w.r.t. the scaled node variables, computed once per node; a lane forms its tangent from the
// seeds of its colour.  pr layout: D_tether[3], dD/d(q0,q1,q2,dq0,dq1,dq2,diam_t)[7][3],
// u_wind, du_wind/dq_z, rho, drho/dq_z.

constexpr int kPreDirs = 7;
__device__ __forceinline__ int pre_var(int j) { return j < 6 ? j : kDirDiam; }

struct LdsSubmodels {
    const double* pr;
    unsigned long long seedA;
    __device__ __forceinline__ void kite_atmosphere(const awe::Dual&, const double*, awe::Dual& uw,
                                                    awe::Dual& rho) const {
        const double sd = ((seedA >> 2) & 1ull) ? 1.0 : 0.0;
        uw = awe::Dual(pr[24], sd * pr[25]);
        rho = awe::Dual(pr[26], sd * pr[27]);
    }
    __device__ __forceinline__ void tether_drag(const awe::Dual*, const awe::Dual*, const awe::Dual&,
                                                const double*, const double*, awe::Dual D[3]) const {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < kPreDirs; ++j)
                if ((seedA >> pre_var(j)) & 1ull) t += pr[3 + 3 * j + i];
            D[i] = awe::Dual(pr[i], t);
        }
    }
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

template <int D>
constexpr int waves_for() { return (D + 2) / 2; }

template <int D>
constexpr int nloc_pad() {
    return ((9 + AWE_NX + AWE_NU + AWE_NX + AWE_NZ + D * (AWE_NX + AWE_NZ) + AWE_NX) + 1) & ~1;
}

// LDS layout (doubles): vloc | pst | wn[NN][64] | gval[NN][36] | dfl[NN][64] | pre[NN][28] |
//                       fnode[NN pad] | scale[64] | tang[tang_total + 1]
// (the sub-model scratch of phase 0 aliases tang, which is written only from phase 1 on)
// P staged for the objective: weights[59] | cost[20] at 64 | theta ref[2] at 84 | ref V slice
constexpr int kPstCost = 64, kPstThRef = 84, kPstRef = 86;
template <int D>
constexpr int pst_pad() {
    return (kPstRef + AWE_NX + AWE_NU + AWE_NX + AWE_NZ + D * (AWE_NX + AWE_NZ) + 1) & ~1;
}

template <int D>
constexpr int lds_fixed_doubles() {
    return nloc_pad<D>() + pst_pad<D>() + (D + 1) * (64 + kGvalStride + 64 + kPreStride) + ((D + 2) & ~1) + 64 + 2;
}

// ---- phases shared by the first- and second-order kernels ---------------------------------

// scaled node values (AWE_NW layout) of the interval's d+1 nodes; xdot at Radau nodes from the
// collocation polynomial (collocation.py:202-258).  vloc = [theta, phi, x[k], u, xdot, z, coll..]
template <int D, int NT>
__device__ __forceinline__ void node_values_pass(const double* vloc, const double* C, int n_k, double* wn,
                                                 int tid) {
    constexpr int NN = D + 1;
    const double* vt = vloc;
    const double* vx = vloc + 9;
    const double* vu = vx + AWE_NX;
    const double* vxd = vu + AWE_NU;
    const double* vz = vxd + AWE_NX;
    const double* vcoll = vz + AWE_NZ;
    const double tf = vt[1];
    const double h = 1.0 / n_k;
    for (int t = tid; t < NN * 64; t += NT) {
        const int n = t >> 6, i = t & 63;
        double val = 0.0;
        if (i < AWE_NX) {
            val = n == 0 ? vx[i] : vcoll[(n - 1) * (AWE_NX + AWE_NZ) + i];
        } else if (i < 2 * AWE_NX) {
            const int s = i - AWE_NX;
            if (n == 0) {
                val = vxd[s];
            } else {
                double xp = 0.0;
#pragma unroll
                for (int r = 0; r < NN; ++r) {
                    const double Xr = (r == 0) ? vx[s] : vcoll[(r - 1) * (AWE_NX + AWE_NZ) + s];
                    xp += C[r * NN + n] * Xr;
                }
                val = xp / h / tf;
            }
        } else if (i < 2 * AWE_NX + AWE_NU) {
            val = vu[i - 2 * AWE_NX];
        } else if (i < 2 * AWE_NX + AWE_NU + AWE_NZ) {
            val = n == 0 ? vz[0] : vcoll[(n - 1) * (AWE_NX + AWE_NZ) + AWE_NX];
        } else if (i < AWE_NW) {
            val = vt[i - (2 * AWE_NX + AWE_NU + AWE_NZ)];
        }
        wn[t] = val;
    }
    __syncthreads();
}

// sub-model preaccumulation: stage A, one (node, height) per thread: wind speed and density at
// the kite and at every tether element midpoint, as functions of q_z; stage B, one (node,
// element, direction) per thread: the element's drag along q0..2, dq0..2, diam_t; then the
// element sums.  tang serves as scratch.
template <int D, int NT>
__device__ __forceinline__ void submodel_pass(const double* cst, const double* th, const double* wn, double* pre,
                                              double* tang, int tid) {
    constexpr int NN = D + 1;
    {
        const double* s = cst + AWE_C_SCALING;
        const int n_el = (int)cst[AWE_C_N_ELEMENTS];
        double* scr = tang;                                   // [NN][n_el][7][6]
        double* atm = tang + NN * n_el * kPreDirs * 6;        // [NN][n_el][4]
        for (int t = tid; t < NN * (n_el + 1); t += NT) {
            const int n = t / (n_el + 1), e = t - n * (n_el + 1) - 1;
            const awe::Dual qz = awe::Dual(wn[n * 64 + 2], 1.0) * s[2];
            awe::Dual uw, rho;
            double* o;
            if (e < 0) {
                awe::InlineSubmodels().kite_atmosphere(qz, th, uw, rho);
                o = pre + n * kPreStride + 24;
            } else {
                const awe::Dual zz = awe::tether_element_height(e, n_el, qz);
                uw = awe::wind_speed(zz, th);
                rho = awe::isa_density(zz, th);
                o = atm + (n * n_el + e) * 4;
            }
            o[0] = uw.v; o[1] = uw.d; o[2] = rho.v; o[3] = rho.d;
        }
        __syncthreads();
        const int ntask = n_el * kPreDirs;
        for (int t = tid; t < NN * ntask; t += NT) {
            const int n = t / ntask, q = t - n * ntask;
            const double* w = wn + n * 64;
            const int e = q / kPreDirs, j = q - e * kPreDirs;
            const int vj = pre_var(j);
            awe::Dual qv[3], vv[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                qv[i] = awe::Dual(w[i], vj == i ? 1.0 : 0.0) * s[i];
                vv[i] = awe::Dual(w[3 + i], vj == 3 + i ? 1.0 : 0.0) * s[3 + i];
            }
            awe::Dual diam = awe::Dual(w[kDirDiam], vj == kDirDiam ? 1.0 : 0.0) * s[kDirDiam];
            const double* at = atm + (n * n_el + e) * 4;
            const double dz = vj == 2 ? 1.0 : 0.0;
            const awe::Dual uw(at[0], dz * at[1]), rho(at[2], dz * at[3]);
            awe::Dual c[3];
            awe::tether_element_drag(e, n_el, qv, vv, diam, uw, rho, th, c);
            double* o = scr + ((n * n_el + e) * kPreDirs + j) * 6;
#pragma unroll
            for (int i = 0; i < 3; ++i) { o[i] = c[i].v; o[3 + i] = c[i].d; }
        }
        __syncthreads();
        // element sums in element order (the order of the inline model)
        for (int t = tid; t < NN * kPreDirs * 3; t += NT) {
            const int n = t / (kPreDirs * 3), j = (t / 3) % kPreDirs, i = t % 3;
            double val = 0.0, tan = 0.0;
            for (int e = 0; e < n_el; ++e) {
                const double* o = scr + ((n * n_el + e) * kPreDirs + j) * 6;
                val = val + o[i];
                tan = tan + o[3 + i];
            }
            if (j == 0) pre[n * kPreStride + i] = val;
            pre[n * kPreStride + 3 + 3 * j + i] = tan;
        }
        __syncthreads();
    }
}

// first-order model pass: half-wavefront slot = node, lane = colour; rows go to the compressed
// tangent buffer, values to gval
template <int D>
__device__ __forceinline__ void first_order_pass(const ColorTabs* ct, const double* wn, const double* pre,
                                                 double* tang, double* gval, double* dump, const double* C,
                                                 const double* vt, const double* th, const double* cst,
                                                 double inv_h_tf, double inv_tf, int wave, int lane) {
    constexpr int NN = D + 1;
    auto toff = [&](int n) { return n == 0 ? 0 : ct->tsize[0] + (n - 1) * ct->tsize[1]; };
    {
        const int n = wave * 2 + (lane >> 5);
        const int c = lane & (kHalf - 1);
        if (n < NN) {
            const int kind = n > 0 ? 1 : 0;
            LaneIn in;
            in.w = wn + n * 64;
            in.seedA = ct->seedA[kind][c];
            in.seedXD = ct->seedXD[kind][c];
            in.cxx = n > 0 ? C[n * NN + n] * inv_h_tf : 0.0;
            in.tfs = (c == ct->tf_color[kind]) ? -inv_tf : 0.0;
            NodeSink sink;
            sink.tp = tang + toff(n) + ct->off[kind][c];
            sink.gv = gval + n * kGvalStride;
            sink.cm = ct->cmask[kind][c];
            sink.c0 = c == 0;
            sink.dump = dump;
            awe::Dual gamma(vt[2 + kPhiGamma], ((in.seedA >> kDirGamma) & 1ull) ? 1.0 : 0.0);
            LdsSubmodels sub{pre + n * kPreStride, in.seedA};
            awe::ap2_node<awe::Dual>(in, gamma, th, cst, sink, n == 0, sub);
        }
    }
}

// occupancy target (waves per SIMD) for the register allocator; build-time tunable
#ifndef AWE_WAVES_PER_EU
#define AWE_WAVES_PER_EU 3
#endif

template <int D>
__global__ __launch_bounds__(64 * waves_for<D>())
__attribute__((amdgpu_waves_per_eu(AWE_WAVES_PER_EU, AWE_WAVES_PER_EU)))
void ap2_interval_kernel(KArgs a) {
    constexpr int NN = D + 1;
    constexpr int W = waves_for<D>();
    constexpr int NT = 64 * W;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int k = blockIdx.x % a.n_k;
    const int b = blockIdx.x / a.n_k;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* th = P + a.n_v + AWE_NW + AWE_NCOST;
    const double* cost = P + a.n_v + AWE_NW;
    const double* wts = P + a.n_v;
    const double* vref = P;
    double* g = a.g + (size_t)b * a.n_g;
    double* jac = a.jac + (size_t)b * a.nnz;
    double* grad = a.grad + (size_t)b * a.n_v;
    const ColorTabs* ct = a.ct;
    const double* C = a.coll.C;

    extern __shared__ double smem[];
    double* vloc = smem;
    double* pst = vloc + nloc_pad<D>();
    double* wn = pst + pst_pad<D>();
    double* gval = wn + NN * 64;
    double* dfl = gval + NN * kGvalStride;
    double* pre = dfl + NN * 64;
    double* fnode = pre + NN * kPreStride;
    double* scl = fnode + ((D + 2) & ~1);
    double* tang = scl + 64;
    auto toff = [&](int n) { return n == 0 ? 0 : ct->tsize[0] + (n - 1) * ct->tsize[1]; };

    // ---- phase 0: stage [theta, phi, x[k], u, xdot, z, coll..., x[k+1]]; constant J entries
    const int base = a.v_int0 + k * a.stride;
    for (int i = tid; i < 9; i += NT) vloc[i] = V[i];
    for (int i = tid; i < a.stride + AWE_NX; i += NT) vloc[9 + i] = V[base + i];
    for (int i = tid; i < kPstRef + a.stride; i += NT) {
        double pv = 0.0;
        if (i < AWE_NW) pv = wts[i];
        else if (i >= kPstCost && i < kPstCost + AWE_NCOST) pv = cost[i - kPstCost];
        else if (i >= kPstThRef && i < kPstRef) pv = vref[i - kPstThRef];
        else if (i >= kPstRef) pv = vref[base + i - kPstRef];
        pst[i] = pv;
    }
    const int obj_b = ct->obj_beta[lane], obj_p = ct->obj_power[lane];
    __syncthreads();
    const double* vt = vloc;                       // theta at 0, phi at 2
    const double* vx = vloc + 9;                   // x[k]
    const double* vu = vx + AWE_NX;
    const double* vxd = vu + AWE_NU;
    const double* vz = vxd + AWE_NX;
    const double* vcoll = vz + AWE_NZ;             // coll_var[j] = vcoll + j*24
    const double* vx1 = vcoll + D * (AWE_NX + AWE_NZ);
    const double tf = vt[1];
    const double h = 1.0 / a.n_k;
    const double inv_h_tf = 1.0 / h / tf;
    const double inv_tf = 1.0 / tf;
    // gather scales: 1, C[r][n] / (h tf) for the polynomial columns, constant entries
    for (int i = tid; i < a.nscale; i += NT) {
        double sv = 1.0;
        if (i >= 1 && i <= NN * NN) sv = C[i - 1] * inv_h_tf;
        else if (i > NN * NN) sv = a.kconst[i - 1 - NN * NN];
        scl[i] = sv;
    }
    if (tid == 0) tang[a.tang_total] = 1.0;

    node_values_pass<D, NT>(vloc, C, a.n_k, wn, tid);

    // ---- phase 0b: sub-models -------------------------------------------------------------
    // stage A, one (node, height) per thread: wind speed and density at the kite and at every
    // tether element midpoint, as functions of q_z; stage B, one (node, element, direction)
    // per thread: the element's drag along q0..2, dq0..2, diam_t
    submodel_pass<D, NT>(a.cst, th, wn, pre, tang, tid);

    // ---- phase 1: model, one node per half-wavefront, one colour per lane ------------------
    first_order_pass<D>(ct, wn, pre, tang, gval, dfl + tid, C, vt, th, a.cst, inv_h_tf, inv_tf, wave, lane);
    __syncthreads();

    // ---- phase 2: objective directional derivatives (one lane per direction) -------------
    const double* pcost = pst + kPstCost;
    const double* pw8 = pst;                                   // weights
    const double psi = vt[2 + kPhiPsi];
    const double w_track = pcost[kCostTracking] / a.cst[AWE_C_NORM_TRACKING];
    const double w_xdot = pcost[kCostXdotRegularisation] / a.cst[AWE_C_NORM_XDOT_REG];
    const double w_ureg = pcost[kCostURegularisation] / a.cst[AWE_C_NORM_U_REG];
    const double w_fict = pcost[kCostFictitious] / a.cst[AWE_C_NORM_FICTITIOUS];
    const double w_theta = pcost[kCostThetaRegularisation] / a.cst[AWE_C_NORM_THETA_REG];
    for (int n = 1 + wave; n < NN; n += W) {
        const int dir = lane;
        const double* tp = tang + toff(n);
        {
            // objective at Radau node j (objective.py:45-544): w_j [psi tracking + xdot, u,
            // fictitious and theta regularisation] + beta cost + (1 - psi) power cost
            const int j = n - 1;
            const double wj = a.coll.w[j];
            const double* w = wn + n * 64;
            const double* rb = pst + kPstRef;                  // reference V slice
            const double* rcx = rb + 2 * AWE_NX + AWE_NU + AWE_NZ + j * (AWE_NX + AWE_NZ);
            const double* ru = rb + AWE_NX;
            const double cxx = C[n * NN + n] * inv_h_tf;
            double trk = 0.0, xdr = 0.0, oth = 0.0, dfd = 0.0;
            if (dir < AWE_NX) {
                const double e = w[dir] - rcx[dir], ww = pw8[dir] * w_track;
                const double xdv = w[AWE_NX + dir], wx = pw8[AWE_NX + dir] * w_xdot;
                trk = ww * (e * e);
                dfd = wj * (psi * (2.0 * ww * e) + cxx * (2.0 * wx * xdv));
            } else if (dir < 2 * AWE_NX) {
                const double xdv = w[dir], wx = pw8[dir] * w_xdot;
                xdr = wx * (xdv * xdv);
                dfd = wj * (2.0 * wx * xdv);
            } else if (dir < 2 * AWE_NX + AWE_NU) {
                const int i = dir - 2 * AWE_NX;
                const double e = w[dir] - ru[i], wu = pw8[dir] * (i < 6 ? w_fict : w_ureg);
                oth = wu * (e * e);
                dfd = wj * (2.0 * wu * e);
            } else if (dir == kDirZ) {
                const double e = w[dir] - rcx[AWE_NX], ww = pw8[dir] * w_track;
                trk = ww * (e * e);
                dfd = wj * psi * (2.0 * ww * e);
            } else if (dir == kDirDiam) {
                const double e = w[dir] - pst[kPstThRef], wt = pw8[dir] * w_theta;
                oth = wt * (e * e);
                dfd = wj * (2.0 * wt * e);
            }
            trk = wave_sum(trk);
            xdr = wave_sum(xdr);
            oth = wave_sum(oth);
            const double bv = gval[n * kGvalStride + kRowBeta];
            const double pv = gval[n * kGvalStride + kRowPower];
            const double cb = pcost[kCostBeta] * wj / a.cst[AWE_C_NORM_BETA];
            const double cp = -pcost[kCostPower] * wj / (double)a.n_k;   // (-c_p)(tf/N) w_j p / tf
            if (dir == kDirTf) dfd = -2.0 * wj * xdr * inv_tf;
            if (dir == kDirPsi) dfd = wj * trk - cp * pv;
            if (obj_b >= 0) dfd += (2.0 * cb * bv) * tp[obj_b];
            if (obj_p >= 0) dfd += ((1.0 - psi) * cp) * tp[obj_p];
            dfl[n * 64 + dir] = dfd;
            if (dir == 0) fnode[n] = wj * (psi * trk + xdr + oth) + cb * (bv * bv) + (1.0 - psi) * (cp * pv);
        }
    }
    __syncthreads();

    // ---- phase 3: write-out ---------------------------------------------------------------
    const DevColl* cc = &a.coll;
    for (int r = tid; r < a.rows; r += NT) {
        double val;
        if (r < AWE_N_EQ + AWE_N_INEQ) {
            val = gval[r];
        } else if (r < AWE_N_EQ + AWE_N_INEQ + D * AWE_N_EQ) {
            const int q = r - (AWE_N_EQ + AWE_N_INEQ);
            val = gval[(1 + q / AWE_N_EQ) * kGvalStride + q % AWE_N_EQ];
        } else {
            // continuity x[k+1] - sum_r D_r X_r (collocation.py:319-336); CasADi drops 0 * X
            const int i = r - (AWE_N_EQ + AWE_N_INEQ + D * AWE_N_EQ);
            double xf = 0.0;
#pragma unroll
            for (int rr = 0; rr < NN; ++rr) {
                if (cc->D[rr] == 0.0) continue;
                const double Xr = (rr == 0) ? vx[i] : vcoll[(rr - 1) * (AWE_NX + AWE_NZ) + i];
                xf += cc->D[rr] * Xr;
            }
            val = vx1[i] - xf;
        }
        g[k * a.rows + r] = val;
    }
    double* part = a.partial + ((size_t)b * a.n_k + k) * kNPartial;
    if (tid == 0) {
        double s = 0.0;
        for (int n = 1; n < NN; ++n) s += fnode[n];
        part[0] = s;
    }
    if (!a.want_derivs) return;
    if (tid >= 1 && tid <= 3) {
        const int dcol = tid == 1 ? kDirDiam : (tid == 2 ? kDirTf : kDirPsi);
        double s = 0.0;
        for (int n = 1; n < NN; ++n) s += dfl[n * 64 + dcol];
        part[tid] = s;
    }
    // gradient of the interval's local columns: x[k], u[k], xdot[k], z[k], coll_var[k]
    for (int col = tid; col < a.stride; col += NT) {
        double gsum = 0.0;
        if (col < AWE_NX) {                                   // x[k]: polynomial path only
#pragma unroll
            for (int n = 1; n < NN; ++n) gsum += C[n] * inv_h_tf * dfl[n * 64 + AWE_NX + col];
        } else if (col < AWE_NX + AWE_NU) {                   // u[k] (zero-order hold)
            const int i = col - AWE_NX;
#pragma unroll
            for (int n = 1; n < NN; ++n) gsum += dfl[n * 64 + 2 * AWE_NX + i];
        } else if (col >= 2 * AWE_NX + AWE_NU + AWE_NZ) {     // coll_var[k][j]
            const int q = col - (2 * AWE_NX + AWE_NU + AWE_NZ);
            const int r = 1 + q / (AWE_NX + AWE_NZ), e = q % (AWE_NX + AWE_NZ);
            if (e < AWE_NX) {
                gsum = dfl[r * 64 + e];
#pragma unroll
                for (int n = 1; n < NN; ++n)
                    if (n != r) gsum += C[r * NN + n] * inv_h_tf * dfl[n * 64 + AWE_NX + e];
            } else {
                gsum = dfl[r * 64 + kDirZ];
            }
        }                                                     // xdot[k], z[k]: 0
        grad[base + col] = gsum;
    }
    // the interval's CCS runs, contiguous in the value array: one gather entry per slot
    const int* sg = a.seg + (size_t)k * kSegs * 3;
    const unsigned* gl = a.glist + a.glist_off[k];
#pragma unroll
    for (int s = 0; s < kSegs; ++s) {
        const int g0 = sg[3 * s], len = sg[3 * s + 1], lo = sg[3 * s + 2];
        for (int i = tid; i < len; i += NT) {
            const unsigned e = gl[lo + i];
            jac[g0 + i] = scl[e >> 16] * tang[e & 0xffffu];
        }
    }
}

// one wave per instance: reduce interval partials, add global costs, periodic rows
__global__ __launch_bounds__(64) void ap2_finalize_kernel(KArgs a) {
    const int lane = threadIdx.x;
    const int b = blockIdx.x;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* cost = P + a.n_v + AWE_NW;
    const double* vref = P;
    double* g = a.g + (size_t)b * a.n_g;
    double* grad = a.grad + (size_t)b * a.n_v;
    const double* part = a.partial + (size_t)b * a.n_k * kNPartial;

    double s[kNPartial] = {0.0, 0.0, 0.0, 0.0};
    for (int k = lane; k < a.n_k; k += 64)
        for (int c = 0; c < kNPartial; ++c) s[c] += part[k * kNPartial + c];
    for (int off = 32; off > 0; off >>= 1)
        for (int c = 0; c < kNPartial; ++c) s[c] += __shfl_xor(s[c], off);

    const double tf = V[1], tf_ref = vref[1];
    // periodic rows: x_0 - x_terminal in sorted-name order (operation.py:245-266); their J
    // entries are constants written by the interval kernel
    const int last = a.v_int0 + (a.n_k - 1) * a.stride + 2 * AWE_NX + AWE_NU + AWE_NZ +
                     (a.d - 1) * (AWE_NX + AWE_NZ);
    if (lane < AWE_NX) {
        const int i = kPeriodicOrder[lane];
        g[a.n_k * a.rows + lane] = V[a.v_int0 + i] - V[last + i];
    }
    // phi order gamma, tau, iota, psi, eta, nu, upsilon (system.py:435-450); cost order
    // gamma, iota, psi, tau, eta, nu, upsilon (discretization.py:129-152)
    constexpr int phi_cost_map[AWE_NPHI] = {3, 6, 4, 5, 7, 8, 9};
    if (lane == 0) {
        double fh = 0.0;
        for (int i = 0; i < AWE_NPHI; ++i) fh += cost[phi_cost_map[i]] * V[AWE_NTH + i];
        const double time_cost = cost[kCostTf] * (tf - tf_ref) * (tf - tf_ref);
        a.f[b] = s[0] + time_cost + fh;
    }
    if (a.want_derivs) {
        if (lane == 0) grad[0] = s[1];
        if (lane == 1) grad[1] = s[2] + cost[kCostTf] * 2.0 * (tf - tf_ref);
        if (lane >= 2 && lane < 2 + AWE_NPHI) {
            const int i = lane - 2;
            double gphi = cost[phi_cost_map[i]];
            if (i == kPhiPsi) gphi += s[3];
            grad[AWE_NTH + i] = gphi;
        }
        if (lane >= 2 + AWE_NPHI && lane < 2 + AWE_NPHI + AWE_NXI) grad[lane] = 0.0;
        if (lane < AWE_NX) grad[a.v_int0 + a.n_k * a.stride + lane] = 0.0;   // x[n_k]
    }
}



// =========================================================================================
// Value-only evaluation (nlp_f / nlp_g): the model in plain double, one thread per node
// =========================================================================================
// The derivative kernel carries 32 colour lanes of dual numbers per node; nlp_f and nlp_g (IPOPT's
// line-search trials) need none of it.  One 64-thread workgroup per (instance, interval): the
// interval's V slice is staged in LDS, node values as in the derivative kernel, then thread n < d+1
// evaluates node n of the same templated model (ap2_model.hpp) with T = double and inline
// sub-models, and the objective terms of its Radau node serially; continuity rows and the
// interval's objective partial follow, and ap2_finalize_kernel adds the global terms and the
// periodicity rows.  Same formulas as the derivative kernel, summed in another order (values agree
// to roundoff, tests/test_gpu_parity.py).
struct ValueIn {
    const double* w;
    __device__ __forceinline__ double operator()(int i) const { return w[i]; }
};

struct ValueSink {
    double* gv;
    __device__ __forceinline__ void eq_row(int r, double v) { gv[r] = v; }
    __device__ __forceinline__ void ineq_row(int r, double v) { gv[AWE_N_EQ + r] = v; }
    __device__ __forceinline__ void power(double v) { gv[kRowPower] = v; }
    __device__ __forceinline__ void beta(double v) { gv[kRowBeta] = v; }
};

template <int D>
__global__ __launch_bounds__(64) void ap2_value_kernel(KArgs a) {
    constexpr int NN = D + 1;
    const int tid = threadIdx.x;
    const int k = blockIdx.x % a.n_k;
    const int b = blockIdx.x / a.n_k;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* th = P + a.n_v + AWE_NW + AWE_NCOST;
    const double* cost = P + a.n_v + AWE_NW;
    const double* wts = P + a.n_v;
    const double* vref = P;
    double* g = a.g + (size_t)b * a.n_g;
    const double* C = a.coll.C;
    __shared__ double vloc[nloc_pad<D>()];
    __shared__ double wn[NN * 64];
    __shared__ double gval[NN * kGvalStride];
    __shared__ double fnode[NN + 1];
    const int base = a.v_int0 + k * a.stride;
    for (int i = tid; i < 9; i += 64) vloc[i] = V[i];
    for (int i = tid; i < a.stride + AWE_NX; i += 64) vloc[9 + i] = V[base + i];
    __syncthreads();
    node_values_pass<D, 64>(vloc, C, a.n_k, wn, tid);
    const double* vt = vloc;
    const double* vx = vloc + 9;
    const double* vcoll = vx + AWE_NX + AWE_NU + AWE_NX + AWE_NZ;
    const double* vx1 = vcoll + D * (AWE_NX + AWE_NZ);
    if (tid < NN) {
        const int n = tid;
        ValueIn in{wn + n * 64};
        ValueSink sink{gval + n * kGvalStride};
        awe::ap2_node<double>(in, vt[2 + kPhiGamma], th, a.cst, sink, n == 0, awe::InlineSubmodels());
        double fn = 0.0;
        if (n > 0) {                                         // objective at Radau node j (objective.py)
            const int j = n - 1;
            const double wj = a.coll.w[j];
            const double* w = wn + n * 64;
            const double* rb = vref + base;
            const double* rcx = rb + 2 * AWE_NX + AWE_NU + AWE_NZ + j * (AWE_NX + AWE_NZ);
            const double* ru = rb + AWE_NX;
            const double psi = vt[2 + kPhiPsi];
            const double w_track = cost[kCostTracking] / a.cst[AWE_C_NORM_TRACKING];
            const double w_xdot = cost[kCostXdotRegularisation] / a.cst[AWE_C_NORM_XDOT_REG];
            const double w_ureg = cost[kCostURegularisation] / a.cst[AWE_C_NORM_U_REG];
            const double w_fict = cost[kCostFictitious] / a.cst[AWE_C_NORM_FICTITIOUS];
            const double w_theta = cost[kCostThetaRegularisation] / a.cst[AWE_C_NORM_THETA_REG];
            double trk = 0.0, xdr = 0.0, oth = 0.0;
            for (int i = 0; i < AWE_NX; ++i) {
                const double e = w[i] - rcx[i];
                trk += wts[i] * w_track * (e * e);
                const double xdv = w[AWE_NX + i];
                xdr += wts[AWE_NX + i] * w_xdot * (xdv * xdv);
            }
            for (int i = 0; i < AWE_NU; ++i) {
                const double e = w[2 * AWE_NX + i] - ru[i];
                oth += wts[2 * AWE_NX + i] * (i < 6 ? w_fict : w_ureg) * (e * e);
            }
            {
                const double e = w[kDirZ] - rcx[AWE_NX];
                trk += wts[kDirZ] * w_track * (e * e);
                const double et = w[kDirDiam] - vref[0];
                oth += wts[kDirDiam] * w_theta * (et * et);
            }
            const double bv = gval[n * kGvalStride + kRowBeta];
            const double pv = gval[n * kGvalStride + kRowPower];
            const double cb = cost[kCostBeta] * wj / a.cst[AWE_C_NORM_BETA];
            const double cp = -cost[kCostPower] * wj / (double)a.n_k;
            fn = wj * (psi * trk + xdr + oth) + cb * (bv * bv) + (1.0 - psi) * (cp * pv);
        }
        fnode[n] = fn;
    }
    __syncthreads();
    const DevColl* cc = &a.coll;
    for (int r = tid; r < a.rows; r += 64) {
        double val;
        if (r < AWE_N_EQ + AWE_N_INEQ) {
            val = gval[r];
        } else if (r < AWE_N_EQ + AWE_N_INEQ + D * AWE_N_EQ) {
            const int q = r - (AWE_N_EQ + AWE_N_INEQ);
            val = gval[(1 + q / AWE_N_EQ) * kGvalStride + q % AWE_N_EQ];
        } else {
            const int i = r - (AWE_N_EQ + AWE_N_INEQ + D * AWE_N_EQ);
            double xf = 0.0;
            for (int rr = 0; rr < NN; ++rr) {
                if (cc->D[rr] == 0.0) continue;
                const double Xr = (rr == 0) ? vx[i] : vcoll[(rr - 1) * (AWE_NX + AWE_NZ) + i];
                xf += cc->D[rr] * Xr;
            }
            val = vx1[i] - xf;
        }
        g[k * a.rows + r] = val;
    }
    if (tid == 0) {
        double s = 0.0;
        for (int n = 1; n < NN; ++n) s += fnode[n];
        a.partial[((size_t)b * a.n_k + k) * kNPartial] = s;
    }
}

// =========================================================================================
// Hessian of the Lagrangian sigma f + lam^T g (nlp_hess_l)
// =========================================================================================
constexpr int kHessWaves = 4;
constexpr int kHessThreads = 64 * kHessWaves;

struct HKArgs {
    KArgs a;                       // V, P, tables and sizes of the first-order kernel
    const HessTabs* ht;
    const int* tasks;              // colour pairs per node kind
    const short* task_target;      // [task][36] direction-pair index of each row
    const int* ent_off;            // [n_k + 1]
    const int* term_off;
    const unsigned* terms;
    const int* slot0;
    const int* nslot;
    const int* gslot;
    const double* sigma;           // [batch]
    const double* lam;             // [batch][n_g]
    double* H;                     // [batch][nnz_h] upper-triangular CCS values
    double* gpart;                 // [batch][n_k][ng]
    int hnnz, ng, hd_total;
    int g_tftf;                    // index of the (t_f, t_f) entry among the global entries
};

// hyper-dual node variable i: e1 along colour c1, e2 along colour c2
struct LaneHIn {
    const double* w;
    unsigned long long sA1, sA2;
    unsigned int sX1, sX2;
    double cxx, t1, t2;
    __device__ __forceinline__ awe::HDual operator()(int i) const {
        double a = ((sA1 >> i) & 1ull) ? 1.0 : 0.0;
        double b = ((sA2 >> i) & 1ull) ? 1.0 : 0.0;
        if (i >= AWE_NX && i < 2 * AWE_NX) {
            const int j = i - AWE_NX;
            if ((sA1 >> j) & 1ull) a += cxx;
            if ((sX1 >> j) & 1u) a += 1.0;
            a += t1 * w[i];
            if ((sA2 >> j) & 1ull) b += cxx;
            if ((sX2 >> j) & 1u) b += 1.0;
            b += t2 * w[i];
        }
        return awe::HDual(w[i], a, b, 0.0);
    }
};

// accumulates mu_r * d2F_r/de1de2 into the node's direction-pair Hessian (branch-free)
struct LaneHSink {
    double* hd;
    double* dump;
    const double* mu;
    const short* tt;               // this task's row targets
    __device__ __forceinline__ void emit(int r, const awe::HDual& v) {
        const int idx = tt[r];
        double* adr = idx >= 0 ? hd + idx : dump;
        *adr += mu[r] * v.ab;
    }
    __device__ __forceinline__ void eq_row(int r, const awe::HDual& v) { emit(r, v); }
    __device__ __forceinline__ void ineq_row(int r, const awe::HDual& v) { emit(AWE_N_EQ + r, v); }
    __device__ __forceinline__ void power(const awe::HDual& v) { emit(kRowPower, v); }
    __device__ __forceinline__ void beta(const awe::HDual& v) { emit(kRowBeta, v); }
};

#ifndef AWE_HESS_WAVES_PER_EU
#define AWE_HESS_WAVES_PER_EU 1
#endif

template <int D>
constexpr int hess_lds_fixed_doubles() {
    return nloc_pad<D>() + pst_pad<D>() + (D + 1) * (64 + kGvalStride + kPreStride + 36 + 24) + 8 + 64 +
           kHessThreads;
}

template <int D>
__global__ __launch_bounds__(kHessThreads)
__attribute__((amdgpu_waves_per_eu(AWE_HESS_WAVES_PER_EU, AWE_HESS_WAVES_PER_EU)))
void ap2_hess_kernel(HKArgs ha) {
    const KArgs& a = ha.a;
    constexpr int NN = D + 1;
    constexpr int NT = kHessThreads;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int k = blockIdx.x % a.n_k;
    const int b = blockIdx.x / a.n_k;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* th = P + a.n_v + AWE_NW + AWE_NCOST;
    const double* cost = P + a.n_v + AWE_NW;
    const double* wts = P + a.n_v;
    const double* vref = P;
    const double* lam = ha.lam + (size_t)b * a.n_g;
    const double sigma = ha.sigma[b];
    const ColorTabs* ct = a.ct;
    const HessTabs* ht = ha.ht;
    const double* C = a.coll.C;

    extern __shared__ double smem[];
    double* vloc = smem;
    double* pst = vloc + nloc_pad<D>();
    double* wn = pst + pst_pad<D>();
    double* gval = wn + NN * 64;
    double* pre = gval + NN * kGvalStride;
    double* mu = pre + NN * kPreStride;            // [NN][36]
    double* G = mu + NN * 36;                      // [NN][24]: G[n][23] holds sum_i G 2 xdot / tf^2
    double* scl = G + NN * 24 + 8;
    double* dump = scl + 64;                       // one slot per thread
    double* tang = dump + NT;
    double* hd = tang + a.tang_total + 1;
    auto toff = [&](int n) { return n == 0 ? 0 : ct->tsize[0] + (n - 1) * ct->tsize[1]; };
    auto hoff = [&](int n) { return n == 0 ? 0 : ht->npairs[0] + (n - 1) * ht->npairs[1]; };

    // ---- stage V slice and P (as in the first-order kernel) ----------------------------------
    const int base = a.v_int0 + k * a.stride;
    for (int i = tid; i < 9; i += NT) vloc[i] = V[i];
    for (int i = tid; i < a.stride + AWE_NX; i += NT) vloc[9 + i] = V[base + i];
    for (int i = tid; i < kPstRef + a.stride; i += NT) {
        double pv = 0.0;
        if (i < AWE_NW) pv = wts[i];
        else if (i >= kPstCost && i < kPstCost + AWE_NCOST) pv = cost[i - kPstCost];
        else if (i >= kPstThRef && i < kPstRef) pv = vref[i - kPstThRef];
        else if (i >= kPstRef) pv = vref[base + i - kPstRef];
        pst[i] = pv;
    }
    for (int i = tid; i < ha.hd_total; i += NT) hd[i] = 0.0;
    __syncthreads();
    const double* vt = vloc;
    const double tf = vt[1];
    const double h = 1.0 / a.n_k;
    const double inv_h_tf = 1.0 / h / tf;
    const double inv_tf = 1.0 / tf;
    const double psi = vt[2 + kPhiPsi];
    for (int i = tid; i < 1 + NN * NN; i += NT) scl[i] = i == 0 ? 1.0 : C[i - 1] * inv_h_tf;
    node_values_pass<D, NT>(vloc, C, a.n_k, wn, tid);
    submodel_pass<D, NT>(a.cst, th, wn, pre, tang, tid);
    first_order_pass<D>(ct, wn, pre, tang, gval, dump + tid, C, vt, th, a.cst, inv_h_tf, inv_tf, wave, lane);
    __syncthreads();

    // ---- row weights: lam for constraint rows, sigma-scaled objective weights -----------------
    const double* pcost = pst + kPstCost;
    for (int t = tid; t < NN * 36; t += NT) {
        const int n = t / 36, r = t % 36;
        double m = 0.0;
        if (n == 0) {
            if (r < kRowPower) m = lam[k * a.rows + r];
        } else {
            const double wj = a.coll.w[n - 1];
            if (r < AWE_N_EQ) m = lam[k * a.rows + AWE_N_EQ + AWE_N_INEQ + (n - 1) * AWE_N_EQ + r];
            else if (r == kRowPower) m = sigma * (1.0 - psi) * (-pcost[kCostPower] * wj / (double)a.n_k);
            else if (r == kRowBeta)
                m = sigma * 2.0 * (pcost[kCostBeta] * wj / a.cst[AWE_C_NORM_BETA]) * gval[n * kGvalStride + kRowBeta];
        }
        mu[t] = m;
    }
    __syncthreads();

    // ---- second-order pass: one (node, colour pair) per thread ---------------------------------
    const int nt0 = ht->ntask[0], nt1 = ht->ntask[1];
    for (int t = tid; t < nt0 + D * nt1; t += NT) {
        const int n = t < nt0 ? 0 : 1 + (t - nt0) / nt1;
        const int kind = n > 0 ? 1 : 0;
        const int ti = (kind == 0 ? t : (t - nt0) % nt1) + ht->task_off[kind];
        const int task = ha.tasks[ti];
        const int c1 = task & 0xff, c2 = task >> 8;
        LaneHIn in;
        in.w = wn + n * 64;
        in.sA1 = ct->seedA[kind][c1]; in.sA2 = ct->seedA[kind][c2];
        in.sX1 = ct->seedXD[kind][c1]; in.sX2 = ct->seedXD[kind][c2];
        in.cxx = n > 0 ? C[n * NN + n] * inv_h_tf : 0.0;
        in.t1 = (c1 == ct->tf_color[kind]) ? -inv_tf : 0.0;
        in.t2 = (c2 == ct->tf_color[kind]) ? -inv_tf : 0.0;
        LaneHSink sink{hd + hoff(n), dump + tid, mu + n * 36, ha.task_target + (size_t)ti * 36};
        const awe::HDual gamma(vt[2 + kPhiGamma], ((in.sA1 >> kDirGamma) & 1ull) ? 1.0 : 0.0,
                               ((in.sA2 >> kDirGamma) & 1ull) ? 1.0 : 0.0, 0.0);
        awe::ap2_node<awe::HDual>(in, gamma, th, a.cst, sink, n == 0);
    }
    __syncthreads();

    // ---- objective terms in direction space and the xdot(t_f) map terms (Radau nodes) --------
    const double w_track = pcost[kCostTracking] / a.cst[AWE_C_NORM_TRACKING];
    const double w_xdot = pcost[kCostXdotRegularisation] / a.cst[AWE_C_NORM_XDOT_REG];
    const double w_ureg = pcost[kCostURegularisation] / a.cst[AWE_C_NORM_U_REG];
    const double w_fict = pcost[kCostFictitious] / a.cst[AWE_C_NORM_FICTITIOUS];
    const double w_theta = pcost[kCostThetaRegularisation] / a.cst[AWE_C_NORM_THETA_REG];
    for (int n = 1 + wave; n < NN; n += kHessWaves) {
        const int p = lane;
        const int j = n - 1;
        const double wj = a.coll.w[j];
        const double* w = wn + n * 64;
        const double* rcx = pst + kPstRef + 2 * AWE_NX + AWE_NU + AWE_NZ + j * (AWE_NX + AWE_NZ);
        const double cxx = C[n * NN + n] * inv_h_tf;
        const double* tp = tang + toff(n);
        double* hn = hd + hoff(n);
        auto addp = [&](int q1, int q2, double v) { hn[ht->pidx[1][q1][q2]] += sigma * v; };
        const double cb = pcost[kCostBeta] * wj / a.cst[AWE_C_NORM_BETA];
        const double cp = -pcost[kCostPower] * wj / (double)a.n_k;
        double tfpart = 0.0, gt = 0.0;
        if (p < AWE_NX) {
            const double ai = pst[p] * w_track, bi = pst[AWE_NX + p] * w_xdot, xd = w[AWE_NX + p];
            addp(p, p, 2.0 * wj * psi * ai + cxx * cxx * 2.0 * wj * bi);
            addp(p, AWE_NX + p, cxx * 2.0 * wj * bi);
            addp(p, kDirTf, cxx * (-xd * inv_tf) * 2.0 * wj * bi);
            addp(p, kDirPsi, 2.0 * wj * ai * (w[p] - rcx[p]));
        } else if (p < 2 * AWE_NX) {
            const int i = p - AWE_NX;
            const double bi = pst[p] * w_xdot, xd = w[p];
            addp(p, p, 2.0 * wj * bi);
            addp(p, kDirTf, (-xd * inv_tf) * 2.0 * wj * bi);
            tfpart = (xd * inv_tf) * (xd * inv_tf) * 2.0 * wj * bi;
            // gradient of the node Lagrangian w.r.t. xdot_i: rows (first-order tangents) + objective
            double gi = sigma * wj * 2.0 * bi * xd;
            const int c = ct->dcolor[1][p];
            if (c >= 0) {
                const unsigned long long m = ct->dmask[1][p], cm = ct->cmask[1][c];
                for (unsigned long long mm = m; mm; mm &= mm - 1ull) {
                    const int r = __builtin_ctzll(mm);
                    gi += mu[n * 36 + r] * tp[ct->off[1][c] + __popcll(cm & ((1ull << r) - 1ull))];
                }
            }
            G[n * 24 + i] = gi;
            gt = gi * 2.0 * xd * inv_tf * inv_tf;
        } else if (p < 2 * AWE_NX + AWE_NU) {
            const int i = p - 2 * AWE_NX;
            addp(p, p, 2.0 * wj * pst[p] * (i < 6 ? w_fict : w_ureg));
        } else if (p == kDirZ) {
            const double az = pst[kDirZ] * w_track;
            addp(p, p, 2.0 * wj * psi * az);
            addp(p, kDirPsi, 2.0 * wj * az * (w[kDirZ] - rcx[AWE_NX]));
        } else if (p == kDirDiam) {
            addp(p, p, 2.0 * wj * pst[kDirDiam] * w_theta);
        }
        if (p <= kDirGamma) {
            const int ip = ct->obj_power[p], ib = ct->obj_beta[p];
            if (ip >= 0) addp(p, kDirPsi, -cp * tp[ip]);
            if (ib >= 0) {
                const double bp = 2.0 * cb * tp[ib];
                for (int q = p; q <= kDirGamma; ++q) {
                    const int iq = ct->obj_beta[q];
                    if (iq >= 0) addp(p, q, bp * tp[iq]);
                }
            }
        }
        tfpart = wave_sum(tfpart);
        gt = wave_sum(gt);
        if (p == kDirTf) addp(kDirTf, kDirTf, tfpart);
        if (p == 0) G[n * 24 + 23] = gt;
    }
    __syncthreads();

    // ---- V-space entries: local CCS slots (contiguous) and the global-global partials ---------
    const int nloc = ha.nslot[k];
    const int e0 = ha.ent_off[k];
    const double ctf2 = inv_h_tf * inv_tf;
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
                const int i = (term >> 22) & 31, r = (term >> 19) & 7;
                v += G[n * 24 + i] * (-C[r * NN + n] * ctf2);
            } else {
                v += G[n * 24 + 23];
            }
        }
        if (e < nloc) Hb[e] = v;
        else gp[e - nloc] = v;
    }
}

// global-global entries: sum of the interval partials plus the time cost (objective.py)
__global__ __launch_bounds__(64) void ap2_hess_finalize_kernel(HKArgs ha) {
    const KArgs& a = ha.a;
    const int b = blockIdx.x;
    const int g = threadIdx.x;
    if (g >= ha.ng) return;
    double v = 0.0;
    for (int k = 0; k < a.n_k; ++k) v += ha.gpart[((size_t)b * a.n_k + k) * ha.ng + g];
    if (g == ha.g_tftf) v += ha.sigma[b] * 2.0 * a.P[(size_t)b * a.n_p + a.n_v + AWE_NW + kCostTf];
    ha.H[(size_t)b * ha.hnnz + ha.gslot[g]] = v;
}
}  // namespace

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
struct awe_handle_s {
    awt::Ap2Tables t;               // host tables (layout, pattern, colouring, gather list)
    awt::Ap2HessTables ht;          // Hessian structure, tasks and gather terms
    int batch = 0;
    size_t lds_bytes = 0, hess_lds_bytes = 0;
    int hd_total = 0, g_tftf = -1;
    awt::HessTabs* d_ht = nullptr;
    int* d_tasks = nullptr;
    short* d_task_target = nullptr;
    int* d_ent_off = nullptr;
    int* d_term_off = nullptr;
    unsigned* d_terms = nullptr;
    int* d_slot0 = nullptr;
    int* d_nslot = nullptr;
    int* d_gslot = nullptr;
    double* d_gpart = nullptr;
    double* d_scr_sigma = nullptr;
    double* d_scr_lam = nullptr;
    double* d_scr_H = nullptr;
    hipEvent_t hev[2] = {nullptr, nullptr};
    bool htimed = false;
    // device
    double* d_cst = nullptr;
    awt::ColorTabs* d_ct = nullptr;
    int* d_seg = nullptr;
    unsigned* d_glist = nullptr;
    int* d_glist_off = nullptr;
    double* d_partial = nullptr;
    // scratch for value-only calls and host wrappers
    double* d_scr_jac = nullptr;
    double* d_scr_grad = nullptr;
    double* d_scr_g = nullptr;
    double* d_scr_f = nullptr;
    double* d_in_V = nullptr;
    double* d_in_P = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool timed = false;
};

namespace {


template <int D>
int launch_interval(awe_handle h, const KArgs& a, hipStream_t stream) {
    constexpr int W = waves_for<D>();
    hipLaunchKernelGGL(ap2_interval_kernel<D>, dim3(h->batch * h->t.n_k), dim3(64 * W), h->lds_bytes,
                       stream, a);
    return AWE_OK;
}

int launch(awe_handle h, const double* V, const double* P, double* f, double* g, double* grad,
           double* jac, int want_derivs, hipStream_t stream) {
    KArgs a{};
    const awt::Ap2Tables& T = h->t;
    a.V = V; a.P = P; a.cst = h->d_cst; a.coll = T.dcoll; a.ct = h->d_ct;
    a.seg = h->d_seg; a.glist = h->d_glist; a.glist_off = h->d_glist_off;
    a.nscale = h->t.nscale; a.nconst = (int)h->t.kconst.size();
    for (size_t q = 0; q < h->t.kconst.size(); ++q) a.kconst[q] = h->t.kconst[q];
    a.g = g; a.jac = jac; a.grad = grad; a.partial = h->d_partial; a.f = f;
    a.n_k = h->t.n_k; a.d = h->t.d; a.n_v = h->t.lay.n_v; a.n_g = h->t.lay.n_g; a.n_p = h->t.lay.n_p;
    a.nnz = h->t.nnz; a.batch = h->batch; a.stride = h->t.lay.stride; a.rows = h->t.lay.rows;
    a.v_int0 = h->t.lay.v_int0; a.tang_total = h->t.tang_total;
    a.want_derivs = want_derivs;
    HIP_TRY(hipEventRecord(h->ev[0], stream));
    if (want_derivs) {
        switch (h->t.d) {
            case 1: launch_interval<1>(h, a, stream); break;
            case 2: launch_interval<2>(h, a, stream); break;
            case 3: launch_interval<3>(h, a, stream); break;
            case 4: launch_interval<4>(h, a, stream); break;
            case 5: launch_interval<5>(h, a, stream); break;
            default: return fail(AWE_ERR_ARG, "unsupported collocation degree");
        }
    } else {                                          // nlp_f / nlp_g: the value-only kernel
        const dim3 grid(h->batch * h->t.n_k), block(64);
        switch (h->t.d) {
            case 1: hipLaunchKernelGGL(ap2_value_kernel<1>, grid, block, 0, stream, a); break;
            case 2: hipLaunchKernelGGL(ap2_value_kernel<2>, grid, block, 0, stream, a); break;
            case 3: hipLaunchKernelGGL(ap2_value_kernel<3>, grid, block, 0, stream, a); break;
            case 4: hipLaunchKernelGGL(ap2_value_kernel<4>, grid, block, 0, stream, a); break;
            case 5: hipLaunchKernelGGL(ap2_value_kernel<5>, grid, block, 0, stream, a); break;
            default: return fail(AWE_ERR_ARG, "unsupported collocation degree");
        }
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev[1], stream));
    hipLaunchKernelGGL(ap2_finalize_kernel, dim3(h->batch), dim3(64), 0, stream, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev[2], stream));
    h->timed = true;
    return AWE_OK;
}

size_t lds_fixed_bytes(int d) {
    switch (d) {
        case 1: return sizeof(double) * lds_fixed_doubles<1>();
        case 2: return sizeof(double) * lds_fixed_doubles<2>();
        case 3: return sizeof(double) * lds_fixed_doubles<3>();
        case 4: return sizeof(double) * lds_fixed_doubles<4>();
        default: return sizeof(double) * lds_fixed_doubles<5>();
    }
}

size_t hess_lds_fixed_bytes(int d) {
    switch (d) {
        case 1: return sizeof(double) * hess_lds_fixed_doubles<1>();
        case 2: return sizeof(double) * hess_lds_fixed_doubles<2>();
        case 3: return sizeof(double) * hess_lds_fixed_doubles<3>();
        case 4: return sizeof(double) * hess_lds_fixed_doubles<4>();
        default: return sizeof(double) * hess_lds_fixed_doubles<5>();
    }
}

int launch_hess(awe_handle h, const double* V, const double* P, const double* sigma, const double* lam,
                double* H, hipStream_t stream) {
    const awt::Ap2Tables& T = h->t;
    const awt::Ap2HessTables& HT = h->ht;
    HKArgs ha{};
    KArgs& a = ha.a;
    a.V = V; a.P = P; a.cst = h->d_cst; a.coll = T.dcoll; a.ct = h->d_ct;
    a.n_k = T.n_k; a.d = T.d; a.n_v = T.lay.n_v; a.n_g = T.lay.n_g; a.n_p = T.lay.n_p;
    a.nnz = T.nnz; a.batch = h->batch; a.stride = T.lay.stride; a.rows = T.lay.rows;
    a.v_int0 = T.lay.v_int0; a.tang_total = T.tang_total;
    ha.ht = h->d_ht; ha.tasks = h->d_tasks; ha.task_target = h->d_task_target; ha.ent_off = h->d_ent_off;
    ha.term_off = h->d_term_off; ha.terms = h->d_terms; ha.slot0 = h->d_slot0; ha.nslot = h->d_nslot;
    ha.gslot = h->d_gslot; ha.sigma = sigma; ha.lam = lam; ha.H = H; ha.gpart = h->d_gpart;
    ha.hnnz = HT.nnz; ha.ng = (int)HT.gslot.size(); ha.hd_total = h->hd_total; ha.g_tftf = h->g_tftf;
    dim3 grid(h->batch * T.n_k), block(kHessThreads);
    HIP_TRY(hipEventRecord(h->hev[0], stream));
    switch (T.d) {
        case 1: hipLaunchKernelGGL(ap2_hess_kernel<1>, grid, block, h->hess_lds_bytes, stream, ha); break;
        case 2: hipLaunchKernelGGL(ap2_hess_kernel<2>, grid, block, h->hess_lds_bytes, stream, ha); break;
        case 3: hipLaunchKernelGGL(ap2_hess_kernel<3>, grid, block, h->hess_lds_bytes, stream, ha); break;
        case 4: hipLaunchKernelGGL(ap2_hess_kernel<4>, grid, block, h->hess_lds_bytes, stream, ha); break;
        case 5: hipLaunchKernelGGL(ap2_hess_kernel<5>, grid, block, h->hess_lds_bytes, stream, ha); break;
        default: return fail(AWE_ERR_ARG, "unsupported collocation degree");
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->hev[1], stream));
    hipLaunchKernelGGL(ap2_hess_finalize_kernel, dim3(h->batch), dim3(64), 0, stream, ha);
    HIP_TRY(hipGetLastError());
    h->htimed = true;
    return AWE_OK;
}

}  // namespace

extern "C" {

const char* awe_last_error(void) { return g_last_error.c_str(); }

int awe_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int awe_create(int n_k, int d, const double* consts, int n_consts, int batch, awe_handle* out) {
    if (!out || !consts) return fail(AWE_ERR_ARG, "null argument");
    if (n_consts != AWE_NCONST) return fail(AWE_ERR_ARG, "consts must have AWE_NCONST entries");
    if (n_k < 1 || d < 1 || d > 5 || batch < 1) return fail(AWE_ERR_ARG, "bad n_k/d/batch");
    if ((int)consts[AWE_C_N_K] != n_k || (int)consts[AWE_C_D] != d)
        return fail(AWE_ERR_ARG, "consts n_k/d mismatch");
    if (awe_device_count() <= 0)
        return fail(AWE_ERR_NODEVICE, "no HIP device visible: the HIP evaluator has no CPU fallback");

    auto h = new awe_handle_s();
    h->batch = batch;
    std::string err;
    int rc = awt::build_ap2_tables(n_k, d, consts, n_consts, h->t, err);
    if (rc) { delete h; return fail(rc, err); }
    const awt::Ap2Tables& T = h->t;
    h->lds_bytes = lds_fixed_bytes(d) + sizeof(double) * (size_t)(T.tang_total + 1);
    if (h->lds_bytes > 65536) { delete h; return fail(AWE_ERR_ARG, "internal: LDS image exceeds 64 KiB"); }
    rc = awt::build_hess_tables(T, h->ht, err);
    if (rc) { delete h; return fail(rc, err); }
    const awt::Ap2HessTables& HT = h->ht;
    h->hd_total = HT.ht.npairs[0] + d * HT.ht.npairs[1];
    h->hess_lds_bytes = hess_lds_fixed_bytes(d) + sizeof(double) * (size_t)(T.tang_total + 1 + h->hd_total);
    if (h->hess_lds_bytes > 65536) { delete h; return fail(AWE_ERR_ARG, "internal: Hessian LDS image exceeds 64 KiB"); }
    for (size_t g = 0; g < HT.gslot.size(); ++g) {
        const int slot = HT.gslot[g], itf = T.lay.theta(1);
        if (HT.row[slot] == itf && slot >= HT.colind[itf] && slot < HT.colind[itf + 1]) h->g_tftf = (int)g;
    }

#define ALLOC_COPY(dst, src, n)                                                     \
    HIP_TRY(hipMalloc((void**)&dst, sizeof(*dst) * (n)));                          \
    HIP_TRY(hipMemcpy(dst, src, sizeof(*dst) * (n), hipMemcpyHostToDevice))
    ALLOC_COPY(h->d_cst, T.cst.data(), T.cst.size());
    ALLOC_COPY(h->d_ct, &T.ct, 1);
    ALLOC_COPY(h->d_seg, T.seg.data(), T.seg.size());
    ALLOC_COPY(h->d_glist, T.glist.data(), T.glist.size());
    ALLOC_COPY(h->d_glist_off, T.glist_off.data(), T.glist_off.size());
    ALLOC_COPY(h->d_ht, &HT.ht, 1);
    ALLOC_COPY(h->d_tasks, HT.tasks.data(), HT.tasks.size());
    ALLOC_COPY(h->d_task_target, HT.task_target.data(), HT.task_target.size());
    ALLOC_COPY(h->d_ent_off, HT.ent_off.data(), HT.ent_off.size());
    ALLOC_COPY(h->d_term_off, HT.term_off.data(), HT.term_off.size());
    ALLOC_COPY(h->d_terms, HT.terms.data(), HT.terms.size());
    ALLOC_COPY(h->d_slot0, HT.slot0.data(), HT.slot0.size());
    ALLOC_COPY(h->d_nslot, HT.nslot.data(), HT.nslot.size());
    ALLOC_COPY(h->d_gslot, HT.gslot.data(), HT.gslot.size());
#undef ALLOC_COPY
    HIP_TRY(hipMalloc((void**)&h->d_gpart, sizeof(double) * (size_t)batch * n_k * std::max<size_t>(1, HT.gslot.size())));
    for (int i = 0; i < 2; ++i) HIP_TRY(hipEventCreate(&h->hev[i]));
    HIP_TRY(hipMalloc((void**)&h->d_partial, sizeof(double) * (size_t)batch * n_k * kNPartial));
    for (int i = 0; i < 3; ++i) HIP_TRY(hipEventCreate(&h->ev[i]));
    *out = h;
    return AWE_OK;
}

int awe_sparsity_jac_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind,
                            int* row) {
    if (!consts || !nnz) return fail(AWE_ERR_ARG, "null argument");
    if (n_consts != AWE_NCONST) return fail(AWE_ERR_ARG, "consts must have AWE_NCONST entries");
    if (n_k < 1 || d < 1 || d > 5) return fail(AWE_ERR_ARG, "bad n_k/d");
    if ((int)consts[AWE_C_N_K] != n_k || (int)consts[AWE_C_D] != d)
        return fail(AWE_ERR_ARG, "consts n_k/d mismatch");
    awt::Ap2Tables T;
    std::string err;
    int rc = awt::build_ap2_tables(n_k, d, consts, n_consts, T, err);
    if (rc) return fail(rc, err);
    *nnz = T.nnz;
    if (colind) std::memcpy(colind, T.colind.data(), sizeof(int) * T.colind.size());
    if (row) std::memcpy(row, T.row.data(), sizeof(int) * T.row.size());
    return AWE_OK;
}

int awe_destroy(awe_handle h) {
    if (!h) return AWE_OK;
    hipFree(h->d_cst); hipFree(h->d_ct); hipFree(h->d_seg);
    hipFree(h->d_glist); hipFree(h->d_glist_off); hipFree(h->d_partial);
    hipFree(h->d_scr_jac); hipFree(h->d_scr_grad); hipFree(h->d_scr_g); hipFree(h->d_scr_f);
    hipFree(h->d_in_V); hipFree(h->d_in_P);
    hipFree(h->d_ht); hipFree(h->d_tasks); hipFree(h->d_task_target); hipFree(h->d_ent_off);
    hipFree(h->d_term_off); hipFree(h->d_terms); hipFree(h->d_slot0); hipFree(h->d_nslot);
    hipFree(h->d_gslot); hipFree(h->d_gpart); hipFree(h->d_scr_sigma); hipFree(h->d_scr_lam);
    hipFree(h->d_scr_H);
    for (int i = 0; i < 3; ++i) if (h->ev[i]) hipEventDestroy(h->ev[i]);
    for (int i = 0; i < 2; ++i) if (h->hev[i]) hipEventDestroy(h->hev[i]);
    delete h;
    return AWE_OK;
}

int awe_sizes(awe_handle h, int* n_v, int* n_g, int* n_p, int* nnz_jac) {
    if (!h) return fail(AWE_ERR_ARG, "null handle");
    if (n_v) *n_v = h->t.lay.n_v;
    if (n_g) *n_g = h->t.lay.n_g;
    if (n_p) *n_p = h->t.lay.n_p;
    if (nnz_jac) *nnz_jac = h->t.nnz;
    return AWE_OK;
}

int awe_sparsity_jac(awe_handle h, int* colind, int* row) {
    if (!h || !colind || !row) return fail(AWE_ERR_ARG, "null argument");
    std::memcpy(colind, h->t.colind.data(), sizeof(int) * h->t.colind.size());
    std::memcpy(row, h->t.row.data(), sizeof(int) * h->t.row.size());
    return AWE_OK;
}

static int ensure_scratch(awe_handle h) {
    if (!h->d_scr_jac) HIP_TRY(hipMalloc((void**)&h->d_scr_jac, sizeof(double) * (size_t)h->batch * h->t.nnz));
    if (!h->d_scr_grad) HIP_TRY(hipMalloc((void**)&h->d_scr_grad, sizeof(double) * (size_t)h->batch * h->t.lay.n_v));
    if (!h->d_scr_g) HIP_TRY(hipMalloc((void**)&h->d_scr_g, sizeof(double) * (size_t)h->batch * h->t.lay.n_g));
    if (!h->d_scr_f) HIP_TRY(hipMalloc((void**)&h->d_scr_f, sizeof(double) * (size_t)h->batch));
    return AWE_OK;
}

int awe_eval_nlp(awe_handle h, const double* V, const double* P, double* f, double* g,
                 double* grad_f, double* jac, void* stream) {
    if (!h || !V || !P || !f || !g || !grad_f || !jac) return fail(AWE_ERR_ARG, "null argument");
    return launch(h, V, P, f, g, grad_f, jac, 1, (hipStream_t)stream);
}

int awe_eval_g(awe_handle h, const double* V, const double* P, double* g, void* stream) {
    if (!h || !V || !P || !g) return fail(AWE_ERR_ARG, "null argument");
    int rc = ensure_scratch(h);
    if (rc) return rc;
    return launch(h, V, P, h->d_scr_f, g, h->d_scr_grad, h->d_scr_jac, 0, (hipStream_t)stream);
}

int awe_eval_f(awe_handle h, const double* V, const double* P, double* f, void* stream) {
    if (!h || !V || !P || !f) return fail(AWE_ERR_ARG, "null argument");
    int rc = ensure_scratch(h);
    if (rc) return rc;
    return launch(h, V, P, f, h->d_scr_g, h->d_scr_grad, h->d_scr_jac, 0, (hipStream_t)stream);
}

int awe_eval_nlp_host(awe_handle h, const double* V, const double* P, double* f, double* g,
                      double* grad_f, double* jac) {
    if (!h || !V || !P || !f || !g || !grad_f || !jac) return fail(AWE_ERR_ARG, "null argument");
    int rc = ensure_scratch(h);
    if (rc) return rc;
    const size_t nb = (size_t)h->batch;
    if (!h->d_in_V) HIP_TRY(hipMalloc((void**)&h->d_in_V, sizeof(double) * nb * h->t.lay.n_v));
    if (!h->d_in_P) HIP_TRY(hipMalloc((void**)&h->d_in_P, sizeof(double) * nb * h->t.lay.n_p));
    HIP_TRY(hipMemcpy(h->d_in_V, V, sizeof(double) * nb * h->t.lay.n_v, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->d_in_P, P, sizeof(double) * nb * h->t.lay.n_p, hipMemcpyHostToDevice));
    rc = launch(h, h->d_in_V, h->d_in_P, h->d_scr_f, h->d_scr_g, h->d_scr_grad, h->d_scr_jac, 1, nullptr);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(f, h->d_scr_f, sizeof(double) * nb, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(g, h->d_scr_g, sizeof(double) * nb * h->t.lay.n_g, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(grad_f, h->d_scr_grad, sizeof(double) * nb * h->t.lay.n_v, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(jac, h->d_scr_jac, sizeof(double) * nb * h->t.nnz, hipMemcpyDeviceToHost));
    auto finite = [](const double* x, size_t n) {
        for (size_t i = 0; i < n; ++i) if (!std::isfinite(x[i])) return false;
        return true;
    };
    if (!finite(f, nb) || !finite(g, nb * h->t.lay.n_g) || !finite(grad_f, nb * h->t.lay.n_v) ||
        !finite(jac, nb * h->t.nnz))
        return fail(AWE_ERR_NONFINITE, "non-finite value in NLP evaluation");
    return AWE_OK;
}

static int eval_value_host(awe_handle h, const double* V, const double* P, double* f, double* g) {
    int rc = ensure_scratch(h);
    if (rc) return rc;
    const size_t nb = (size_t)h->batch;
    if (!h->d_in_V) HIP_TRY(hipMalloc((void**)&h->d_in_V, sizeof(double) * nb * h->t.lay.n_v));
    if (!h->d_in_P) HIP_TRY(hipMalloc((void**)&h->d_in_P, sizeof(double) * nb * h->t.lay.n_p));
    HIP_TRY(hipMemcpy(h->d_in_V, V, sizeof(double) * nb * h->t.lay.n_v, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->d_in_P, P, sizeof(double) * nb * h->t.lay.n_p, hipMemcpyHostToDevice));
    rc = launch(h, h->d_in_V, h->d_in_P, h->d_scr_f, h->d_scr_g, h->d_scr_grad, h->d_scr_jac, 0, nullptr);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    bool ok = true;
    if (f) {
        HIP_TRY(hipMemcpy(f, h->d_scr_f, sizeof(double) * nb, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < nb; ++i) ok = ok && std::isfinite(f[i]);
    }
    if (g) {
        HIP_TRY(hipMemcpy(g, h->d_scr_g, sizeof(double) * nb * h->t.lay.n_g, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < nb * (size_t)h->t.lay.n_g; ++i) ok = ok && std::isfinite(g[i]);
    }
    if (!ok) return fail(AWE_ERR_NONFINITE, "non-finite value in NLP evaluation");
    return AWE_OK;
}

int awe_eval_f_host(awe_handle h, const double* V, const double* P, double* f) {
    if (!h || !V || !P || !f) return fail(AWE_ERR_ARG, "null argument");
    return eval_value_host(h, V, P, f, nullptr);
}

int awe_eval_g_host(awe_handle h, const double* V, const double* P, double* g) {
    if (!h || !V || !P || !g) return fail(AWE_ERR_ARG, "null argument");
    return eval_value_host(h, V, P, nullptr, g);
}

int awe_hess_nnz(awe_handle h, int* nnz_h) {
    if (!h || !nnz_h) return fail(AWE_ERR_ARG, "null argument");
    *nnz_h = h->ht.nnz;
    return AWE_OK;
}

int awe_sparsity_hess(awe_handle h, int* colind, int* row) {
    if (!h || !colind || !row) return fail(AWE_ERR_ARG, "null argument");
    std::memcpy(colind, h->ht.colind.data(), sizeof(int) * h->ht.colind.size());
    std::memcpy(row, h->ht.row.data(), sizeof(int) * h->ht.row.size());
    return AWE_OK;
}

int awe_sparsity_hess_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind,
                             int* row) {
    if (!consts || !nnz) return fail(AWE_ERR_ARG, "null argument");
    if (n_consts != AWE_NCONST) return fail(AWE_ERR_ARG, "consts must have AWE_NCONST entries");
    if (n_k < 1 || d < 1 || d > 5) return fail(AWE_ERR_ARG, "bad n_k/d");
    if ((int)consts[AWE_C_N_K] != n_k || (int)consts[AWE_C_D] != d)
        return fail(AWE_ERR_ARG, "consts n_k/d mismatch");
    awt::Ap2Tables T;
    awt::Ap2HessTables H;
    std::string err;
    int rc = awt::build_ap2_tables(n_k, d, consts, n_consts, T, err);
    if (!rc) rc = awt::build_hess_tables(T, H, err);
    if (rc) return fail(rc, err);
    *nnz = H.nnz;
    if (colind) std::memcpy(colind, H.colind.data(), sizeof(int) * H.colind.size());
    if (row) std::memcpy(row, H.row.data(), sizeof(int) * H.row.size());
    return AWE_OK;
}

int awe_eval_hess(awe_handle h, const double* V, const double* P, const double* sigma, const double* lam_g,
                  double* H, void* stream) {
    if (!h || !V || !P || !sigma || !lam_g || !H) return fail(AWE_ERR_ARG, "null argument");
    return launch_hess(h, V, P, sigma, lam_g, H, (hipStream_t)stream);
}

int awe_eval_hess_host(awe_handle h, const double* V, const double* P, const double* sigma,
                       const double* lam_g, double* H) {
    if (!h || !V || !P || !sigma || !lam_g || !H) return fail(AWE_ERR_ARG, "null argument");
    const size_t nb = (size_t)h->batch;
    const awt::Ap2Tables& T = h->t;
    if (!h->d_in_V) HIP_TRY(hipMalloc((void**)&h->d_in_V, sizeof(double) * nb * T.lay.n_v));
    if (!h->d_in_P) HIP_TRY(hipMalloc((void**)&h->d_in_P, sizeof(double) * nb * T.lay.n_p));
    if (!h->d_scr_sigma) HIP_TRY(hipMalloc((void**)&h->d_scr_sigma, sizeof(double) * nb));
    if (!h->d_scr_lam) HIP_TRY(hipMalloc((void**)&h->d_scr_lam, sizeof(double) * nb * T.lay.n_g));
    if (!h->d_scr_H) HIP_TRY(hipMalloc((void**)&h->d_scr_H, sizeof(double) * nb * h->ht.nnz));
    HIP_TRY(hipMemcpy(h->d_in_V, V, sizeof(double) * nb * T.lay.n_v, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->d_in_P, P, sizeof(double) * nb * T.lay.n_p, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->d_scr_sigma, sigma, sizeof(double) * nb, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->d_scr_lam, lam_g, sizeof(double) * nb * T.lay.n_g, hipMemcpyHostToDevice));
    int rc = launch_hess(h, h->d_in_V, h->d_in_P, h->d_scr_sigma, h->d_scr_lam, h->d_scr_H, nullptr);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(H, h->d_scr_H, sizeof(double) * nb * h->ht.nnz, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nb * h->ht.nnz; ++i)
        if (!std::isfinite(H[i])) return fail(AWE_ERR_NONFINITE, "non-finite value in the Hessian");
    return AWE_OK;
}

int awe_last_hess_ms(awe_handle h, float* ms) {
    if (!h || !h->htimed || !ms) return fail(AWE_ERR_ARG, "no timed Hessian launch yet");
    HIP_TRY(hipEventSynchronize(h->hev[1]));
    HIP_TRY(hipEventElapsedTime(ms, h->hev[0], h->hev[1]));
    return AWE_OK;
}

int awe_last_kernel_ms(awe_handle h, float* ms_main, float* ms_finalize) {
    if (!h || !h->timed) return fail(AWE_ERR_ARG, "no timed launch yet");
    HIP_TRY(hipEventSynchronize(h->ev[2]));
    if (ms_main) HIP_TRY(hipEventElapsedTime(ms_main, h->ev[0], h->ev[1]));
    if (ms_finalize) HIP_TRY(hipEventElapsedTime(ms_finalize, h->ev[1], h->ev[2]));
    return AWE_OK;
}

}  // extern "C"
