// awempc -- MI355X (gfx950) evaluator for the awebox tracking-MPC NLP of a 3-DOF kite
// (pmpc.py:193-217; SURVEY.md section 8 row a37, config 5: B MPC instances per launch).
//
// Execution model (same shape as the AP2 evaluator, awegpu.hip, specialised for the small node):
//   * one workgroup per (MPC instance, horizon interval), W = ceil((d+1)/2) wavefronts; the
//     interval's slice of V and the parameters it reads are staged in LDS with coalesced loads;
//   * model pass: every half-wavefront evaluates ONE node of kite3_node in forward-mode dual
//     arithmetic with one seed direction per lane -- 31 node variables + phi.gamma = 32 lanes, so
//     a wavefront produces two complete node Jacobian blocks and no colouring is needed.  The
//     collocation chain rule xdot = C X / (h tf) is folded into the seeds (kite3_tables.hpp);
//   * tracking objective (pmpc.py:304-358) and its gradient are closed-form per V column;
//   * J_g values come from a host-built gather list (one entry per CCS slot: tangent index and
//     polynomial scale, or a constant for the initial-condition and continuity rows), so the J
//     stores of one interval are contiguous; a one-wave finalize kernel per instance reduces the
//     interval objective partials in a fixed order and adds the terminal cost (no float atomics).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <type_traits>
#include <string>
#include <vector>

#include "../../include/awegpu.h"
#include "../../include/awempc.h"
#include "im_layout.hpp"
#include "kite3_model.hpp"
#include "kite3_nodejac.gen.hpp"
#include "kite3_tables.hpp"

namespace {

using namespace k3t;

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define MPC_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess)                                                          \
            return fail(AWE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

struct MArgs {
    int n_k, d, n_v, n_g, n_p, nnz, stride;
    const double* V;
    const double* P;
    double* f;
    double* g;
    double* grad;
    double* jac;
    const double* cst;
    const awt::DevColl* coll;
    const int* goff;
    const int* gslot;
    const uint32_t* gcode;
    double* fpart;       // [B][n_k]
};

struct LaneIn {
    const double* w;     // node values (scaled), [32]
    const double* nc;    // LDS: C[n][n] / (h tf) at a Radau node (0 at the shooting node), 1 / tf
    int lane;
    __device__ __forceinline__ awe::Dual operator()(int i) const {
        double t = (i == lane) ? 1.0 : 0.0;
        if (i >= K3_NX && i < 2 * K3_NX) {
            // re-read at each use (volatile): two fewer live doubles per lane in the model pass
            const volatile double* vn = nc;
            if (lane == i - K3_NX) t = vn[0];
            if (lane == kDirTf) t = -w[i] * vn[1];
        }
        return awe::Dual(w[i], t);
    }
};

struct LaneSink {
    double* tang;        // node base: [row][32]
    double* gval;        // node base: [16]
    int lane;
    __device__ __forceinline__ void eq_row(int r, const awe::Dual& v) {
        tang[r * kLanes + lane] = v.d;
        if (lane == 0) gval[r] = v.v;
    }
    __device__ __forceinline__ void ineq_row(int r, const awe::Dual& v) { eq_row(K3_N_EQ + r, v); }
};

// Main-tether drag preaccumulated per node (K3InlineDrag's element sum): values and partials
// w.r.t. the scaled node variables q0..2, dq0..2, diam_t; pr = D[3] | dD/d(var j)[7][3].
constexpr int kDragDirs = 7, kDragStride = 24;
__device__ __forceinline__ int drag_var(int j) { return j < 6 ? j : awe::k3::TH_DIAM; }

struct LdsDrag {
    const double* pr;
    int lane;
    __device__ __forceinline__ void operator()(const awe::Dual*, const awe::Dual*, const awe::Dual&, double,
                                               const double*, awe::Dual D[3]) const {
        // lane = direction (uncompressed seeds): its tangent is the partial along its own variable
        const int j = lane < 6 ? lane : (lane == awe::k3::TH_DIAM ? 6 : -1);
#pragma unroll
        for (int i = 0; i < 3; ++i) D[i] = awe::Dual(pr[i], j >= 0 ? pr[3 + 3 * j + i] : 0.0);
    }
};

template <int D>
constexpr int waves_for() { return (D + 2) / 2; }

template <int D>
// 3 waves per SIMD (168 VGPRs, 15 spilled): four 3-wave workgroups per CU; 0.190 -> 0.146 ms at B = 256
// against 225 VGPRs and two workgroups (tools/mpc_variants.py)
__global__ __launch_bounds__(64 * waves_for<D>(), 3) void mpc_interval_kernel(MArgs a) {
    constexpr int NN = D + 1;
    constexpr int NT = 64 * waves_for<D>();
    constexpr int STRIDE = K3_NX + K3_NU + K3_NX + K3_NZ + D * (K3_NX + K3_NZ);
    constexpr int NLOC = 9 + STRIDE + K3_NX;
    __shared__ double vloc[NLOC];                  // theta, phi, x[k], u, xdot, z, coll.., x[k+1]
    __shared__ double rloc[STRIDE + K3_NX];        // p.ref slice of the same block
    __shared__ double wts[K3_NX + K3_NZ + K3_NU];  // Q, Z(=1), R
    __shared__ double wn[NN][kLanes];
    __shared__ double tang[NN * kRowsPerNode * kLanes];
    __shared__ double gval[NN][16];
    __shared__ double fterm[STRIDE];
    __shared__ double pre[NN][kDragStride];
    __shared__ double nodec[NN][2];

    const int b = blockIdx.x / a.n_k, k = blockIdx.x % a.n_k;
    const int tid = threadIdx.x;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const int base = 9 + 2 + k * STRIDE;            // v_int0 = 11
    // ---- stage ---------------------------------------------------------------------------
    for (int i = tid; i < NLOC; i += NT) vloc[i] = i < 9 ? V[i] : V[base + (i - 9)];
    const double* pref = P + K3_NX;                 // p.ref (V-shaped)
    for (int i = tid; i < STRIDE + K3_NX; i += NT) rloc[i] = pref[base + i];
    const double u_ref = P[K3_NX + a.n_v];
    const double* pQ = P + K3_NX + a.n_v + 1;
    for (int i = tid; i < K3_NX + K3_NZ + K3_NU; i += NT)
        wts[i] = i < K3_NX ? pQ[i] : (i == K3_NX ? 1.0 : pQ[K3_NX + (i - K3_NX - 1)]);
    __syncthreads();

    const double tf = vloc[1];
    const double inv_h_tf = (double)a.n_k / tf;
    const double* C = a.coll->C;                    // C[j*(d+1)+r] = l_j'(tau_r)
    const double* xk = vloc + 9;
    const double* uk = xk + K3_NX;
    const double* xdk = uk + K3_NU;
    const double* zk = xdk + K3_NX;
    const double* coll = zk + K3_NZ;
    const double* xk1 = coll + D * (K3_NX + K3_NZ);
    auto Xv = [&](int r, int i) -> double { return r == 0 ? xk[i] : coll[(r - 1) * (K3_NX + K3_NZ) + i]; };

    // ---- node values -----------------------------------------------------------------------
    for (int t = tid; t < NN * kLanes; t += NT) {
        const int n = t / kLanes, i = t % kLanes;
        double val;
        if (i < K3_NX) val = Xv(n, i);
        else if (i < 2 * K3_NX) {
            if (n == 0) val = xdk[i - K3_NX];
            else {
                double s = 0.0;
                for (int r = 0; r < NN; ++r) s += C[r * NN + n] * Xv(r, i - K3_NX);
                val = s * inv_h_tf;
            }
        } else if (i < 2 * K3_NX + K3_NU) val = uk[i - 2 * K3_NX];
        else if (i == 2 * K3_NX + K3_NU) val = n == 0 ? zk[0] : coll[(n - 1) * (K3_NX + K3_NZ) + K3_NX];
        else if (i < K3_NW) val = vloc[i - (2 * K3_NX + K3_NU + K3_NZ)];
        else val = vloc[2];                         // phi.gamma
        wn[n][i] = val;
    }
    __syncthreads();

    if (tid < NN) {
        nodec[tid][0] = tid > 0 ? C[tid * NN + tid] * inv_h_tf : 0.0;
        nodec[tid][1] = tid > 0 ? 1.0 / tf : 0.0;     // the t_f direction acts at Radau nodes only
    }
    // ---- tether drag, one (node, direction) per thread: the element sum in the model's order --
    for (int t = tid; t < NN * kDragDirs; t += NT) {
        const int n = t / kDragDirs, j = t - n * kDragDirs, vj = drag_var(j);
        const double* s = a.cst + K3_C_SCALING;
        awe::Dual q[3], v[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            q[i] = awe::Dual(wn[n][awe::k3::Q + i], vj == awe::k3::Q + i ? 1.0 : 0.0) * s[awe::k3::Q + i];
            v[i] = awe::Dual(wn[n][awe::k3::DQ + i], vj == awe::k3::DQ + i ? 1.0 : 0.0) * s[awe::k3::DQ + i];
        }
        const awe::Dual diam = awe::Dual(wn[n][awe::k3::TH_DIAM], vj == awe::k3::TH_DIAM ? 1.0 : 0.0) * s[awe::k3::TH_DIAM];
        awe::Dual Dt[3];
        awe::K3InlineDrag()(q, v, diam, u_ref, a.cst, Dt);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (j == 0) pre[n][i] = Dt[i].v;
            pre[n][3 + 3 * j + i] = Dt[i].d;
        }
    }
    __syncthreads();

    // ---- model pass: half-wave = node, lane = direction --------------------------------------
    {
        const int n = tid / kLanes, lane = tid % kLanes;
        if (n < NN) {
            LaneIn in{wn[n], nodec[n], lane};
            LaneSink sink{tang + n * kRowsPerNode * kLanes, gval[n], lane};
            awe::Dual gamma(wn[n][kDirGamma], lane == kDirGamma ? 1.0 : 0.0);
            awe::kite3_node<awe::Dual>(in, gamma, u_ref, a.cst, sink, n == 0, LdsDrag{pre[n], lane});
        }
    }
    // ---- tracking objective: per local column (pmpc.py:304-358) -----------------------------
    double* grad = a.grad + (size_t)b * a.n_v + base;
    const double* w = a.coll->w;
    const double invN = 1.0 / a.n_k;
    for (int c = tid; c < STRIDE; c += NT) {
        double gr = 0.0, ft = 0.0;
        if (c >= K3_NX && c < K3_NX + K3_NU) {                       // u[k], zero-order hold
            const int i = c - K3_NX;
            const double e = vloc[9 + c] - rloc[c], W = wts[K3_NX + K3_NZ + i];
            double sw = 0.0;
            for (int j = 0; j < D; ++j) sw += w[j];
            gr = 2.0 * sw * W * e * invN;
            ft = sw * W * e * e;
        } else if (c >= 2 * K3_NX + K3_NU + K3_NZ) {                 // coll_var[k][j] = {x, z}
            const int q = c - (2 * K3_NX + K3_NU + K3_NZ);
            const int j = q / (K3_NX + K3_NZ), e_ = q % (K3_NX + K3_NZ);
            const double e = vloc[9 + c] - rloc[c], W = wts[e_];
            gr = 2.0 * w[j] * W * e * invN;
            ft = w[j] * W * e * e;
        }
        grad[c] = gr;
        fterm[c] = ft;
    }
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int c = 0; c < STRIDE; ++c) s += fterm[c];
        a.fpart[(size_t)b * a.n_k + k] = s * invN;
    }

    // ---- g ---------------------------------------------------------------------------------------
    double* g = a.g + (size_t)b * a.n_g;
    const int row0 = K3_NX + k * (K3_N_EQ + K3_N_INEQ + D * K3_N_EQ + K3_NX);
    constexpr int ROWS = K3_N_EQ + K3_N_INEQ + D * K3_N_EQ + K3_NX;
    const double* Dc = a.coll->D;
    for (int r = tid; r < ROWS; r += NT) {
        double val;
        if (r < K3_N_EQ + K3_N_INEQ) val = gval[0][r];
        else if (r < K3_N_EQ + K3_N_INEQ + D * K3_N_EQ) {
            const int q = r - (K3_N_EQ + K3_N_INEQ);
            val = gval[1 + q / K3_N_EQ][q % K3_N_EQ];
        } else {
            const int i = r - (K3_N_EQ + K3_N_INEQ + D * K3_N_EQ);
            double s = 0.0;
            for (int rr = 0; rr < NN; ++rr) s += Dc[rr] * Xv(rr, i);
            val = xk1[i] - s;
        }
        g[row0 + r] = val;
    }
    if (k == 0)
        for (int i = tid; i < K3_NX; i += NT) g[i] = xk[i] - P[i];     // initial conditions

    // ---- J_g values through the gather list ------------------------------------------------------
    double* jac = a.jac + (size_t)b * a.nnz;
    const int e0 = a.goff[k], e1 = a.goff[k + 1];
    for (int e = e0 + tid; e < e1; e += NT) {
        const uint32_t cd = a.gcode[e];
        const uint32_t kind = cd >> 29;
        const int rr = (cd >> 25) & 15, n = (cd >> 21) & 15, idx = cd & ((1u << 21) - 1u);
        double val;
        if (kind == kKindTang) val = tang[idx];
        else if (kind == kKindTangPoly) val = tang[idx] * (C[rr * NN + n] * inv_h_tf);
        else if (kind == kKindOne) val = 1.0;
        else val = -Dc[rr];
        __builtin_nontemporal_store(val, &jac[a.gslot[e]]);  // written once (as the AP2 path's J_g)
    }
}

// one wave per instance: objective partials in a fixed order, terminal cost, global gradient
__global__ __launch_bounds__(64) void mpc_finalize_kernel(MArgs a) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* ref = P + K3_NX;
    const double* pP = P + K3_NX + a.n_v + 1 + K3_NX + K3_NU;
    double* grad = a.grad + (size_t)b * a.n_v;
    const int xN = 11 + a.n_k * a.stride;
    double term = 0.0;
    if (lane < K3_NX) {
        const double e = V[xN + lane] - ref[xN + lane];
        grad[xN + lane] = 2.0 * pP[lane] * e;
        term = pP[lane] * e * e;
    }
    if (lane < 11) grad[lane] = 0.0;                     // theta, phi, xi
    __shared__ double tt[64];
    tt[lane] = term;
    __syncthreads();
    if (lane == 0) {
        double s = 0.0;
        for (int k = 0; k < a.n_k; ++k) s += a.fpart[(size_t)b * a.n_k + k];
        for (int i = 0; i < K3_NX; ++i) s += tt[i];
        a.f[b] = s;
    }
}

// ---------------------------------------------------------------------------------------------
// nlp_hess_l: sigma f + lam^T g (kite3_tables.hpp, build_hess_tables)
// ---------------------------------------------------------------------------------------------
struct HArgs {
    MArgs a;
    const double* sigma;     // [B]
    const double* lam;       // [B][n_g]
    double* H;               // [B][hnnz]
    double* gpart;           // [B][n_k][ng]
    const int* task;         // p | q << 8
    int ntask0, ntask1, npair1, hnnz, ng, hd_total;
    const int* slot0;
    const int* nslot;
    const int* ent_off;
    const int* term_off;
    const unsigned* terms;
    const int* gslot;
    const int* xnslot;
};

constexpr int kHessThreads = 256;

// hyper-dual node variable i: e1 along direction p, e2 along direction q (the first-order seeds)
struct LaneHIn {
    const double* w;
    int p, q;
    double cxx, inv_tf;      // C[n][n] / (h tf) and 1 / tf at a Radau node, 0 at the shooting node
    __device__ __forceinline__ double seed(int dir, int i) const {
        double t = (i == dir) ? 1.0 : 0.0;
        if (i >= K3_NX && i < 2 * K3_NX) {
            if (dir == i - K3_NX) t += cxx;
            if (dir == kDirTf) t += -w[i] * inv_tf;
        }
        return t;
    }
    __device__ __forceinline__ awe::HDual operator()(int i) const {
        return awe::HDual(w[i], seed(p, i), q == kGTask ? 0.0 : seed(q, i), 0.0);
    }
};

// sum_r mu_r d2F_r / de1 de2 (pair task) or sum_r mu_r dF_r / de1 (first-order task)
struct LaneHSink {
    const double* mu;
    bool first;
    double acc;
    __device__ __forceinline__ void eq_row(int r, const awe::HDual& v) { acc += mu[r] * (first ? v.a : v.ab); }
    __device__ __forceinline__ void ineq_row(int r, const awe::HDual& v) { eq_row(K3_N_EQ + r, v); }
};

template <int D>
__global__ __launch_bounds__(kHessThreads) void mpc_hess_kernel(HArgs ha) {
    const MArgs& a = ha.a;
    constexpr int NN = D + 1;
    constexpr int NT = kHessThreads;
    constexpr int STRIDE = K3_NX + K3_NU + K3_NX + K3_NZ + D * (K3_NX + K3_NZ);
    constexpr int NLOC = 9 + STRIDE + K3_NX;
    __shared__ double vloc[NLOC];
    __shared__ double wn[NN][kLanes];
    __shared__ double mu[NN][kRowsPerNode];
    __shared__ double wq[K3_NX + K3_NU];                  // Q, R tracking weights
    __shared__ double scl[1 + NN * NN];
    extern __shared__ double hd[];                        // [hd_total]: per node, its tasks' values

    const int b = blockIdx.x / a.n_k, k = blockIdx.x % a.n_k;
    const int tid = threadIdx.x;
    const double* V = a.V + (size_t)b * a.n_v;
    const double* P = a.P + (size_t)b * a.n_p;
    const double* lam = ha.lam + (size_t)b * a.n_g;
    const double sigma = ha.sigma[b];
    const int base = 9 + 2 + k * STRIDE;
    for (int i = tid; i < NLOC; i += NT) vloc[i] = i < 9 ? V[i] : V[base + (i - 9)];
    const double* pQ = P + K3_NX + a.n_v + 1;
    for (int i = tid; i < K3_NX + K3_NU; i += NT) wq[i] = pQ[i];
    const double u_ref = P[K3_NX + a.n_v];
    const int row0 = K3_NX + k * (K3_N_EQ + K3_N_INEQ + D * K3_N_EQ + K3_NX);
    for (int t = tid; t < NN * kRowsPerNode; t += NT) {
        const int n = t / kRowsPerNode, r = t % kRowsPerNode;
        double m = 0.0;
        if (n == 0) m = lam[row0 + r];
        else if (r < K3_N_EQ) m = lam[row0 + K3_N_EQ + K3_N_INEQ + (n - 1) * K3_N_EQ + r];
        mu[n][r] = m;
    }
    __syncthreads();
    const double tf = vloc[1];
    const double inv_h_tf = (double)a.n_k / tf, inv_tf = 1.0 / tf;
    const double* C = a.coll->C;
    for (int i = tid; i < 1 + NN * NN; i += NT) scl[i] = i == 0 ? 1.0 : C[i - 1] * inv_h_tf;
    const double* xk = vloc + 9;
    const double* uk = xk + K3_NX;
    const double* xdk = uk + K3_NU;
    const double* zk = xdk + K3_NX;
    const double* coll = zk + K3_NZ;
    auto Xv = [&](int r, int i) -> double { return r == 0 ? xk[i] : coll[(r - 1) * (K3_NX + K3_NZ) + i]; };
    for (int t = tid; t < NN * kLanes; t += NT) {
        const int n = t / kLanes, i = t % kLanes;
        double val;
        if (i < K3_NX) val = Xv(n, i);
        else if (i < 2 * K3_NX) {
            if (n == 0) val = xdk[i - K3_NX];
            else {
                double s = 0.0;
                for (int r = 0; r < NN; ++r) s += C[r * NN + n] * Xv(r, i - K3_NX);
                val = s * inv_h_tf;
            }
        } else if (i < 2 * K3_NX + K3_NU) val = uk[i - 2 * K3_NX];
        else if (i == 2 * K3_NX + K3_NU) val = n == 0 ? zk[0] : coll[(n - 1) * (K3_NX + K3_NZ) + K3_NX];
        else if (i < K3_NW) val = vloc[i - (2 * K3_NX + K3_NU + K3_NZ)];
        else val = vloc[2];                               // phi.gamma
        wn[n][i] = val;
    }
    __syncthreads();

    // ---- second-order pass: one (node, direction pair) per thread --------------------------------
    const int nt0 = ha.ntask0, nt1 = ha.ntask1;
    for (int t = tid; t < nt0 + D * nt1; t += NT) {
        const int n = t < nt0 ? 0 : 1 + (t - nt0) / nt1;
        const int ti = n == 0 ? t : (t - nt0) % nt1;
        const int pq = ha.task[(n == 0 ? 0 : nt0) + ti];
        LaneHIn in{wn[n], pq & 0xff, pq >> 8, n > 0 ? C[n * NN + n] * inv_h_tf : 0.0, n > 0 ? inv_tf : 0.0};
        LaneHSink sink{mu[n], in.q == kGTask, 0.0};
        const awe::HDual gamma(wn[n][kDirGamma], in.p == kDirGamma ? 1.0 : 0.0,
                               in.q == kDirGamma ? 1.0 : 0.0, 0.0);
        awe::kite3_node<awe::HDual>(in, gamma, u_ref, a.cst, sink, n == 0);
        hd[(n == 0 ? 0 : nt0 + (n - 1) * nt1) + ti] = sink.acc;
    }
    __syncthreads();

    // ---- V-space entries: the interval's contiguous local slots, then its global partials ---------
    const int nloc = ha.nslot[k];
    const int e0 = ha.ent_off[k];
    const double* w = a.coll->w;
    const double invN = 1.0 / a.n_k;
    double sw = 0.0;
    for (int j = 0; j < D; ++j) sw += w[j];
    double* Hb = ha.H + (size_t)b * ha.hnnz + ha.slot0[k];
    double* gp = ha.gpart + ((size_t)b * a.n_k + k) * ha.ng;
    auto hoff = [&](int n) { return n == 0 ? 0 : nt0 + (n - 1) * nt1; };
    for (int e = tid; e < nloc + ha.ng; e += NT) {
        double v = 0.0;
        for (int t = ha.term_off[e0 + e]; t < ha.term_off[e0 + e + 1]; ++t) {
            const unsigned term = ha.terms[t];
            const int type = term >> 30, n = (term >> 27) & 7;
            if (type == kHTA) {
                v += scl[(term >> 7) & 127] * scl[term & 127] * hd[hoff(n) + ((term >> 14) & 8191)];
            } else if (type == kHTB) {
                const int i = (term >> 22) & 31, r = (term >> 19) & 7;
                v += hd[hoff(n) + ha.npair1 + i] * (-C[r * NN + n] * inv_h_tf * inv_tf);
            } else if (type == kHTC) {
                const int i = (term >> 22) & 31;
                v += hd[hoff(n) + ha.npair1 + i] * (2.0 * wn[n][K3_NX + i] * inv_tf * inv_tf);
            } else {
                const int sub = (term >> 22) & 3, i = (term >> 17) & 31;
                const double wt = sub == 0 ? w[n - 1] * wq[i] : (sub == 1 ? w[n - 1] : sw * wq[K3_NX + i]);
                v += sigma * 2.0 * wt * invN;
            }
        }
        if (e < nloc) Hb[e] = v;
        else gp[e - nloc] = v;
    }
}

// global-global entries (sums of the interval partials, fixed order) and the terminal cost
__global__ __launch_bounds__(64) void mpc_hess_finalize_kernel(HArgs ha) {
    const MArgs& a = ha.a;
    const int b = blockIdx.x, lane = threadIdx.x;
    if (lane < ha.ng) {
        double v = 0.0;
        for (int k = 0; k < a.n_k; ++k) v += ha.gpart[((size_t)b * a.n_k + k) * ha.ng + lane];
        ha.H[(size_t)b * ha.hnnz + ha.gslot[lane]] = v;
    }
    if (lane < K3_NX) {
        const double* pP = a.P + (size_t)b * a.n_p + K3_NX + a.n_v + 1 + K3_NX + K3_NU;
        ha.H[(size_t)b * ha.hnnz + ha.xnslot[lane]] = ha.sigma[b] * 2.0 * pP[lane];
    }
}


// ---------------------------------------------------------------------------------------------
// Generated instance-minor path (awempc_eval_nlp_im): one lane per MPC instance.
//   mpc_gen_in (im::transpose_in_kernel): V, p -> VT[i * ld + b], PT[i * ld + b]
//   mpc_gen_node_kernel: three kinds of tiles in one launch, so that they run side by side --
//     Radau and shooting tiles: lane = instance, one wavefront per node, the node in the straight-line
//     code generated from kite3_node (kite3_nodejac.gen.hpp: the node's rows and the values of its
//     J_g pattern entries, no dual numbers, no zero tangents); each tangent slot goes straight to its
//     J_g entries (1, or the d polynomial columns X_r, r != n, of a Radau xdot direction, scaled by
//     C[r][n] / (h t_f)) through the node's destination row staged in LDS;
//     interval tiles: the interval's tracking-cost gradient and partial sum, continuity rows and
//     constant J_g entries, every load of the interval issued at once.
//   At the config-5 batch (256 instances) the launch is one round of wavefronts, so it takes as long
//   as its longest wavefront: in separate launches, with the interval work behind the shooting node
//   in a loop that waited on each column's loads, 0.070 ms; merged and unrolled 0.029 ms
//   (profiles/r05/mpc_ab/: direction strips on separate wavefronts and preloaded node inputs measured
//   no faster, outputs bitwise equal).
//   mpc_gen_finalize_kernel: objective (fixed order), terminal cost, global gradient rows.
// J_g and grad f leave instance-minor (jac[e * ldj + b]), every store one 512-byte row; g stays
// per-instance (g[b * n_g + i]) as the solver reads it.
// ---------------------------------------------------------------------------------------------
constexpr int kGenMaxTan = 128;
static_assert(awe_k3gen::kNTan[0] <= kGenMaxTan && awe_k3gen::kNTan[1] <= kGenMaxTan, "slot table too small");

// destination count of every tangent slot (1, or d for the xdot directions of a Radau node) and its
// first entry in the node's destination row; compile-time on the device (the generated code's slot
// numbers are constants), built with the run-time d on the host
struct GenSlotTab {
    int first[2][kGenMaxTan];
    int cnt[2][kGenMaxTan];
    int total[2];
    __host__ __device__ constexpr GenSlotTab(int d) : first(), cnt(), total() {
        for (int kind = 0; kind < 2; ++kind) {
            int dir_of[kGenMaxTan] = {};
            for (int s = 0; s < kGenMaxTan; ++s) dir_of[s] = -1;
            for (int r = 0; r < kRowsPerNode; ++r)
                for (int l = 0; l < kLanes; ++l)
                    if (awe_k3gen::kTanIdx[kind][r][l] >= 0) dir_of[awe_k3gen::kTanIdx[kind][r][l]] = l;
            int f = 0;
            for (int s = 0; s < awe_k3gen::kNTan[kind]; ++s) {
                const bool xd = kind == 1 && dir_of[s] >= K3_NX && dir_of[s] < 2 * K3_NX;
                first[kind][s] = f;
                cnt[kind][s] = xd ? d : 1;
                f += cnt[kind][s];
            }
            total[kind] = f;
        }
    }
};
template <int D>
constexpr GenSlotTab kGenSlots{D};

struct GenArgs {
    awt::DevColl coll;
    int n_k, batch, n_v, n_g, n_p, stride, v_int0, rows, nib, dstride;
    unsigned ld8;                // bytes between VT / PT / fpart rows
    unsigned ldj8;               // bytes between J_g / grad rows
    double kconst[8];            // constant J_g values: 1, -D[0..d]
};

// node inputs of node n of interval k (first column c0) from VT; n = 0 the shooting node
template <int D>
struct GenIn {
    const double* v;
    unsigned ld8, lb;
    int c0, n;
    double inv_h_tf;
    const double* C;
    __device__ __forceinline__ double at(int col) const { return im::at(v, (unsigned)col, ld8, lb); }
    __device__ __forceinline__ double operator()(int i) const {
        constexpr int NN = D + 1;
        constexpr int CO = 2 * K3_NX + K3_NU + K3_NZ;          // x, u, xdot, z of the interval
        if (n > 0) {
            const int xc = c0 + CO + (n - 1) * (K3_NX + K3_NZ);
            if (i < K3_NX) return at(xc + i);
            if (i < 2 * K3_NX) {                               // xdot from the collocation polynomial
                const int s = i - K3_NX;
                double acc = 0.0;
#pragma unroll
                for (int r = 0; r < NN; ++r)
                    acc += C[r * NN + n] * at(r == 0 ? c0 + s : c0 + CO + (r - 1) * (K3_NX + K3_NZ) + s);
                return acc * inv_h_tf;
            }
            if (i == 2 * K3_NX + K3_NU) return at(xc + K3_NX);
        } else {
            if (i < K3_NX) return at(c0 + i);
            if (i < 2 * K3_NX) return at(c0 + K3_NX + K3_NU + (i - K3_NX));
            if (i == 2 * K3_NX + K3_NU) return at(c0 + 2 * K3_NX + K3_NU);
        }
        if (i < 2 * K3_NX + K3_NU) return at(c0 + K3_NX + (i - 2 * K3_NX));   // u[k], zero-order hold
        if (i < K3_NW) return at(i - (2 * K3_NX + K3_NU + K3_NZ));             // theta: diam_t, t_f
        return at(K3_NTH + 0);                                                 // phi.gamma
    }
};

// tan[s] = v  ->  the J_g entries of slot s (dt: the node's destination row in LDS, byte offsets)
template <int D, int KIND>
struct GenJSink {
    double* jac;
    unsigned lb;
    const unsigned* dt;
    const double* xs;
    struct Ref {
        const GenJSink* s;
        int slot;
        __device__ __forceinline__ void operator=(double v) const { s->put(slot, v); }
    };
    __device__ __forceinline__ Ref operator[](int slot) const { return Ref{this, slot}; }
    __device__ __forceinline__ void put(int slot, double v) const {
        const int f = kGenSlots<D>.first[KIND][slot], c = kGenSlots<D>.cnt[KIND][slot];
        if (c == 1) {
            __builtin_nontemporal_store(v, &im::at_byte(jac, dt[f] + lb));
            return;
        }
#pragma unroll
        for (int q = 0; q < D; ++q) __builtin_nontemporal_store(xs[q] * v, &im::at_byte(jac, dt[f + q] + lb));
    }
};

// node inputs preloaded into registers: every load of the node issued at once (one memory latency)
// instead of at the generated code's first use of each input (one exposed latency per input)
template <int D>
struct GenInPre {
    double w[K3_NW + 1];
    __device__ __forceinline__ explicit GenInPre(const GenIn<D>& in) {
#pragma unroll
        for (int i = 0; i <= K3_NW; ++i) w[i] = in(i);
    }
    __device__ __forceinline__ double operator()(int i) const { return w[i]; }
};

#ifndef AWE_MPC_PRELOAD
#define AWE_MPC_PRELOAD 1
#endif
#ifndef AWE_MPC_STRIP_WAVES
#define AWE_MPC_STRIP_WAVES 1
#endif

// calls f(std::integral_constant<int, s>) for the direction strip s == sg of the generated code
template <int S, int I = 0, class F>
__device__ __forceinline__ void gen_strip(int sg, const F& f) {
    if constexpr (I < S) {
        if (sg == I) f(std::integral_constant<int, I>{});
        else gen_strip<S, I + 1>(sg, f);
    }
}

// Strip groups: with AWE_MPC_STRIP_WAVES the kNStrips direction strips of a node run in separate
// workgroups side by side (each recomputes the values it needs: more, shorter wavefronts -- at the
// config-5 batch of 256 instances one node per wavefront leaves most SIMDs idle and the kernel is the
// latency of one wavefront); otherwise one wavefront runs the strips of its node in turn.
constexpr int kGenStripGroups = AWE_MPC_STRIP_WAVES ? awe_k3gen::kNStrips : 1;
constexpr int kGenNodeWaves = 4;
constexpr int kGenShootWaves = kGenNodeWaves;
template <int D>
constexpr int gen_radau_waves() { return D < kGenNodeWaves ? D : kGenNodeWaves; }

template <int D>
__device__ __forceinline__ void gen_radau_tile(int t, unsigned* ldt, const double* __restrict__ VT,
                                               const double* __restrict__ PT, const double* __restrict__ cst,
                                               const unsigned* __restrict__ dtab, double* __restrict__ g,
                                               double* __restrict__ jac, const GenArgs& a) {
    constexpr int NN = D + 1;
    constexpr int W = gen_radau_waves<D>();
    constexpr int T1 = kGenSlots<D>.total[1];
    const int sg = t % kGenStripGroups, tk = t / kGenStripGroups;
    const int ib = tk / a.n_k, k = tk - ib * a.n_k;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int m = 1; m < NN; ++m)
        im::stage_offsets<64 * kGenNodeWaves>(ldt + (m - 1) * T1, dtab + (size_t)(k * NN + m) * a.dstride, T1,
                                              a.ldj8, tid);
    __syncthreads();
    const int b = ib * 64 + lane;
    if (wave >= W || b >= a.batch) return;
    const unsigned lb = 8u * (unsigned)b, ld8 = a.ld8;
    const int c0 = a.v_int0 + k * a.stride;
    const double* C = a.coll.C;
    const double tf = im::at(VT, 1u, ld8, lb);
    const double inv_h_tf = (double)a.n_k / tf;
    const double u_ref = im::at(PT, (unsigned)(K3_NX + a.n_v), ld8, lb);
    double* gb = g + (size_t)b * a.n_g + K3_NX + k * a.rows + K3_N_EQ + K3_N_INEQ;
    for (int n = 1 + wave; n < NN; n += W) {
        double xs[D];                                 // C[r][n] / (h t_f) of the columns X_r, r != n
#pragma unroll
        for (int q = 0; q < D; ++q) xs[q] = C[(q < n ? q : q + 1) * NN + n] * inv_h_tf;
        const GenIn<D> gin{VT, ld8, lb, c0, n, inv_h_tf, C};
#if AWE_MPC_PRELOAD
        const GenInPre<D> in(gin);
#else
        const GenIn<D>& in = gin;
#endif
        GenJSink<D, 1> js{jac, lb, ldt + (n - 1) * T1, xs};
        const double cxx = C[n * NN + n] * inv_h_tf, itf = 1.0 / tf;
        auto run = [&](auto st) {
            awe_k3gen::k3_node_radau<1, decltype(st)::value>(in, u_ref, cxx, itf, cst, gb + (n - 1) * K3_N_EQ, js);
        };
        if constexpr (kGenStripGroups > 1) {
            gen_strip<awe_k3gen::kNStrips>(sg, run);
        } else {
            gen_strip<awe_k3gen::kNStrips>(0, run);
            if constexpr (awe_k3gen::kNStrips > 1) gen_strip<awe_k3gen::kNStrips, 1>(1, run);
            if constexpr (awe_k3gen::kNStrips > 2) gen_strip<awe_k3gen::kNStrips, 2>(2, run);
            if constexpr (awe_k3gen::kNStrips > 3) gen_strip<awe_k3gen::kNStrips, 3>(3, run);
            static_assert(awe_k3gen::kNStrips <= 4, "strip loop");
        }
    }
}

#ifndef AWE_MPC_EXTRA_TILES
#define AWE_MPC_EXTRA_TILES 1
#endif
template <int D>
__device__ __forceinline__ void gen_interval_extras(int k, int b, const double* __restrict__ VT,
                                                    const double* __restrict__ PT, const unsigned* __restrict__ ctab,
                                                    const int* __restrict__ coff, double* __restrict__ g,
                                                    double* __restrict__ grad, double* __restrict__ jac,
                                                    double* __restrict__ fpart, const GenArgs& a);

// shooting nodes: one wavefront per interval (kGenShootWaves intervals of one instance block per
// workgroup); strip group 0 then writes the interval's tracking-cost gradient and partial sum,
// continuity rows, initial conditions and constant J_g entries
template <int D>
__device__ __forceinline__ void gen_shoot_tile(int t, unsigned* ldt, const double* __restrict__ VT,
                                               const double* __restrict__ PT, const double* __restrict__ cst,
                                               const unsigned* __restrict__ dtab, const unsigned* __restrict__ ctab,
                                               const int* __restrict__ coff, double* __restrict__ g,
                                               double* __restrict__ grad, double* __restrict__ jac,
                                               double* __restrict__ fpart, const GenArgs& a) {
    constexpr int NN = D + 1;
    constexpr int T0 = kGenSlots<D>.total[0];
    const int nk4 = (a.n_k + kGenShootWaves - 1) / kGenShootWaves;
    const int sg = t % kGenStripGroups, tk = t / kGenStripGroups;
    const int ib = tk / nk4, k0 = (tk - ib * nk4) * kGenShootWaves;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int w = 0; w < kGenShootWaves && k0 + w < a.n_k; ++w)
        im::stage_offsets<64 * kGenNodeWaves>(ldt + w * T0, dtab + (size_t)((k0 + w) * NN) * a.dstride, T0, a.ldj8,
                                              tid);
    __syncthreads();
    const int k = k0 + wave;
    const int b = ib * 64 + lane;
    if (k >= a.n_k || b >= a.batch) return;
    const unsigned lb = 8u * (unsigned)b, ld8 = a.ld8;
    const int c0 = a.v_int0 + k * a.stride;
    const double* C = a.coll.C;
    const double tf = im::at(VT, 1u, ld8, lb);
    const double inv_h_tf = (double)a.n_k / tf;
    const double u_ref = im::at(PT, (unsigned)(K3_NX + a.n_v), ld8, lb);
    double* gb = g + (size_t)b * a.n_g;
    const int row0 = K3_NX + k * a.rows;
    {
        const GenIn<D> gin{VT, ld8, lb, c0, 0, inv_h_tf, C};
#if AWE_MPC_PRELOAD
        const GenInPre<D> in(gin);
#else
        const GenIn<D>& in = gin;
#endif
        GenJSink<D, 0> js{jac, lb, ldt + wave * T0, nullptr};
        auto run = [&](auto st) { awe_k3gen::k3_node_shoot<1, decltype(st)::value>(in, u_ref, cst, gb + row0, js); };
        if constexpr (kGenStripGroups > 1) {
            gen_strip<awe_k3gen::kNStrips>(sg, run);
        } else {
            gen_strip<awe_k3gen::kNStrips>(0, run);
            if constexpr (awe_k3gen::kNStrips > 1) gen_strip<awe_k3gen::kNStrips, 1>(1, run);
            if constexpr (awe_k3gen::kNStrips > 2) gen_strip<awe_k3gen::kNStrips, 2>(2, run);
            if constexpr (awe_k3gen::kNStrips > 3) gen_strip<awe_k3gen::kNStrips, 3>(3, run);
        }
    }
    if (AWE_MPC_EXTRA_TILES || sg != 0) return;
    gen_interval_extras<D>(k, b, VT, PT, ctab, coff, g, grad, jac, fpart, a);
}

// the interval's tracking-cost gradient and partial sum, continuity rows, initial conditions and
// constant J_g entries (lane b = instance)
template <int D>
__device__ __forceinline__ void gen_interval_extras(int k, int b, const double* __restrict__ VT,
                                                    const double* __restrict__ PT, const unsigned* __restrict__ ctab,
                                                    const int* __restrict__ coff, double* __restrict__ g,
                                                    double* __restrict__ grad, double* __restrict__ jac,
                                                    double* __restrict__ fpart, const GenArgs& a) {
    constexpr int NN = D + 1;
    constexpr int STRIDE = K3_NX + K3_NU + K3_NX + K3_NZ + D * (K3_NX + K3_NZ);
    const unsigned lb = 8u * (unsigned)b, ld8 = a.ld8;
    const int c0 = a.v_int0 + k * a.stride;
    double* gb = g + (size_t)b * a.n_g;
    const int row0 = K3_NX + k * a.rows;
    auto V = [&](int col) { return im::at(VT, (unsigned)col, ld8, lb); };
    auto Pp = [&](int row) { return im::at(PT, (unsigned)row, ld8, lb); };
    // tracking objective of the interval's columns (pmpc.py:304-358), as mpc_interval_kernel
    const double* w = a.coll.w;
    const double invN = 1.0 / a.n_k;
    double sw = 0.0;
#pragma unroll
    for (int j = 0; j < D; ++j) sw += w[j];
    const int pref = K3_NX + c0;                       // p.ref row of column c0
    const int pq = K3_NX + a.n_v + 1;                  // Q, then R
    double fs = 0.0;
#pragma unroll
    for (int c = 0; c < STRIDE; ++c) {
        double gr = 0.0, ft = 0.0;
        if (c >= K3_NX && c < K3_NX + K3_NU) {
            const int i = c - K3_NX;
            const double e = V(c0 + c) - Pp(pref + c), W = Pp(pq + K3_NX + i);
            gr = 2.0 * sw * W * e * invN;
            ft = sw * W * e * e;
        } else if (c >= 2 * K3_NX + K3_NU + K3_NZ) {
            const int q = c - (2 * K3_NX + K3_NU + K3_NZ);
            const int j = q / (K3_NX + K3_NZ), e_ = q % (K3_NX + K3_NZ);
            const double e = V(c0 + c) - Pp(pref + c), W = e_ < K3_NX ? Pp(pq + e_) : 1.0;
            gr = 2.0 * w[j] * W * e * invN;
            ft = w[j] * W * e * e;
        }
        __builtin_nontemporal_store(gr, &im::at(grad, (unsigned)(c0 + c), a.ldj8, lb));
        fs += ft;
    }
    im::at(fpart, (unsigned)k, ld8, lb) = fs * invN;
    // continuity x[k+1] - sum_r D_r X_{k,r} (collocation.py:319-336) and the initial conditions
    const int gc = row0 + K3_N_EQ + K3_N_INEQ + D * K3_N_EQ;
    constexpr int CO = 2 * K3_NX + K3_NU + K3_NZ;
#pragma unroll
    for (int i = 0; i < K3_NX; ++i) {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < NN; ++r) s += a.coll.D[r] * V(r == 0 ? c0 + i : c0 + CO + (r - 1) * (K3_NX + K3_NZ) + i);
        gb[gc + i] = V(c0 + a.stride + i) - s;
    }
    if (k == 0)
        for (int i = 0; i < K3_NX; ++i) gb[i] = V(c0 + i) - Pp(i);
    // the interval's constant J_g entries (initial-condition and continuity rows)
    for (int q = coff[k]; q < coff[k + 1]; ++q) {
        const unsigned e = ctab[q];
        __builtin_nontemporal_store(a.kconst[e >> 24], &im::at(jac, e & 0xffffffu, a.ldj8, lb));
    }
}

// The node kernel: the Radau tiles (instance block, interval, strip group) and the shooting tiles
// (instance block, kGenShootWaves intervals, strip group) in one launch, so that the two node kinds
// run side by side; one wavefront per SIMD (the node code keeps 100-150 values live)
template <int D>
constexpr int gen_radau_tiles(const GenArgs& a) { return a.nib * a.n_k * kGenStripGroups; }
template <int D>
__global__ __launch_bounds__(64 * kGenNodeWaves) __attribute__((amdgpu_waves_per_eu(1)))
void mpc_gen_node_kernel(const double* __restrict__ VT, const double* __restrict__ PT,
                         const double* __restrict__ cst, const unsigned* __restrict__ dtab,
                         const unsigned* __restrict__ ctab, const int* __restrict__ coff, double* __restrict__ g,
                         double* __restrict__ grad, double* __restrict__ jac, double* __restrict__ fpart, GenArgs a) {
    constexpr int T0 = kGenSlots<D>.total[0], T1 = kGenSlots<D>.total[1];
    constexpr int NLDT = D * T1 > kGenShootWaves * T0 ? D * T1 : kGenShootWaves * T0;
    __shared__ unsigned ldt[NLDT];
    const int nr = gen_radau_tiles<D>(a);
    const int nk4 = (a.n_k + kGenShootWaves - 1) / kGenShootWaves;
    const int ns = a.nib * nk4 * kGenStripGroups;
    const int ne = AWE_MPC_EXTRA_TILES ? a.nib * nk4 : 0;
    const int t = im::xcd_tile(ne + nr + ns);
    if (t >= ne + nr + ns) return;
    if (t < ne) {                        // first: the extras tiles are short and latency-bound
        const int ib = t / nk4, k = (t - ib * nk4) * kGenShootWaves + (int)(threadIdx.x >> 6);
        const int b = ib * 64 + (int)(threadIdx.x & 63);
        if (k < a.n_k && b < a.batch) gen_interval_extras<D>(k, b, VT, PT, ctab, coff, g, grad, jac, fpart, a);
    } else if (t < ne + nr) {
        gen_radau_tile<D>(t - ne, ldt, VT, PT, cst, dtab, g, jac, a);
    } else {
        gen_shoot_tile<D>(t - ne - nr, ldt, VT, PT, cst, dtab, ctab, coff, g, grad, jac, fpart, a);
    }
}

// one lane per instance: objective partials in a fixed order, terminal cost, global gradient rows
__global__ __launch_bounds__(64) void mpc_gen_finalize_kernel(const double* __restrict__ VT,
                                                             const double* __restrict__ PT,
                                                             const double* __restrict__ fpart, double* __restrict__ f,
                                                             double* __restrict__ grad, GenArgs a) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= a.batch) return;
    const unsigned lb = 8u * (unsigned)b;
    double s = 0.0;
    int k = 0;
    for (; k + 8 <= a.n_k; k += 8) {                   // 8 loads in flight, the sum in interval order
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = im::at(fpart, (unsigned)(k + u), a.ld8, lb);
#pragma unroll
        for (int u = 0; u < 8; ++u) s += t[u];
    }
    for (; k < a.n_k; ++k) s += im::at(fpart, (unsigned)k, a.ld8, lb);
    const int xN = a.v_int0 + a.n_k * a.stride;
    const int pP = K3_NX + a.n_v + 1 + K3_NX + K3_NU;
    for (int i = 0; i < K3_NX; ++i) {
        const double e = im::at(VT, (unsigned)(xN + i), a.ld8, lb) - im::at(PT, (unsigned)(K3_NX + xN + i), a.ld8, lb);
        const double W = im::at(PT, (unsigned)(pP + i), a.ld8, lb);
        im::at(grad, (unsigned)(xN + i), a.ldj8, lb) = 2.0 * W * e;
        s += W * e * e;
    }
    for (int i = 0; i < a.v_int0; ++i) im::at(grad, (unsigned)i, a.ldj8, lb) = 0.0;   // theta, phi, xi
    f[b] = s;
}

}  // namespace

struct awempc_handle_s {
    Tables t;
    int batch = 0;
    std::vector<double> consts;
    double* d_cst = nullptr;
    awt::DevColl* d_coll = nullptr;
    int* d_goff = nullptr;
    int* d_gslot = nullptr;
    uint32_t* d_gcode = nullptr;
    double* d_fpart = nullptr;
    double *d_V = nullptr, *d_P = nullptr, *d_f = nullptr, *d_g = nullptr, *d_grad = nullptr, *d_jac = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    bool timed = false;
    // Hessian (built on first use: awempc_hess_init)
    HessTables ht;
    bool hess_ready = false;
    int hd_total = 0;
    int *d_task = nullptr, *d_slot0 = nullptr, *d_nslot = nullptr, *d_ent_off = nullptr, *d_term_off = nullptr;
    int *d_hgslot = nullptr, *d_xnslot = nullptr;
    unsigned* d_terms = nullptr;
    double* d_gpart = nullptr;
    double *d_hsig = nullptr, *d_hlam = nullptr, *d_H = nullptr;
    hipEvent_t hev[2] = {nullptr, nullptr};
    bool htimed = false;
    // generated instance-minor path (awempc_eval_nlp_im)
    bool gen_ok = false;
    std::string gen_why;
    int gen_dstride = 0;
    size_t gen_ld = 0;                       // row length of VT / PT / fpart
    unsigned *d_gdtab = nullptr, *d_gctab = nullptr;
    int* d_gcoff = nullptr;
    double *d_VT = nullptr, *d_PT = nullptr, *d_gfpart = nullptr;
    double gen_kconst[8] = {};
    hipEvent_t gev[4] = {nullptr, nullptr, nullptr, nullptr};
    bool gtimed = false;
};

namespace {

// destination tables of the generated path from the gather list of build_tables: per (interval k,
// node n) a row of CCS positions in kGenSlots order (slot s of the node's generated code, then its
// d polynomial columns for a Radau xdot direction), and per interval the constant entries
// (position | value index << 24, values 1, -D[r])
int build_gen(awempc_handle_s* h) {
    const Tables& T = h->t;
    const int n_k = T.lay.n_k, d = T.lay.d, NN = d + 1;
    if ((int)h->consts[K3_C_N_ELEMENTS] != awe_k3gen::kNElements) {
        h->gen_why = "the generated node code has " + std::to_string(awe_k3gen::kNElements) +
                     " tether elements, the constants " + std::to_string((int)h->consts[K3_C_N_ELEMENTS]);
        return AWE_OK;
    }
    if ((size_t)T.row.size() >= (1u << 24)) { h->gen_why = "J_g too large for the constant table"; return AWE_OK; }
    const GenSlotTab st(d);
    const int dstride = std::max(st.total[0], st.total[1]);
    std::vector<unsigned> dtab((size_t)n_k * NN * dstride, 0xffffffffu);
    std::vector<unsigned> ctab;
    std::vector<int> coff(n_k + 1, 0);
    for (int k = 0; k < n_k; ++k) {
        for (int e = T.goff[k]; e < T.goff[k + 1]; ++e) {
            const unsigned pos = (unsigned)T.gslot[e];
            const uint32_t cd = T.gcode[e];
            const uint32_t kind = cd >> 29;
            const int rr = (cd >> 25) & 15, idx = (int)(cd & ((1u << 21) - 1u));
            if (kind == kKindOne || kind == kKindMinusD) {
                ctab.push_back(pos | ((kind == kKindOne ? 0u : 1u + (unsigned)rr) << 24));
                continue;
            }
            const int n = idx / (kRowsPerNode * kLanes), r = (idx / kLanes) % kRowsPerNode, l = idx % kLanes;
            const int kd = n > 0 ? 1 : 0;
            const int s = awe_k3gen::kTanIdx[kd][r][l];
            if (s < 0) return fail(AWE_ERR_ARG, "internal: J_g entry without a generated tangent");
            int q = 0;
            if (kind == kKindTangPoly) q = rr < n ? rr : rr - 1;
            if (q >= st.cnt[kd][s]) return fail(AWE_ERR_ARG, "internal: destination count of a generated tangent");
            unsigned& slot = dtab[(size_t)(k * NN + n) * dstride + st.first[kd][s] + q];
            if (slot != 0xffffffffu) return fail(AWE_ERR_ARG, "internal: two J_g entries for one generated destination");
            slot = pos;
        }
        coff[k + 1] = (int)ctab.size();
        for (int n = 0; n < NN; ++n)
            for (int i = 0; i < st.total[n > 0 ? 1 : 0]; ++i)
                if (dtab[(size_t)(k * NN + n) * dstride + i] == 0xffffffffu)
                    return fail(AWE_ERR_ARG, "internal: generated destination without a J_g entry");
    }
    if (ctab.empty()) ctab.push_back(0);
    for (auto& x : dtab) if (x == 0xffffffffu) x = 0;   // padding of the shorter node kind
    h->gen_kconst[0] = 1.0;
    for (int r = 0; r < NN; ++r) h->gen_kconst[1 + r] = -h->t.coll.D[r];
    h->gen_dstride = dstride;
    h->gen_ld = (size_t)h->batch;
    MPC_TRY(hipMalloc((void**)&h->d_gdtab, sizeof(unsigned) * dtab.size()));
    MPC_TRY(hipMemcpy(h->d_gdtab, dtab.data(), sizeof(unsigned) * dtab.size(), hipMemcpyHostToDevice));
    MPC_TRY(hipMalloc((void**)&h->d_gctab, sizeof(unsigned) * ctab.size()));
    MPC_TRY(hipMemcpy(h->d_gctab, ctab.data(), sizeof(unsigned) * ctab.size(), hipMemcpyHostToDevice));
    MPC_TRY(hipMalloc((void**)&h->d_gcoff, sizeof(int) * coff.size()));
    MPC_TRY(hipMemcpy(h->d_gcoff, coff.data(), sizeof(int) * coff.size(), hipMemcpyHostToDevice));
    MPC_TRY(hipMalloc((void**)&h->d_VT, sizeof(double) * h->gen_ld * T.lay.n_v));
    MPC_TRY(hipMalloc((void**)&h->d_PT, sizeof(double) * h->gen_ld * T.lay.n_p));
    MPC_TRY(hipMalloc((void**)&h->d_gfpart, sizeof(double) * h->gen_ld * n_k));
    for (auto& e : h->gev) MPC_TRY(hipEventCreate(&e));
    h->gen_ok = true;
    return AWE_OK;
}

}  // namespace

extern "C" {

const char* awempc_last_error(void) { return g_err.c_str(); }

int awempc_sparsity_jac_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind, int* row) {
    if (!consts || !nnz) return fail(AWE_ERR_ARG, "null argument");
    Tables T;
    std::string err;
    if (build_tables(n_k, d, consts, n_consts, T, err)) return fail(AWE_ERR_ARG, err);
    *nnz = (int)T.row.size();
    if (colind) std::memcpy(colind, T.colind.data(), sizeof(int) * T.colind.size());
    if (row) std::memcpy(row, T.row.data(), sizeof(int) * T.row.size());
    return AWE_OK;
}

int awempc_create(int n_k, int d, const double* consts, int n_consts, int batch, awempc_handle* out) {
    if (!consts || !out || batch < 1) return fail(AWE_ERR_ARG, "bad argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(AWE_ERR_NODEVICE, "no HIP device");
    if (d < 2 || d > 5) return fail(AWE_ERR_ARG, "the MPC kernel is instantiated for 2 <= d <= 5");
    auto* h = new awempc_handle_s();
    std::string err;
    if (build_tables(n_k, d, consts, n_consts, h->t, err)) {
        delete h;
        return fail(AWE_ERR_ARG, err);
    }
    if (consts[K3_C_N_K] != (double)n_k || consts[K3_C_D] != (double)d) {
        delete h;
        return fail(AWE_ERR_ARG, "consts[K3_C_N_K], consts[K3_C_D] disagree with n_k, d");
    }
    h->batch = batch;
    h->consts.assign(consts, consts + n_consts);
    awt::DevColl dc{};
    const int NN = d + 1;
    for (int j = 0; j < NN; ++j) {
        for (int r = 0; r < NN; ++r) dc.C[j * NN + r] = h->t.coll.C[j][r];
        dc.D[j] = h->t.coll.D[j];
    }
    for (int j = 0; j < d; ++j) dc.w[j] = h->t.coll.w[j];
    const Tables& T = h->t;
#define MPC_UPLOAD(dst, src, n)                                                         \
    MPC_TRY(hipMalloc((void**)&dst, sizeof(*dst) * (n)));                              \
    MPC_TRY(hipMemcpy(dst, src, sizeof(*dst) * (n), hipMemcpyHostToDevice));
    MPC_UPLOAD(h->d_cst, consts, n_consts);
    MPC_UPLOAD(h->d_coll, &dc, 1);
    MPC_UPLOAD(h->d_goff, T.goff.data(), T.goff.size());
    MPC_UPLOAD(h->d_gslot, T.gslot.data(), T.gslot.size());
    MPC_UPLOAD(h->d_gcode, T.gcode.data(), T.gcode.size());
#undef MPC_UPLOAD
    MPC_TRY(hipMalloc((void**)&h->d_fpart, sizeof(double) * (size_t)batch * n_k));
    for (auto& e : h->ev) MPC_TRY(hipEventCreate(&e));
    if (int rc = build_gen(h)) {
        awempc_destroy(h);
        return rc;
    }
    *out = h;
    return AWE_OK;
}

int awempc_destroy(awempc_handle h) {
    if (!h) return AWE_OK;
    void* bufs[] = {h->d_cst, h->d_coll, h->d_goff, h->d_gslot, h->d_gcode, h->d_fpart,
                    h->d_V, h->d_P, h->d_f, h->d_g, h->d_grad, h->d_jac,
                    h->d_task, h->d_slot0, h->d_nslot, h->d_ent_off, h->d_term_off, h->d_hgslot, h->d_xnslot,
                    h->d_terms, h->d_gpart, h->d_hsig, h->d_hlam, h->d_H,
                    h->d_gdtab, h->d_gctab, h->d_gcoff, h->d_VT, h->d_PT, h->d_gfpart};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : h->hev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : h->gev)
        if (e) (void)hipEventDestroy(e);
    delete h;
    return AWE_OK;
}

int awempc_sizes(awempc_handle h, int* n_v, int* n_g, int* n_p, int* nnz) {
    if (!h) return fail(AWE_ERR_ARG, "null handle");
    if (n_v) *n_v = h->t.lay.n_v;
    if (n_g) *n_g = h->t.lay.n_g;
    if (n_p) *n_p = h->t.lay.n_p;
    if (nnz) *nnz = (int)h->t.row.size();
    return AWE_OK;
}

int awempc_sparsity_jac(awempc_handle h, int* colind, int* row) {
    if (!h || !colind || !row) return fail(AWE_ERR_ARG, "null argument");
    std::memcpy(colind, h->t.colind.data(), sizeof(int) * h->t.colind.size());
    std::memcpy(row, h->t.row.data(), sizeof(int) * h->t.row.size());
    return AWE_OK;
}

int awempc_eval_nlp(awempc_handle h, const double* V, const double* p, double* f, double* g, double* grad_f,
                    double* jac, void* stream) {
    if (!h || !V || !p || !f || !g || !grad_f || !jac) return fail(AWE_ERR_ARG, "null argument");
    const Tables& T = h->t;
    hipStream_t s = (hipStream_t)stream;
    MArgs a{T.lay.n_k, T.lay.d, T.lay.n_v, T.lay.n_g, T.lay.n_p, (int)T.row.size(), T.lay.stride,
            V, p, f, g, grad_f, jac, h->d_cst, h->d_coll, h->d_goff, h->d_gslot, h->d_gcode, h->d_fpart};
    const dim3 grid((unsigned)(h->batch * T.lay.n_k));
    MPC_TRY(hipEventRecord(h->ev[0], s));
    switch (T.lay.d) {
        case 2: mpc_interval_kernel<2><<<grid, 64 * waves_for<2>(), 0, s>>>(a); break;
        case 3: mpc_interval_kernel<3><<<grid, 64 * waves_for<3>(), 0, s>>>(a); break;
        case 4: mpc_interval_kernel<4><<<grid, 64 * waves_for<4>(), 0, s>>>(a); break;
        case 5: mpc_interval_kernel<5><<<grid, 64 * waves_for<5>(), 0, s>>>(a); break;
        default: return fail(AWE_ERR_ARG, "unsupported d");
    }
    MPC_TRY(hipGetLastError());
    MPC_TRY(hipEventRecord(h->ev[1], s));
    mpc_finalize_kernel<<<dim3((unsigned)h->batch), 64, 0, s>>>(a);
    MPC_TRY(hipGetLastError());
    MPC_TRY(hipEventRecord(h->ev[2], s));
    h->timed = true;
    return AWE_OK;
}

int awempc_gen_status(awempc_handle h, int* available) {
    if (!h || !available) return fail(AWE_ERR_ARG, "null argument");
    *available = h->gen_ok ? 1 : 0;
    if (!h->gen_ok) g_err = h->gen_why;
    return AWE_OK;
}

int awempc_eval_nlp_im(awempc_handle h, const double* V, const double* p, double* f, double* g, double* grad_f,
                       double* jac, size_t ld, void* stream) {
    if (!h || !V || !p || !f || !g || !grad_f || !jac) return fail(AWE_ERR_ARG, "null argument");
    if (!h->gen_ok) return fail(AWE_ERR_ARG, "generated path unavailable: " + h->gen_why);
    const Tables& T = h->t;
    const int B = h->batch;
    if (ld < (size_t)B) return fail(AWE_ERR_ARG, "ld must be >= batch");
    const size_t nrows = std::max((size_t)T.row.size(), (size_t)T.lay.n_v);
    if (nrows * ld * 8 >= ((size_t)1 << 32)) return fail(AWE_ERR_ARG, "instance-minor J_g must stay below 4 GiB");
    if ((size_t)std::max(T.lay.n_v, T.lay.n_p) * h->gen_ld * 8 >= ((size_t)1 << 32))
        return fail(AWE_ERR_ARG, "instance-minor inputs must stay below 4 GiB");
    hipStream_t s = (hipStream_t)stream;
    GenArgs a{};
    const int NN = T.lay.d + 1;
    for (int j = 0; j < NN; ++j) {
        for (int r = 0; r < NN; ++r) a.coll.C[j * NN + r] = T.coll.C[j][r];
        a.coll.D[j] = T.coll.D[j];
    }
    for (int j = 0; j < T.lay.d; ++j) a.coll.w[j] = T.coll.w[j];
    a.n_k = T.lay.n_k;
    a.batch = B;
    a.n_v = T.lay.n_v;
    a.n_g = T.lay.n_g;
    a.n_p = T.lay.n_p;
    a.stride = T.lay.stride;
    a.v_int0 = T.lay.v_int0;
    a.rows = T.lay.rows;
    a.nib = (B + 63) / 64;
    a.dstride = h->gen_dstride;
    a.ld8 = (unsigned)(8 * h->gen_ld);
    a.ldj8 = (unsigned)(8 * ld);
    for (int i = 0; i < 8; ++i) a.kconst[i] = h->gen_kconst[i];
    MPC_TRY(hipEventRecord(h->gev[0], s));
    const dim3 tgrid((unsigned)((T.lay.n_v + T.lay.n_p + 63) / 64), (unsigned)a.nib);
    im::transpose_in_kernel<<<tgrid, 256, 0, s>>>(V, p, h->d_VT, h->d_PT, B, T.lay.n_v, T.lay.n_p, (int)h->gen_ld);
    MPC_TRY(hipGetLastError());
    MPC_TRY(hipEventRecord(h->gev[1], s));
    const int n_tiles = a.nib * (a.n_k + (a.n_k + kGenShootWaves - 1) / kGenShootWaves) * kGenStripGroups +
                        (AWE_MPC_EXTRA_TILES ? a.nib * ((a.n_k + kGenShootWaves - 1) / kGenShootWaves) : 0);
    const dim3 ngrid((unsigned)im::xcd_grid(n_tiles));
#define MPC_GEN_NODE(DD)                                                                                           \
    mpc_gen_node_kernel<DD><<<ngrid, 64 * kGenNodeWaves, 0, s>>>(h->d_VT, h->d_PT, h->d_cst, h->d_gdtab, h->d_gctab, \
                                                                 h->d_gcoff, g, grad_f, jac, h->d_gfpart, a)
    switch (T.lay.d) {
        case 2: MPC_GEN_NODE(2); break;
        case 3: MPC_GEN_NODE(3); break;
        case 4: MPC_GEN_NODE(4); break;
        case 5: MPC_GEN_NODE(5); break;
        default: return fail(AWE_ERR_ARG, "unsupported d");
    }
#undef MPC_GEN_NODE
    MPC_TRY(hipGetLastError());
    MPC_TRY(hipEventRecord(h->gev[2], s));
    mpc_gen_finalize_kernel<<<dim3((unsigned)a.nib), 64, 0, s>>>(h->d_VT, h->d_PT, h->d_gfpart, f, grad_f, a);
    MPC_TRY(hipGetLastError());
    MPC_TRY(hipEventRecord(h->gev[3], s));
    h->gtimed = true;
    return AWE_OK;
}

int awempc_last_kernel_ms_im(awempc_handle h, float* ms_in, float* ms_node, float* ms_fin) {
    if (!h || !h->gtimed) return fail(AWE_ERR_ARG, "no timed instance-minor evaluation yet");
    MPC_TRY(hipEventSynchronize(h->gev[3]));
    if (ms_in) MPC_TRY(hipEventElapsedTime(ms_in, h->gev[0], h->gev[1]));
    if (ms_node) MPC_TRY(hipEventElapsedTime(ms_node, h->gev[1], h->gev[2]));
    if (ms_fin) MPC_TRY(hipEventElapsedTime(ms_fin, h->gev[2], h->gev[3]));
    return AWE_OK;
}

int awempc_last_kernel_ms(awempc_handle h, float* ms_main, float* ms_fin) {
    if (!h || !h->timed) return fail(AWE_ERR_ARG, "no timed evaluation yet");
    MPC_TRY(hipEventSynchronize(h->ev[2]));
    if (ms_main) MPC_TRY(hipEventElapsedTime(ms_main, h->ev[0], h->ev[1]));
    if (ms_fin) MPC_TRY(hipEventElapsedTime(ms_fin, h->ev[1], h->ev[2]));
    return AWE_OK;
}

int awempc_eval_nlp_host(awempc_handle h, const double* V, const double* p, double* f, double* g, double* grad_f,
                         double* jac) {
    if (!h || !V || !p || !f || !g || !grad_f || !jac) return fail(AWE_ERR_ARG, "null argument");
    const Tables& T = h->t;
    const size_t nb = (size_t)h->batch, nnz = T.row.size();
    if (!h->d_V) {
        MPC_TRY(hipMalloc((void**)&h->d_V, sizeof(double) * nb * T.lay.n_v));
        MPC_TRY(hipMalloc((void**)&h->d_P, sizeof(double) * nb * T.lay.n_p));
        MPC_TRY(hipMalloc((void**)&h->d_f, sizeof(double) * nb));
        MPC_TRY(hipMalloc((void**)&h->d_g, sizeof(double) * nb * T.lay.n_g));
        MPC_TRY(hipMalloc((void**)&h->d_grad, sizeof(double) * nb * T.lay.n_v));
        MPC_TRY(hipMalloc((void**)&h->d_jac, sizeof(double) * nb * nnz));
    }
    MPC_TRY(hipMemcpy(h->d_V, V, sizeof(double) * nb * T.lay.n_v, hipMemcpyHostToDevice));
    MPC_TRY(hipMemcpy(h->d_P, p, sizeof(double) * nb * T.lay.n_p, hipMemcpyHostToDevice));
    int rc = awempc_eval_nlp(h, h->d_V, h->d_P, h->d_f, h->d_g, h->d_grad, h->d_jac, nullptr);
    if (rc) return rc;
    MPC_TRY(hipDeviceSynchronize());
    MPC_TRY(hipMemcpy(f, h->d_f, sizeof(double) * nb, hipMemcpyDeviceToHost));
    MPC_TRY(hipMemcpy(g, h->d_g, sizeof(double) * nb * T.lay.n_g, hipMemcpyDeviceToHost));
    MPC_TRY(hipMemcpy(grad_f, h->d_grad, sizeof(double) * nb * T.lay.n_v, hipMemcpyDeviceToHost));
    MPC_TRY(hipMemcpy(jac, h->d_jac, sizeof(double) * nb * nnz, hipMemcpyDeviceToHost));
    auto finite = [](const double* x, size_t n) {
        for (size_t i = 0; i < n; ++i)
            if (!std::isfinite(x[i])) return false;
        return true;
    };
    if (!finite(f, nb) || !finite(g, nb * T.lay.n_g) || !finite(grad_f, nb * T.lay.n_v) || !finite(jac, nb * nnz))
        return fail(AWE_ERR_NONFINITE, "non-finite output");
    return AWE_OK;
}

// ---- nlp_hess_l ------------------------------------------------------------------------------
int awempc_sparsity_hess_static(int n_k, int d, const double* consts, int n_consts, int* nnz, int* colind, int* row) {
    if (!consts || !nnz) return fail(AWE_ERR_ARG, "null argument");
    Tables T;
    HessTables H;
    std::string err;
    if (build_tables(n_k, d, consts, n_consts, T, err) || build_hess_tables(T, consts, H, err))
        return fail(AWE_ERR_ARG, err);
    *nnz = H.nnz;
    if (colind) std::memcpy(colind, H.colind.data(), sizeof(int) * H.colind.size());
    if (row) std::memcpy(row, H.row.data(), sizeof(int) * H.row.size());
    return AWE_OK;
}

int awempc_hess_init(awempc_handle h, int* nnz) {
    if (!h) return fail(AWE_ERR_ARG, "null handle");
    if (!h->hess_ready) {
        std::string err;
        if (build_hess_tables(h->t, h->consts.data(), h->ht, err)) return fail(AWE_ERR_ARG, err);
        const HessTables& H = h->ht;
        h->hd_total = H.ntask[0] + h->t.lay.d * H.ntask[1];
        if ((size_t)h->hd_total * sizeof(double) > 60 * 1024) return fail(AWE_ERR_ARG, "Hessian tasks exceed the LDS budget");
        if ((int)H.gslot.size() > 64) return fail(AWE_ERR_ARG, "too many global Hessian entries");
#define MPC_UPLOAD(dst, vec)                                                               \
        MPC_TRY(hipMalloc((void**)&dst, sizeof(*dst) * (vec).size()));                      \
        MPC_TRY(hipMemcpy(dst, (vec).data(), sizeof(*dst) * (vec).size(), hipMemcpyHostToDevice));
        MPC_UPLOAD(h->d_task, H.task);
        MPC_UPLOAD(h->d_slot0, H.slot0);
        MPC_UPLOAD(h->d_nslot, H.nslot);
        MPC_UPLOAD(h->d_ent_off, H.ent_off);
        MPC_UPLOAD(h->d_term_off, H.term_off);
        MPC_UPLOAD(h->d_terms, H.terms);
        MPC_UPLOAD(h->d_hgslot, H.gslot);
        MPC_UPLOAD(h->d_xnslot, H.xnslot);
#undef MPC_UPLOAD
        MPC_TRY(hipMalloc((void**)&h->d_gpart, sizeof(double) * (size_t)h->batch * h->t.lay.n_k * std::max<size_t>(1, H.gslot.size())));
        for (auto& e : h->hev) MPC_TRY(hipEventCreate(&e));
        h->hess_ready = true;
    }
    if (nnz) *nnz = h->ht.nnz;
    return AWE_OK;
}

int awempc_sparsity_hess(awempc_handle h, int* colind, int* row) {
    if (!h || !colind || !row) return fail(AWE_ERR_ARG, "null argument");
    int rc = awempc_hess_init(h, nullptr);
    if (rc) return rc;
    std::memcpy(colind, h->ht.colind.data(), sizeof(int) * h->ht.colind.size());
    std::memcpy(row, h->ht.row.data(), sizeof(int) * h->ht.row.size());
    return AWE_OK;
}

int awempc_eval_hess(awempc_handle h, const double* V, const double* p, const double* sigma, const double* lam_g,
                     double* H, void* stream) {
    if (!h || !V || !p || !sigma || !lam_g || !H) return fail(AWE_ERR_ARG, "null argument");
    int rc = awempc_hess_init(h, nullptr);
    if (rc) return rc;
    const Tables& T = h->t;
    const HessTables& HT = h->ht;
    hipStream_t s = (hipStream_t)stream;
    MArgs a{T.lay.n_k, T.lay.d, T.lay.n_v, T.lay.n_g, T.lay.n_p, (int)T.row.size(), T.lay.stride,
            V, p, nullptr, nullptr, nullptr, nullptr, h->d_cst, h->d_coll, h->d_goff, h->d_gslot, h->d_gcode, h->d_fpart};
    HArgs ha{a, sigma, lam_g, H, h->d_gpart, h->d_task, HT.ntask[0], HT.ntask[1], HT.npair1, HT.nnz,
             (int)HT.gslot.size(), h->hd_total, h->d_slot0, h->d_nslot, h->d_ent_off, h->d_term_off, h->d_terms,
             h->d_hgslot, h->d_xnslot};
    const dim3 grid((unsigned)(h->batch * T.lay.n_k));
    const size_t lds = sizeof(double) * (size_t)h->hd_total;
    MPC_TRY(hipEventRecord(h->hev[0], s));
    switch (T.lay.d) {
        case 2: mpc_hess_kernel<2><<<grid, kHessThreads, lds, s>>>(ha); break;
        case 3: mpc_hess_kernel<3><<<grid, kHessThreads, lds, s>>>(ha); break;
        case 4: mpc_hess_kernel<4><<<grid, kHessThreads, lds, s>>>(ha); break;
        case 5: mpc_hess_kernel<5><<<grid, kHessThreads, lds, s>>>(ha); break;
        default: return fail(AWE_ERR_ARG, "unsupported d");
    }
    MPC_TRY(hipGetLastError());
    mpc_hess_finalize_kernel<<<dim3((unsigned)h->batch), 64, 0, s>>>(ha);
    MPC_TRY(hipGetLastError());
    MPC_TRY(hipEventRecord(h->hev[1], s));
    h->htimed = true;
    return AWE_OK;
}

int awempc_last_hess_ms(awempc_handle h, float* ms) {
    if (!h || !h->htimed) return fail(AWE_ERR_ARG, "no timed Hessian evaluation yet");
    MPC_TRY(hipEventSynchronize(h->hev[1]));
    if (ms) MPC_TRY(hipEventElapsedTime(ms, h->hev[0], h->hev[1]));
    return AWE_OK;
}

int awempc_eval_hess_host(awempc_handle h, const double* V, const double* p, const double* sigma, const double* lam_g,
                          double* H) {
    if (!h || !V || !p || !sigma || !lam_g || !H) return fail(AWE_ERR_ARG, "null argument");
    int rc = awempc_hess_init(h, nullptr);
    if (rc) return rc;
    const Tables& T = h->t;
    const size_t nb = (size_t)h->batch, hnnz = h->ht.nnz;
    if (!h->d_V) {
        MPC_TRY(hipMalloc((void**)&h->d_V, sizeof(double) * nb * T.lay.n_v));
        MPC_TRY(hipMalloc((void**)&h->d_P, sizeof(double) * nb * T.lay.n_p));
    }
    if (!h->d_H) {
        MPC_TRY(hipMalloc((void**)&h->d_hsig, sizeof(double) * nb));
        MPC_TRY(hipMalloc((void**)&h->d_hlam, sizeof(double) * nb * T.lay.n_g));
        MPC_TRY(hipMalloc((void**)&h->d_H, sizeof(double) * nb * hnnz));
    }
    MPC_TRY(hipMemcpy(h->d_V, V, sizeof(double) * nb * T.lay.n_v, hipMemcpyHostToDevice));
    MPC_TRY(hipMemcpy(h->d_P, p, sizeof(double) * nb * T.lay.n_p, hipMemcpyHostToDevice));
    MPC_TRY(hipMemcpy(h->d_hsig, sigma, sizeof(double) * nb, hipMemcpyHostToDevice));
    MPC_TRY(hipMemcpy(h->d_hlam, lam_g, sizeof(double) * nb * T.lay.n_g, hipMemcpyHostToDevice));
    rc = awempc_eval_hess(h, h->d_V, h->d_P, h->d_hsig, h->d_hlam, h->d_H, nullptr);
    if (rc) return rc;
    MPC_TRY(hipDeviceSynchronize());
    MPC_TRY(hipMemcpy(H, h->d_H, sizeof(double) * nb * hnnz, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < nb * hnnz; ++i)
        if (!std::isfinite(H[i])) return fail(AWE_ERR_NONFINITE, "non-finite Hessian");
    return AWE_OK;
}

}  // extern "C"
