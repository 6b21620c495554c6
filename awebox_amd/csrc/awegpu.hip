// awegpu -- MI355X (gfx950) evaluator for the awebox AP2 direct-collocation NLP.
//
// Replaces, for the AP2 configuration, the CasADi-expanded SX evaluation that IPOPT calls
// through nlpsol (awebox/opti/preparation.py:366-400): f, g, grad f and the CCS values of J_g.
//
// Execution model:
//   * one 64-lane wavefront (one workgroup) per shooting interval k of one NLP instance b;
//   * the interval's slice of V is staged in LDS with coalesced loads;
//   * the wave walks the interval's d+1 nodes (shooting node + d Radau nodes); at each node every
//     lane evaluates the hand-written model in forward-mode dual arithmetic along its own
//     direction, so the 64 lanes together produce the node's Jacobian block in one pass;
//   * directions are chosen in V-space where that is free: at a collocation node the lane of
//     state i seeds x_i AND the matching polynomial derivative xdot_i = C[jj,jj]/(h tf), and one
//     lane seeds the full d/d t_f (t_f and every xdot_i = -xdot_i/t_f), so the chain rule through
//     the collocation polynomial (collocation.py:202-258) costs no extra pass;
//   * J values are written straight into their fixed CCS slots (positions derived on the host
//     from a structural-dependency instantiation of the same model), g rows and the interval's
//     grad f entries are written directly, and the few global gradient entries are reduced
//     deterministically by a small finalize kernel (no float atomics).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/awegpu.h"
#include "ap2_model.hpp"

namespace {

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

constexpr int kMaxD = 9;
constexpr int kLanes = 64;
constexpr int kTargets = 4;     // max V columns one lane direction feeds at one node
constexpr int kLaneGamma = 59;  // direction d/d phi.gamma
constexpr int kLanePsi = 60;    // direction d/d phi.psi (objective only)
constexpr int kPhiGamma = 0, kPhiPsi = 3;
constexpr int kCostTracking = 0, kCostURegularisation = 1, kCostXdotRegularisation = 2,
              kCostGamma = 3, kCostPsi = 5, kCostFictitious = 10, kCostPower = 11, kCostTf = 13,
              kCostThetaRegularisation = 14, kCostBeta = 18;
constexpr int kNPartial = 4;    // per interval: f, df/d diam_t, df/d t_f, df/d psi

// Radau IIA nodes (what casadi::collocation_points returns, collocation.py:76)
const long double kRadau[kMaxD + 1][kMaxD] = {
    {},
    {1.0L},
    {0.3333333333333333333333333L, 1.0L},
    {0.1550510257216821901802716L, 0.6449489742783178098197284L, 1.0L},
    {0.08858795951270394739554614L, 0.4094668644407347108649263L, 0.7876594617608470560252419L, 1.0L},
    {0.05710419611451768219312119L, 0.2768430136381238276800460L, 0.5835904323689168200566977L,
     0.8602401356562194478479129L, 1.0L},
    {0.03980985705146874234080669L, 0.1980134178736081725357921L, 0.4379748102473861440050125L,
     0.6954642733536360945146148L, 0.9014649142011735738765011L, 1.0L},
    {0.02931642715978489197205028L, 0.1480785996684842918499769L, 0.3369846902811542990970530L,
     0.5586715187715501320813933L, 0.7692338620300545009168834L, 0.9269456713197411148518740L, 1.0L},
    {0.02247938643871249810882550L, 0.1146790531609042319096402L, 0.2657898227845894684767894L,
     0.4528463736694446169985514L, 0.6473752828868303626260922L, 0.8197593082631076350124201L,
     0.9437374394630778535343478L, 1.0L},
    {0.01777991514736345181320510L, 0.09132360789979395600374146L, 0.2143084793956307583575413L,
     0.3719321645832723024308540L, 0.5451866848034266490322722L, 0.7131752428555694810513138L,
     0.8556337429578544285147815L, 0.9553660447100301492668790L, 1.0L},
};

// Collocation coefficients (collocation.py:67-200): C[j][r] = l_j'(tau_r), D[j] = l_j(1),
// w = C[1:,1:]^{-1} D[1:]
struct Coll {
    int d;
    double tau[kMaxD + 1];
    double C[kMaxD + 1][kMaxD + 1];
    double D[kMaxD + 1];
    double w[kMaxD];
};

Coll make_coll(int d) {
    Coll c{};
    c.d = d;
    const int n = d + 1;
    c.tau[0] = 0.0;
    for (int j = 0; j < d; ++j) c.tau[j + 1] = (double)kRadau[d][j];
    for (int j = 0; j < n; ++j) {
        double val = 1.0;
        for (int r = 0; r < n; ++r)
            if (r != j) val *= (1.0 - c.tau[r]) / (c.tau[j] - c.tau[r]);
        c.D[j] = val;
        for (int m = 0; m < n; ++m) {
            double t = c.tau[m], der = 0.0;
            for (int skip = 0; skip < n; ++skip) {
                if (skip == j) continue;
                double term = 1.0 / (c.tau[j] - c.tau[skip]);
                for (int r = 0; r < n; ++r)
                    if (r != j && r != skip) term *= (t - c.tau[r]) / (c.tau[j] - c.tau[r]);
                der += term;
            }
            c.C[j][m] = der;
        }
    }
    // w = solve(C[1:,1:], D[1:]) by Gaussian elimination with partial pivoting
    double A[kMaxD][kMaxD + 1];
    for (int i = 0; i < d; ++i) {
        for (int j = 0; j < d; ++j) A[i][j] = c.C[i + 1][j + 1];
        A[i][d] = c.D[i + 1];
    }
    for (int col = 0; col < d; ++col) {
        int piv = col;
        for (int i = col + 1; i < d; ++i)
            if (std::fabs(A[i][col]) > std::fabs(A[piv][col])) piv = i;
        for (int j = 0; j <= d; ++j) std::swap(A[col][j], A[piv][j]);
        for (int i = 0; i < d; ++i) {
            if (i == col) continue;
            double fct = A[i][col] / A[col][col];
            for (int j = col; j <= d; ++j) A[i][j] -= fct * A[col][j];
        }
    }
    for (int i = 0; i < d; ++i) c.w[i] = A[i][d] / A[i][i];
    return c;
}

// coefficients the kernel reads (flat, device)
struct DevColl {
    double C[(kMaxD + 1) * (kMaxD + 1)];  // C[j * (d+1) + r] = l_j'(tau_r)
    double D[kMaxD + 1];
    double w[kMaxD];
};

// ---------------------------------------------------------------------------------------
// V / g layout (awebox/ocp/var_struct.py:39-97, constraints.py:48-145)
struct Layout {
    int n_k, d;
    int stride;      // per-interval V stride: x, u, xdot, z, d x (x, z)
    int n_v, n_g, n_p;
    int rows;        // g rows per interval: shooting 24 + path 9 + d*24 + continuity 23
    int v_int0;      // first interval entry in V
    Layout(int nk, int dd) : n_k(nk), d(dd) {
        stride = AWE_NX + AWE_NU + AWE_NX + AWE_NZ + dd * (AWE_NX + AWE_NZ);
        v_int0 = AWE_NTH + AWE_NPHI + AWE_NXI;
        n_v = v_int0 + nk * stride + AWE_NX;
        rows = AWE_N_EQ + AWE_N_INEQ + dd * AWE_N_EQ + AWE_NX;
        n_g = nk * rows + AWE_NX;
        n_p = n_v + AWE_NW + AWE_NCOST + AWE_NTHETA0;
    }
    int x(int k, int i) const { return v_int0 + k * stride + i; }
    int u(int k, int i) const { return v_int0 + k * stride + AWE_NX + i; }
    int xdot(int k, int i) const { return v_int0 + k * stride + AWE_NX + AWE_NU + i; }
    int z(int k) const { return v_int0 + k * stride + 2 * AWE_NX + AWE_NU; }
    int coll_x(int k, int j, int i) const {
        return v_int0 + k * stride + 2 * AWE_NX + AWE_NU + AWE_NZ + j * (AWE_NX + AWE_NZ) + i;
    }
    int coll_z(int k, int j) const {
        return v_int0 + k * stride + 2 * AWE_NX + AWE_NU + AWE_NZ + j * (AWE_NX + AWE_NZ) + AWE_NX;
    }
    int X(int k, int r, int i) const { return r == 0 ? x(k, i) : coll_x(k, r - 1, i); }
    int theta(int i) const { return i; }
    int phi(int i) const { return AWE_NTH + i; }
    int g_shoot(int k) const { return k * rows; }
    int g_coll(int k, int j) const { return k * rows + AWE_N_EQ + AWE_N_INEQ + j * AWE_N_EQ; }
    int g_cont(int k) const { return k * rows + AWE_N_EQ + AWE_N_INEQ + d * AWE_N_EQ; }
    int g_periodic() const { return n_k * rows; }
};

// sorted-name order of the x entries (periodicity, operation.py:245-266)
const int kPeriodicOrder[AWE_NX] = {18, 19, 20, 22, 3, 4, 5, 21, 6, 7, 8, 0, 1, 2,
                                     9, 10, 11, 12, 13, 14, 15, 16, 17};

// ---------------------------------------------------------------------------------------
// device side
// ---------------------------------------------------------------------------------------
struct KArgs {
    const double* V;
    const double* P;
    const double* cst;
    const DevColl* coll;
    const int* pos;                    // [n_k][d+1][64][kTargets]
    const unsigned long long* rowmask; // [d+1][64]
    const int* cont_pos;               // [n_k][23][2]  (x[k+1] col, coll_x[k][d-1] col)
    const int* per_pos;                // [23][2]
    double* g;
    double* jac;
    double* grad;
    double* partial;                   // [batch][n_k][kNPartial]
    double* f;
    int n_k, d, n_v, n_g, n_p, nnz, batch;
    int stride, rows, v_int0;
    int want_derivs;
};

struct LaneIn {
    const double* w;   // LDS: 59 node values (scaled)
    int lane;
    int coll;          // 0 shooting node, 1 collocation node
    double cxx;        // C[jj][jj] / (h tf): xdot_i sensitivity to the node's own state
    double inv_tf;
    __device__ __forceinline__ awe::Dual operator()(int i) const {
        double t = (i == lane) ? 1.0 : 0.0;
        if (coll) {
            if (i >= AWE_NX && i < 2 * AWE_NX) {
                if (lane == i - AWE_NX) t = cxx;
                if (lane == AWE_NW - 1) t = -w[i] * inv_tf;   // d/d t_f of xdot = C X/(h tf)
            }
        }
        return awe::Dual(w[i], t);
    }
};

// streams one node's rows: g value (lane r writes row r) and the lane's Jacobian entries
struct KernelSink {
    double* g;
    double* jac;
    int g_eq0, g_ineq0, lane;
    bool derivs;
    unsigned long long m;
    int p[kTargets];
    double sc[kTargets];
    awe::Dual pw, bt;
    __device__ __forceinline__ void emit(int r, const awe::Dual& v, int g_row) {
        if (lane == r) g[g_row] = v.v;
        if (derivs && ((m >> r) & 1ull)) {
            const int c = __popcll(m & ((1ull << r) - 1ull));
#pragma unroll
            for (int t = 0; t < kTargets; ++t)
                if (p[t] >= 0) jac[p[t] + c] = sc[t] * v.d;
        }
    }
    __device__ __forceinline__ void eq_row(int r, const awe::Dual& v) { emit(r, v, g_eq0 + r); }
    __device__ __forceinline__ void ineq_row(int r, const awe::Dual& v) {
        emit(AWE_N_EQ + r, v, g_ineq0 + r);
    }
    __device__ __forceinline__ void power(const awe::Dual& v) { pw = v; }
    __device__ __forceinline__ void beta(const awe::Dual& v) { bt = v; }
};

template <int D>
__global__ __launch_bounds__(64) void ap2_interval_kernel(KArgs a) {
    constexpr int NN = D + 1;
    const int lane = threadIdx.x;
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

    // ---- stage the interval's V slice: [theta, phi, x[k], u, xdot, z, coll..., x[k+1]] ---
    constexpr int NLOC_MAX = 9 + AWE_NX + AWE_NU + AWE_NX + AWE_NZ + 9 * (AWE_NX + AWE_NZ) + AWE_NX;
    __shared__ double vloc[NLOC_MAX];
    __shared__ double wn[AWE_NW];
    const int nloc_int = a.stride + AWE_NX;
    const int base = a.v_int0 + k * a.stride;
    for (int i = lane; i < 9; i += kLanes) vloc[i] = V[i];
    for (int i = lane; i < nloc_int; i += kLanes) vloc[9 + i] = V[base + i];
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
    const double* C = a.coll->C;

    awe::Dual gamma(vt[2 + kPhiGamma], lane == kLaneGamma ? 1.0 : 0.0);
    awe::Dual psi(vt[2 + kPhiPsi], lane == kLanePsi ? 1.0 : 0.0);
    awe::Dual tfd(tf, lane == AWE_NW - 1 ? 1.0 : 0.0);

    // effective regularisation weights (objective.py:147-170)
    const double w_track = cost[kCostTracking] / a.cst[AWE_C_NORM_TRACKING];
    const double w_xdot = cost[kCostXdotRegularisation] / a.cst[AWE_C_NORM_XDOT_REG];
    const double w_ureg = cost[kCostURegularisation] / a.cst[AWE_C_NORM_U_REG];
    const double w_fict = cost[kCostFictitious] / a.cst[AWE_C_NORM_FICTITIOUS];
    const double w_theta = cost[kCostThetaRegularisation] / a.cst[AWE_C_NORM_THETA_REG];

    // gradient accumulators (lane = direction)
    double gx[NN], gxd[NN];
    for (int r = 0; r < NN; ++r) { gx[r] = 0.0; gxd[r] = 0.0; }
    double gu = 0.0, gglob = 0.0;
    double gz[NN];
    for (int r = 0; r < NN; ++r) gz[r] = 0.0;
    double fsum = 0.0;

    const unsigned long long* rmask = a.rowmask;
    const int* pos_k = a.pos + (size_t)k * NN * kLanes * kTargets;

#pragma unroll 1
    for (int node = 0; node < NN; ++node) {
        // ---- node variables into LDS --------------------------------------------------
        __syncthreads();
        if (node == 0) {
            if (lane < AWE_NX) wn[lane] = vx[lane];
            else if (lane < 2 * AWE_NX) wn[lane] = vxd[lane - AWE_NX];
            else if (lane < 2 * AWE_NX + AWE_NU) wn[lane] = vu[lane - 2 * AWE_NX];
            else if (lane < 2 * AWE_NX + AWE_NU + AWE_NZ) wn[lane] = vz[0];
            else if (lane < AWE_NW) wn[lane] = vt[lane - (2 * AWE_NX + AWE_NU + AWE_NZ)];
        } else {
            const double* cx = vcoll + (node - 1) * (AWE_NX + AWE_NZ);
            if (lane < AWE_NX) {
                wn[lane] = cx[lane];
            } else if (lane < 2 * AWE_NX) {
                const int i = lane - AWE_NX;
                double xp = 0.0;
#pragma unroll
                for (int r = 0; r < NN; ++r) {
                    const double Xr = (r == 0) ? vx[i] : vcoll[(r - 1) * (AWE_NX + AWE_NZ) + i];
                    xp += C[r * NN + node] * Xr;
                }
                wn[lane] = xp / h / tf;
            } else if (lane < 2 * AWE_NX + AWE_NU) {
                wn[lane] = vu[lane - 2 * AWE_NX];
            } else if (lane < 2 * AWE_NX + AWE_NU + AWE_NZ) {
                wn[lane] = cx[AWE_NX];
            } else if (lane < AWE_NW) {
                wn[lane] = vt[lane - (2 * AWE_NX + AWE_NU + AWE_NZ)];
            }
        }
        __syncthreads();

        LaneIn in{wn, lane, node > 0 ? 1 : 0, C[node * NN + node] * inv_h_tf, 1.0 / tf};
        KernelSink sink;
        sink.g = g;
        sink.jac = jac;
        sink.lane = lane;
        sink.derivs = a.want_derivs != 0 && lane <= kLaneGamma;
        sink.g_eq0 = node == 0 ? k * a.rows : k * a.rows + AWE_N_EQ + AWE_N_INEQ + (node - 1) * AWE_N_EQ;
        sink.g_ineq0 = k * a.rows + AWE_N_EQ;
        sink.m = (lane <= kLaneGamma) ? rmask[node * kLanes + lane] : 0ull;
        {
            const int* pl = pos_k + ((size_t)node * kLanes + (lane & 63)) * kTargets;
            const bool xd_lane = node > 0 && lane >= AWE_NX && lane < 2 * AWE_NX;
            int t = 0;
#pragma unroll
            for (int rr = 0; rr < NN; ++rr) {
                if (xd_lane && rr != node && t < kTargets) {
                    sink.p[t] = pl[t];
                    sink.sc[t] = C[rr * NN + node] * inv_h_tf;
                    ++t;
                }
            }
            if (!xd_lane) {
                sink.p[0] = pl[0];
                sink.sc[0] = 1.0;
                t = 1;
            }
            for (; t < kTargets; ++t) { sink.p[t] = -1; sink.sc[t] = 0.0; }
        }
        awe::ap2_node<awe::Dual>(in, gamma, th, a.cst, sink, node == 0);

        // ---- objective (collocation nodes only; objective.py:45-544) ----------------------
        if (node > 0) {
            const int j = node - 1;
            const double wj = a.coll->w[j];
            // refs: coll x/z from P.p.ref, xdot ref 0, u ref u[k], theta ref
            const double* rb = vref + base;  // ref V slice of this interval
            const double* rcx = rb + 2 * AWE_NX + AWE_NU + AWE_NZ + j * (AWE_NX + AWE_NZ);
            awe::Dual track(0.0), xdreg(0.0), ureg(0.0), fict(0.0), threg(0.0);
            for (int i = 0; i < AWE_NX; ++i) {
                awe::Dual dv = in(i) - rcx[i];
                track += (wts[i] * w_track) * (dv * dv);
            }
            {
                awe::Dual dz = in(2 * AWE_NX + AWE_NU) - rcx[AWE_NX];
                track += (wts[2 * AWE_NX + AWE_NU] * w_track) * (dz * dz);
            }
            for (int i = 0; i < AWE_NX; ++i) {
                awe::Dual dv = in(AWE_NX + i);
                xdreg += (wts[AWE_NX + i] * w_xdot) * (dv * dv);
            }
            const double* ru = rb + AWE_NX;
            for (int i = 0; i < AWE_NU; ++i) {
                awe::Dual dv = in(2 * AWE_NX + i) - ru[i];
                const double wi = wts[2 * AWE_NX + i];
                if (i < 6) fict += (wi * w_fict) * (dv * dv);
                else ureg += (wi * w_ureg) * (dv * dv);
            }
            {
                awe::Dual dv = in(2 * AWE_NX + AWE_NU + AWE_NZ) - vref[0];
                threg += (wts[2 * AWE_NX + AWE_NU + AWE_NZ] * w_theta) * (dv * dv);
            }
            awe::Dual regs = wj * (psi * track + xdreg + ureg + fict + threg);
            awe::Dual beta_c = (cost[kCostBeta] * wj / a.cst[AWE_C_NORM_BETA]) * (sink.bt * sink.bt);
            // power: -c_p * (tf/N) w_j p / tf  (collocation.py:272-316, objective.py:279-298)
            awe::Dual pw = (-cost[kCostPower]) * ((tfd / (double)a.n_k) * (wj * sink.pw)) / tfd;
            awe::Dual fn = regs + beta_c + (1.0 - psi) * pw;
            fsum += fn.v;
            const double dfn = fn.d;
            if (lane < AWE_NX) {
                gx[node] += dfn;
            } else if (lane < 2 * AWE_NX) {
#pragma unroll
                for (int rr = 0; rr < NN; ++rr)
                    if (rr != node) gxd[rr] += C[rr * NN + node] * inv_h_tf * dfn;
            } else if (lane < 2 * AWE_NX + AWE_NU) {
                gu += dfn;
            } else if (lane == 2 * AWE_NX + AWE_NU) {
                gz[node] += dfn;
            } else {
                gglob += dfn;   // diam_t (57), t_f (58), gamma (59), psi (60)
            }
        }
    }

    // ---- continuity rows (collocation.py:319-336) ---------------------------------------
    const DevColl* cc = a.coll;
    if (lane < AWE_NX) {
        double xf = 0.0;
#pragma unroll
        for (int r = 0; r < NN; ++r) {
            if (cc->D[r] == 0.0) continue;   // structural zero (CasADi drops 0 * x)
            const double Xr = (r == 0) ? vx[lane] : vcoll[(r - 1) * (AWE_NX + AWE_NZ) + lane];
            xf += cc->D[r] * Xr;
        }
        g[k * a.rows + AWE_N_EQ + AWE_N_INEQ + D * AWE_N_EQ + lane] = vx1[lane] - xf;
        if (a.want_derivs) {
            const int* cp = a.cont_pos + ((size_t)k * AWE_NX + lane) * 2;
            jac[cp[0]] = 1.0;
            jac[cp[1]] = -cc->D[D];
        }
    }

    if (!a.want_derivs) {
        if (lane == 0) a.partial[((size_t)b * a.n_k + k) * kNPartial] = fsum;
        return;
    }

    // ---- gradient of the interval's local columns --------------------------------------
    // X_{k,r} columns: xdot-lane i holds sum over nodes of the polynomial path, x-lane i the
    // direct path of node r.
    double gx_from_x[NN];
#pragma unroll
    for (int r = 0; r < NN; ++r) gx_from_x[r] = __shfl(gx[r], lane - AWE_NX);
    if (lane >= AWE_NX && lane < 2 * AWE_NX) {
        const int i = lane - AWE_NX;
        grad[base + i] = gxd[0];                                       // x[k]
#pragma unroll
        for (int r = 1; r < NN; ++r)
            grad[base + 2 * AWE_NX + AWE_NU + AWE_NZ + (r - 1) * (AWE_NX + AWE_NZ) + i] = gxd[r] + gx_from_x[r];
        grad[base + AWE_NX + AWE_NU + i] = 0.0;                         // xdot[k] (shooting)
    } else if (lane >= 2 * AWE_NX && lane < 2 * AWE_NX + AWE_NU) {
        grad[base + AWE_NX + (lane - 2 * AWE_NX)] = gu;                 // u[k]
    } else if (lane == 2 * AWE_NX + AWE_NU) {
        grad[base + 2 * AWE_NX + AWE_NU] = 0.0;                         // z[k] (shooting)
#pragma unroll
        for (int r = 1; r < NN; ++r)
            grad[base + 2 * AWE_NX + AWE_NU + AWE_NZ + (r - 1) * (AWE_NX + AWE_NZ) + AWE_NX] = gz[r];
    }
    double* part = a.partial + ((size_t)b * a.n_k + k) * kNPartial;
    if (lane == 0) part[0] = fsum;
    if (lane == AWE_NW - 2) part[1] = gglob;   // diam_t
    if (lane == AWE_NW - 1) part[2] = gglob;   // t_f
    if (lane == kLanePsi) part[3] = gglob;     // psi
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
    double* jac = a.jac + (size_t)b * a.nnz;
    double* grad = a.grad + (size_t)b * a.n_v;
    const double* part = a.partial + (size_t)b * a.n_k * kNPartial;

    double s[kNPartial] = {0.0, 0.0, 0.0, 0.0};
    for (int k = lane; k < a.n_k; k += kLanes)
        for (int c = 0; c < kNPartial; ++c) s[c] += part[k * kNPartial + c];
    for (int off = 32; off > 0; off >>= 1)
        for (int c = 0; c < kNPartial; ++c) s[c] += __shfl_xor(s[c], off);

    const double tf = V[1], tf_ref = vref[1];
    // periodic rows: x_0 - x_terminal in sorted-name order
    const int last = a.v_int0 + (a.n_k - 1) * a.stride + 2 * AWE_NX + AWE_NU + AWE_NZ +
                     (a.d - 1) * (AWE_NX + AWE_NZ);
    if (lane < AWE_NX) {
        const int i = kPeriodicOrder[lane];
        g[a.n_k * a.rows + lane] = V[a.v_int0 + i] - V[last + i];
        if (a.want_derivs) {
            jac[a.per_pos[lane * 2 + 0]] = 1.0;
            jac[a.per_pos[lane * 2 + 1]] = -1.0;
        }
    }
    if (lane == 0) {
        double fh = 0.0;
        for (int i = 0; i < AWE_NPHI; ++i) {
            // phi order gamma, tau, iota, psi, eta, nu, upsilon (system.py:435-450); cost
            // order gamma, iota, psi, tau, eta, nu, upsilon (discretization.py:129-152)
            static const int phi_cost_map[AWE_NPHI] = {3, 6, 4, 5, 7, 8, 9};
            fh += cost[phi_cost_map[i]] * V[AWE_NTH + i];
        }
        const double time_cost = cost[kCostTf] * (tf - tf_ref) * (tf - tf_ref);
        a.f[b] = s[0] + time_cost + fh;
    }
    if (a.want_derivs) {
        if (lane == 0) grad[0] = s[1];
        if (lane == 1) grad[1] = s[2] + cost[kCostTf] * 2.0 * (tf - tf_ref);
        if (lane >= 2 && lane < 2 + AWE_NPHI) {
            static const int phi_cost_map[AWE_NPHI] = {3, 6, 4, 5, 7, 8, 9};
            const int i = lane - 2;
            double gphi = cost[phi_cost_map[i]];
            if (i == kPhiPsi) gphi += s[3];
            grad[AWE_NTH + i] = gphi;
        }
        if (lane >= 2 + AWE_NPHI && lane < 2 + AWE_NPHI + AWE_NXI) grad[lane] = 0.0;
        if (lane < AWE_NX) grad[a.v_int0 + a.n_k * a.stride + lane] = 0.0;   // x[n_k]
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
struct awe_handle_s {
    int n_k = 0, d = 0, batch = 0;
    Layout lay{1, 1};
    Coll coll{};
    std::vector<double> cst;
    std::vector<int> colind, row;
    int nnz = 0;
    // device
    double* d_cst = nullptr;
    DevColl* d_coll = nullptr;
    int* d_pos = nullptr;
    unsigned long long* d_rowmask = nullptr;
    int* d_cont = nullptr;
    int* d_per = nullptr;
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

// structural dependency of every model output on the 59 node variables + gamma (bit 59)
struct DepIn {
    __host__ awe::Dep operator()(int i) const { return awe::Dep::bit(i); }
};

void model_masks(const double* cst, unsigned long long eqm[AWE_N_EQ], unsigned long long ineqm[AWE_N_INEQ]) {
    std::vector<double> th(AWE_NTHETA0, 1.0);   // values are irrelevant for the structure
    DepIn in;
    awe::NodeResult<awe::Dep> res;
    awe::ap2_node<awe::Dep>(in, awe::Dep::bit(kLaneGamma), th.data(), cst, res, true);
    for (int r = 0; r < AWE_N_EQ; ++r) eqm[r] = res.eq[r].m;
    for (int r = 0; r < AWE_N_INEQ; ++r) ineqm[r] = res.ineq[r].m;
}

int launch(awe_handle h, const double* V, const double* P, double* f, double* g, double* grad,
           double* jac, int want_derivs, hipStream_t stream) {
    KArgs a{};
    a.V = V; a.P = P; a.cst = h->d_cst; a.coll = h->d_coll; a.pos = h->d_pos;
    a.rowmask = h->d_rowmask; a.cont_pos = h->d_cont; a.per_pos = h->d_per;
    a.g = g; a.jac = jac; a.grad = grad; a.partial = h->d_partial; a.f = f;
    a.n_k = h->n_k; a.d = h->d; a.n_v = h->lay.n_v; a.n_g = h->lay.n_g; a.n_p = h->lay.n_p;
    a.nnz = h->nnz; a.batch = h->batch; a.stride = h->lay.stride; a.rows = h->lay.rows;
    a.v_int0 = h->lay.v_int0; a.want_derivs = want_derivs;
    dim3 grid(h->batch * h->n_k), block(kLanes);
    HIP_TRY(hipEventRecord(h->ev[0], stream));
    switch (h->d) {
        case 1: hipLaunchKernelGGL(ap2_interval_kernel<1>, grid, block, 0, stream, a); break;
        case 2: hipLaunchKernelGGL(ap2_interval_kernel<2>, grid, block, 0, stream, a); break;
        case 3: hipLaunchKernelGGL(ap2_interval_kernel<3>, grid, block, 0, stream, a); break;
        case 4: hipLaunchKernelGGL(ap2_interval_kernel<4>, grid, block, 0, stream, a); break;
        case 5: hipLaunchKernelGGL(ap2_interval_kernel<5>, grid, block, 0, stream, a); break;
        default: return fail(AWE_ERR_ARG, "unsupported collocation degree");
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev[1], stream));
    hipLaunchKernelGGL(ap2_finalize_kernel, dim3(h->batch), block, 0, stream, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(h->ev[2], stream));
    h->timed = true;
    return AWE_OK;
}

}  // namespace

namespace {
struct HostTables {
    std::vector<int> pos, cont, per;
    std::vector<unsigned long long> rowmask;
};

// CPU-only: collocation coefficients, structural masks of the node model, the CCS pattern of
// J_g and the kernel's slot tables.
int build_tables(awe_handle_s* h, int n_k, int d, const double* consts, int n_consts, HostTables& T) {
    h->n_k = n_k; h->d = d;
    h->lay = Layout(n_k, d);
    h->coll = make_coll(d);
    h->cst.assign(consts, consts + n_consts);
    const Layout& L = h->lay;
    const Coll& cl = h->coll;
    const int NN = d + 1;

    // ---- structural masks of the node model --------------------------------------------
    unsigned long long eqm[AWE_N_EQ], ineqm[AWE_N_INEQ];
    model_masks(h->cst.data(), eqm, ineqm);
    auto rows_on = [&](int var, bool with_ineq) {   // bitmask of rows depending on node var
        unsigned long long m = 0;
        for (int r = 0; r < AWE_N_EQ; ++r) if ((eqm[r] >> var) & 1ull) m |= 1ull << r;
        if (with_ineq)
            for (int r = 0; r < AWE_N_INEQ; ++r) if ((ineqm[r] >> var) & 1ull) m |= 1ull << (AWE_N_EQ + r);
        return m;
    };
    // lane row masks: [node][lane]
    std::vector<unsigned long long> rowmask((size_t)NN * kLanes, 0ull);
    for (int lane = 0; lane <= kLaneGamma; ++lane) rowmask[lane] = rows_on(lane, true);
    for (int node = 1; node < NN; ++node) {
        for (int lane = 0; lane <= kLaneGamma; ++lane) {
            unsigned long long m = rows_on(lane, false);
            if (lane < AWE_NX) m |= rows_on(AWE_NX + lane, false);
            if (lane == AWE_NW - 1)
                for (int i = 0; i < AWE_NX; ++i) m |= rows_on(AWE_NX + i, false);
            rowmask[(size_t)node * kLanes + lane] = m;
        }
    }

    // ---- target columns of each (k, node, lane) -----------------------------------------
    auto lane_col_shoot = [&](int k, int lane) -> int {
        if (lane < AWE_NX) return L.x(k, lane);
        if (lane < 2 * AWE_NX) return L.xdot(k, lane - AWE_NX);
        if (lane < 2 * AWE_NX + AWE_NU) return L.u(k, lane - 2 * AWE_NX);
        if (lane < 2 * AWE_NX + AWE_NU + AWE_NZ) return L.z(k);
        if (lane < AWE_NW) return L.theta(lane - (2 * AWE_NX + AWE_NU + AWE_NZ));
        return L.phi(kPhiGamma);
    };
    auto lane_cols_coll = [&](int k, int node, int lane, std::vector<int>& cols) {
        cols.clear();
        if (lane < AWE_NX) { cols.push_back(L.coll_x(k, node - 1, lane)); return; }
        if (lane < 2 * AWE_NX) {
            for (int r = 0; r < NN; ++r) if (r != node) cols.push_back(L.X(k, r, lane - AWE_NX));
            return;
        }
        if (lane < 2 * AWE_NX + AWE_NU) { cols.push_back(L.u(k, lane - 2 * AWE_NX)); return; }
        if (lane < 2 * AWE_NX + AWE_NU + AWE_NZ) { cols.push_back(L.coll_z(k, node - 1)); return; }
        if (lane < AWE_NW) { cols.push_back(L.theta(lane - (2 * AWE_NX + AWE_NU + AWE_NZ))); return; }
        cols.push_back(L.phi(kPhiGamma));
    };

    // ---- triplets -----------------------------------------------------------------------
    std::vector<std::pair<int, int>> trip;   // (col, row)
    trip.reserve(200000);
    std::vector<int> cols;
    for (int k = 0; k < n_k; ++k) {
        for (int lane = 0; lane <= kLaneGamma; ++lane) {
            unsigned long long m = rowmask[lane];
            for (int r = 0; r < AWE_N_EQ + AWE_N_INEQ; ++r)
                if ((m >> r) & 1ull) trip.emplace_back(lane_col_shoot(k, lane), L.g_shoot(k) + r);
        }
        for (int node = 1; node < NN; ++node)
            for (int lane = 0; lane <= kLaneGamma; ++lane) {
                unsigned long long m = rowmask[(size_t)node * kLanes + lane];
                lane_cols_coll(k, node, lane, cols);
                for (int c : cols)
                    for (int r = 0; r < AWE_N_EQ; ++r)
                        if ((m >> r) & 1ull) trip.emplace_back(c, L.g_coll(k, node - 1) + r);
            }
        for (int i = 0; i < AWE_NX; ++i) {
            trip.emplace_back(L.x(k + 1, i), L.g_cont(k) + i);
            for (int r = 0; r < NN; ++r)
                if (cl.D[r] != 0.0) trip.emplace_back(L.X(k, r, i), L.g_cont(k) + i);
        }
    }
    const int last = L.coll_x(n_k - 1, d - 1, 0);
    for (int i = 0; i < AWE_NX; ++i) {
        trip.emplace_back(L.x(0, kPeriodicOrder[i]), L.g_periodic() + i);
        trip.emplace_back(last + kPeriodicOrder[i], L.g_periodic() + i);
    }
    std::sort(trip.begin(), trip.end());
    trip.erase(std::unique(trip.begin(), trip.end()), trip.end());
    h->nnz = (int)trip.size();
    h->colind.assign(L.n_v + 1, 0);
    h->row.resize(h->nnz);
    for (int i = 0; i < h->nnz; ++i) {
        h->colind[trip[i].first + 1]++;
        h->row[i] = trip[i].second;
    }
    for (int c = 0; c < L.n_v; ++c) h->colind[c + 1] += h->colind[c];
    auto find = [&](int col, int rw) -> int {
        auto b = h->row.begin() + h->colind[col], e = h->row.begin() + h->colind[col + 1];
        auto it = std::lower_bound(b, e, rw);
        if (it == e || *it != rw) return -1;
        return (int)(it - h->row.begin());
    };

    // ---- kernel position tables ---------------------------------------------------------
    std::vector<int> pos((size_t)n_k * NN * kLanes * kTargets, -1);
    int bad = 0;
    for (int k = 0; k < n_k; ++k)
        for (int node = 0; node < NN; ++node)
            for (int lane = 0; lane <= kLaneGamma; ++lane) {
                unsigned long long m = rowmask[(size_t)node * kLanes + lane];
                if (!m) continue;
                if (node == 0) cols.assign(1, lane_col_shoot(k, lane));
                else lane_cols_coll(k, node, lane, cols);
                const int g0 = node == 0 ? L.g_shoot(k) : L.g_coll(k, node - 1);
                const int first = __builtin_ctzll(m);
                for (size_t t = 0; t < cols.size(); ++t) {
                    int p = find(cols[t], g0 + first);
                    // the node's rows must be consecutive entries of the column
                    int cnt = 0;
                    for (int r = 0; r < 64; ++r)
                        if ((m >> r) & 1ull) {
                            if (find(cols[t], g0 + r) != p + cnt) ++bad;
                            ++cnt;
                        }
                    pos[(((size_t)k * NN + node) * kLanes + lane) * kTargets + t] = p;
                }
            }
    std::vector<int> cont((size_t)n_k * AWE_NX * 2, -1);
    for (int k = 0; k < n_k; ++k)
        for (int i = 0; i < AWE_NX; ++i) {
            cont[((size_t)k * AWE_NX + i) * 2 + 0] = find(L.x(k + 1, i), L.g_cont(k) + i);
            cont[((size_t)k * AWE_NX + i) * 2 + 1] = find(L.X(k, d, i), L.g_cont(k) + i);
        }
    std::vector<int> per(AWE_NX * 2);
    for (int i = 0; i < AWE_NX; ++i) {
        per[i * 2 + 0] = find(L.x(0, kPeriodicOrder[i]), L.g_periodic() + i);
        per[i * 2 + 1] = find(last + kPeriodicOrder[i], L.g_periodic() + i);
    }
    for (int c = 0; c < (int)cont.size(); ++c) if (cont[c] < 0) ++bad;
    for (int c = 0; c < (int)per.size(); ++c) if (per[c] < 0) ++bad;
    for (int r = 0; r < NN; ++r)
        if (r < d && cl.D[r] != 0.0) ++bad;   // the kernel assumes D = e_d (Radau)
    if (bad) return fail(AWE_ERR_ARG, "internal: inconsistent sparsity tables");
    T.pos.swap(pos);
    T.rowmask.swap(rowmask);
    T.cont.swap(cont);
    T.per.swap(per);
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
    HostTables T;
    int rc = build_tables(h, n_k, d, consts, n_consts, T);
    if (rc) { delete h; return rc; }
    const Coll& cl = h->coll;
    const int NN = d + 1;
    std::vector<int>& pos = T.pos;
    std::vector<unsigned long long>& rowmask = T.rowmask;
    std::vector<int>& cont = T.cont;
    std::vector<int>& per = T.per;
    DevColl dc{};
    for (int j = 0; j < NN; ++j)
        for (int r = 0; r < NN; ++r) dc.C[j * NN + r] = cl.C[j][r];
    for (int j = 0; j < NN; ++j) dc.D[j] = cl.D[j];
    for (int j = 0; j < d; ++j) dc.w[j] = cl.w[j];

#define ALLOC_COPY(dst, src, n)                                                     \
    HIP_TRY(hipMalloc((void**)&dst, sizeof(*dst) * (n)));                          \
    HIP_TRY(hipMemcpy(dst, src, sizeof(*dst) * (n), hipMemcpyHostToDevice))
    ALLOC_COPY(h->d_cst, h->cst.data(), h->cst.size());
    ALLOC_COPY(h->d_coll, &dc, 1);
    ALLOC_COPY(h->d_pos, pos.data(), pos.size());
    ALLOC_COPY(h->d_rowmask, rowmask.data(), rowmask.size());
    ALLOC_COPY(h->d_cont, cont.data(), cont.size());
    ALLOC_COPY(h->d_per, per.data(), per.size());
#undef ALLOC_COPY
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
    awe_handle_s h;
    HostTables T;
    int rc = build_tables(&h, n_k, d, consts, n_consts, T);
    if (rc) return rc;
    *nnz = h.nnz;
    if (colind) std::memcpy(colind, h.colind.data(), sizeof(int) * h.colind.size());
    if (row) std::memcpy(row, h.row.data(), sizeof(int) * h.row.size());
    return AWE_OK;
}

int awe_destroy(awe_handle h) {
    if (!h) return AWE_OK;
    hipFree(h->d_cst); hipFree(h->d_coll); hipFree(h->d_pos); hipFree(h->d_rowmask);
    hipFree(h->d_cont); hipFree(h->d_per); hipFree(h->d_partial);
    hipFree(h->d_scr_jac); hipFree(h->d_scr_grad); hipFree(h->d_scr_g); hipFree(h->d_scr_f);
    hipFree(h->d_in_V); hipFree(h->d_in_P);
    for (int i = 0; i < 3; ++i) if (h->ev[i]) hipEventDestroy(h->ev[i]);
    delete h;
    return AWE_OK;
}

int awe_sizes(awe_handle h, int* n_v, int* n_g, int* n_p, int* nnz_jac) {
    if (!h) return fail(AWE_ERR_ARG, "null handle");
    if (n_v) *n_v = h->lay.n_v;
    if (n_g) *n_g = h->lay.n_g;
    if (n_p) *n_p = h->lay.n_p;
    if (nnz_jac) *nnz_jac = h->nnz;
    return AWE_OK;
}

int awe_sparsity_jac(awe_handle h, int* colind, int* row) {
    if (!h || !colind || !row) return fail(AWE_ERR_ARG, "null argument");
    std::memcpy(colind, h->colind.data(), sizeof(int) * h->colind.size());
    std::memcpy(row, h->row.data(), sizeof(int) * h->row.size());
    return AWE_OK;
}

static int ensure_scratch(awe_handle h) {
    if (!h->d_scr_jac) HIP_TRY(hipMalloc((void**)&h->d_scr_jac, sizeof(double) * (size_t)h->batch * h->nnz));
    if (!h->d_scr_grad) HIP_TRY(hipMalloc((void**)&h->d_scr_grad, sizeof(double) * (size_t)h->batch * h->lay.n_v));
    if (!h->d_scr_g) HIP_TRY(hipMalloc((void**)&h->d_scr_g, sizeof(double) * (size_t)h->batch * h->lay.n_g));
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
    if (!h->d_in_V) HIP_TRY(hipMalloc((void**)&h->d_in_V, sizeof(double) * nb * h->lay.n_v));
    if (!h->d_in_P) HIP_TRY(hipMalloc((void**)&h->d_in_P, sizeof(double) * nb * h->lay.n_p));
    HIP_TRY(hipMemcpy(h->d_in_V, V, sizeof(double) * nb * h->lay.n_v, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->d_in_P, P, sizeof(double) * nb * h->lay.n_p, hipMemcpyHostToDevice));
    rc = launch(h, h->d_in_V, h->d_in_P, h->d_scr_f, h->d_scr_g, h->d_scr_grad, h->d_scr_jac, 1, nullptr);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(f, h->d_scr_f, sizeof(double) * nb, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(g, h->d_scr_g, sizeof(double) * nb * h->lay.n_g, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(grad_f, h->d_scr_grad, sizeof(double) * nb * h->lay.n_v, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(jac, h->d_scr_jac, sizeof(double) * nb * h->nnz, hipMemcpyDeviceToHost));
    auto finite = [](const double* x, size_t n) {
        for (size_t i = 0; i < n; ++i) if (!std::isfinite(x[i])) return false;
        return true;
    };
    if (!finite(f, nb) || !finite(g, nb * h->lay.n_g) || !finite(grad_f, nb * h->lay.n_v) ||
        !finite(jac, nb * h->nnz))
        return fail(AWE_ERR_NONFINITE, "non-finite value in NLP evaluation");
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
