// CPU port of the AP2 collocation evaluator -- TEST AND BASELINE INFRASTRUCTURE ONLY.
//
// Used by bench.py's cpu_baseline leg (kind "port": the build's C++ CPU restatement of the hot
// path, SURVEY.md section 8(d), OpenMP over (instance, interval)) and by the CPU test suite as a
// check of the evaluator's *algorithm* (direction colouring, gather list, objective pass) on a
// machine without a GPU.  It shares the node model (awebox_amd/csrc/ap2_model.hpp) and the host
// tables (ap2_tables.hpp) with the HIP library, so it is NOT an independent oracle: fp64 parity
// of the product is judged against oracle/ap2_oracle.py (automatic differentiation of a separate
// restatement of the reference's Lagrangian model).
//
// Per interval it mirrors ap2_interval_kernel: node values, one vector-dual model evaluation per
// node carrying all colours at once (DualN<32> instead of one colour per GPU lane), the
// objective's directional derivatives, g rows, grad f columns and the CCS values via the gather
// list; a finalize step per instance reduces the interval partials.
#include <omp.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "ap2_tables.hpp"
#include "dualn.hpp"

namespace {

using namespace awt;
using DN = cpu::DualN<kHalf>;

thread_local std::string g_err;

struct CpuIn {
    const double* w;
    const ColorTabs* ct;
    int kind;
    double cxx, inv_tf;
    DN operator()(int i) const {
        DN r(w[i]);
        for (int c = 0; c < kHalf; ++c) {
            double t = ((ct->seedA[kind][c] >> i) & 1ull) ? 1.0 : 0.0;
            if (i >= AWE_NX && i < 2 * AWE_NX) {
                const int j = i - AWE_NX;
                if ((ct->seedA[kind][c] >> j) & 1ull) t += cxx;
                if ((ct->seedXD[kind][c] >> j) & 1u) t += 1.0;
                if (c == ct->tf_color[kind]) t += -inv_tf * w[i];
            }
            r.d[c] = t;
        }
        return r;
    }
};

struct CpuSink {
    double* tang;   // node's tangent buffer
    double* gv;
    const ColorTabs* ct;
    int kind;
    void emit(int r, const DN& v) {
        gv[r] = v.v;
        for (int c = 0; c < kHalf; ++c) {
            const unsigned long long cm = ct->cmask[kind][c];
            if ((cm >> r) & 1ull) tang[ct->off[kind][c] + __builtin_popcountll(cm & ((1ull << r) - 1ull))] = v.d[c];
        }
    }
    void eq_row(int r, const DN& v) { emit(r, v); }
    void ineq_row(int r, const DN& v) { emit(AWE_N_EQ + r, v); }
    void power(const DN& v) { emit(kRowPower, v); }
    void beta(const DN& v) { emit(kRowBeta, v); }
};

struct Handle {
    Ap2Tables t;
    Ap2HessTables ht;
};

// hyper-dual inputs: e1 along colour c1, e2 along colour c2 (same seeds as the first-order pass)
struct CpuHIn {
    const double* w;
    const ColorTabs* ct;
    int kind, c1, c2;
    double cxx, inv_tf;
    double seed(int c, int i) const {
        double t = ((ct->seedA[kind][c] >> i) & 1ull) ? 1.0 : 0.0;
        if (i >= AWE_NX && i < 2 * AWE_NX) {
            const int j = i - AWE_NX;
            if ((ct->seedA[kind][c] >> j) & 1ull) t += cxx;
            if ((ct->seedXD[kind][c] >> j) & 1u) t += 1.0;
            if (c == ct->tf_color[kind]) t += -inv_tf * w[i];
        }
        return t;
    }
    awe::HDual operator()(int i) const { return awe::HDual(w[i], seed(c1, i), seed(c2, i), 0.0); }
};

struct CpuHSink {
    double* hd;            // node's direction-pair Hessian
    const HessTabs* ht;
    const double* mu;      // row weights
    int kind, c1, c2;
    void emit(int r, const awe::HDual& v) {
        const int p = ht->pdir[kind][c1][r], q = ht->pdir[kind][c2][r];
        if (p < 0 || q < 0) return;
        const int idx = ht->pidx[kind][p][q];
        if (idx >= 0) hd[idx] += mu[r] * v.ab;
    }
    void eq_row(int r, const awe::HDual& v) { emit(r, v); }
    void ineq_row(int r, const awe::HDual& v) { emit(AWE_N_EQ + r, v); }
    void power(const awe::HDual& v) { emit(kRowPower, v); }
    void beta(const awe::HDual& v) { emit(kRowBeta, v); }
};

// scaled node values of the interval's nodes; xdot at Radau nodes from the polynomial
void node_values(const Ap2Tables& T, int k, const double* V, std::vector<double>& wn) {
    const Layout& L = T.lay;
    const int d = T.d, NN = d + 1;
    const double* C = T.dcoll.C;
    const int base = L.v_int0 + k * L.stride;
    const double* vt = V;
    const double* vx = V + base;
    const double* vu = vx + AWE_NX;
    const double* vxd = vu + AWE_NU;
    const double* vz = vxd + AWE_NX;
    const double* vcoll = vz + AWE_NZ;
    const double tf = vt[1];
    const double h = 1.0 / T.n_k;
    wn.assign((size_t)NN * 64, 0.0);
    for (int n = 0; n < NN; ++n)
        for (int i = 0; i < AWE_NW; ++i) {
            double val;
            if (i < AWE_NX) {
                val = n == 0 ? vx[i] : vcoll[(n - 1) * (AWE_NX + AWE_NZ) + i];
            } else if (i < 2 * AWE_NX) {
                const int s = i - AWE_NX;
                if (n == 0) {
                    val = vxd[s];
                } else {
                    double xp = 0.0;
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
            } else {
                val = vt[i - (2 * AWE_NX + AWE_NU + AWE_NZ)];
            }
            wn[n * 64 + i] = val;
        }
}

// one (instance, interval): writes g rows, local grad columns, CCS values, 4 partials
void eval_interval(const Ap2Tables& T, int k, const double* V, const double* P, double* g, double* grad,
                   double* jac, double* part, std::vector<double>& tang, std::vector<double>& wn) {
    const Layout& L = T.lay;
    const ColorTabs& ct = T.ct;
    const int d = T.d, NN = d + 1;
    const double* C = T.dcoll.C;
    const double* cst = T.cst.data();
    const double* th = P + L.n_v + AWE_NW + AWE_NCOST;
    const double* cost = P + L.n_v + AWE_NW;
    const double* wts = P + L.n_v;
    const double* vref = P;
    const int base = L.v_int0 + k * L.stride;
    const double* vt = V;
    const double* vx = V + base;
    const double* vu = vx + AWE_NX;
    const double* vxd = vu + AWE_NU;
    const double* vz = vxd + AWE_NX;
    const double* vcoll = vz + AWE_NZ;
    const double* vx1 = vcoll + d * (AWE_NX + AWE_NZ);
    const double tf = vt[1];
    const double h = 1.0 / T.n_k;
    const double inv_h_tf = 1.0 / h / tf;
    const double inv_tf = 1.0 / tf;
    auto toff = [&](int n) { return n == 0 ? 0 : ct.tsize[0] + (n - 1) * ct.tsize[1]; };

    node_values(T, k, V, wn);

    // model, all colours of a node at once
    tang.assign((size_t)T.tang_total + 1, 0.0);
    tang[T.tang_total] = 1.0;
    double gval[8][kGvalStride];
    for (int n = 0; n < NN; ++n) {
        const int kind = n > 0;
        CpuIn in{&wn[n * 64], &ct, kind, n > 0 ? C[n * NN + n] * inv_h_tf : 0.0, inv_tf};
        CpuSink sink{&tang[toff(n)], gval[n], &ct, kind};
        DN gamma(vt[2 + kPhiGamma]);
        for (int c = 0; c < kHalf; ++c) gamma.d[c] = ((ct.seedA[kind][c] >> kDirGamma) & 1ull) ? 1.0 : 0.0;
        awe::ap2_node<DN>(in, gamma, th, cst, sink, n == 0);
    }

    // objective directional derivatives (objective.py:45-544)
    const double psi = vt[2 + kPhiPsi];
    const double w_track = cost[kCostTracking] / cst[AWE_C_NORM_TRACKING];
    const double w_xdot = cost[kCostXdotRegularisation] / cst[AWE_C_NORM_XDOT_REG];
    const double w_ureg = cost[kCostURegularisation] / cst[AWE_C_NORM_U_REG];
    const double w_fict = cost[kCostFictitious] / cst[AWE_C_NORM_FICTITIOUS];
    const double w_theta = cost[kCostThetaRegularisation] / cst[AWE_C_NORM_THETA_REG];
    double dfl[8][64] = {};
    double fnode[8] = {};
    for (int n = 1; n < NN; ++n) {
        const int j = n - 1;
        const double wj = T.dcoll.w[j];
        const double* w = &wn[n * 64];
        const double* rb = vref + base;
        const double* rcx = rb + 2 * AWE_NX + AWE_NU + AWE_NZ + j * (AWE_NX + AWE_NZ);
        const double* ru = rb + AWE_NX;
        const double cxx = C[n * NN + n] * inv_h_tf;
        const double* tp = &tang[toff(n)];
        double trk = 0.0, xdr = 0.0, oth = 0.0;
        double dfd[64] = {};
        for (int dir = 0; dir < 64; ++dir) {
            if (dir < AWE_NX) {
                const double e = w[dir] - rcx[dir], ww = wts[dir] * w_track;
                const double xdv = w[AWE_NX + dir], wx = wts[AWE_NX + dir] * w_xdot;
                trk += ww * (e * e);
                dfd[dir] = wj * (psi * (2.0 * ww * e) + cxx * (2.0 * wx * xdv));
            } else if (dir < 2 * AWE_NX) {
                const double xdv = w[dir], wx = wts[dir] * w_xdot;
                xdr += wx * (xdv * xdv);
                dfd[dir] = wj * (2.0 * wx * xdv);
            } else if (dir < 2 * AWE_NX + AWE_NU) {
                const int i = dir - 2 * AWE_NX;
                const double e = w[dir] - ru[i], wu = wts[dir] * (i < 6 ? w_fict : w_ureg);
                oth += wu * (e * e);
                dfd[dir] = wj * (2.0 * wu * e);
            } else if (dir == kDirZ) {
                const double e = w[dir] - rcx[AWE_NX], ww = wts[dir] * w_track;
                trk += ww * (e * e);
                dfd[dir] = wj * psi * (2.0 * ww * e);
            } else if (dir == kDirDiam) {
                const double e = w[dir] - vref[0], wt = wts[dir] * w_theta;
                oth += wt * (e * e);
                dfd[dir] = wj * (2.0 * wt * e);
            }
        }
        const double bv = gval[n][kRowBeta], pv = gval[n][kRowPower];
        const double cb = cost[kCostBeta] * wj / cst[AWE_C_NORM_BETA];
        const double cp = -cost[kCostPower] * wj / (double)T.n_k;
        dfd[kDirTf] = -2.0 * wj * xdr * inv_tf;
        dfd[kDirPsi] = wj * trk - cp * pv;
        for (int dir = 0; dir < 64; ++dir) {
            if (ct.obj_beta[dir] >= 0) dfd[dir] += (2.0 * cb * bv) * tp[ct.obj_beta[dir]];
            if (ct.obj_power[dir] >= 0) dfd[dir] += ((1.0 - psi) * cp) * tp[ct.obj_power[dir]];
            dfl[n][dir] = dfd[dir];
        }
        fnode[n] = wj * (psi * trk + xdr + oth) + cb * (bv * bv) + (1.0 - psi) * (cp * pv);
    }

    // g rows (shooting, path, collocation, continuity)
    for (int r = 0; r < L.rows; ++r) {
        double val;
        if (r < AWE_N_EQ + AWE_N_INEQ) {
            val = gval[0][r];
        } else if (r < AWE_N_EQ + AWE_N_INEQ + d * AWE_N_EQ) {
            const int q = r - (AWE_N_EQ + AWE_N_INEQ);
            val = gval[1 + q / AWE_N_EQ][q % AWE_N_EQ];
        } else {
            const int i = r - (AWE_N_EQ + AWE_N_INEQ + d * AWE_N_EQ);
            double xf = 0.0;
            for (int rr = 0; rr < NN; ++rr) {
                if (T.dcoll.D[rr] == 0.0) continue;
                const double Xr = (rr == 0) ? vx[i] : vcoll[(rr - 1) * (AWE_NX + AWE_NZ) + i];
                xf += T.dcoll.D[rr] * Xr;
            }
            val = vx1[i] - xf;
        }
        g[k * L.rows + r] = val;
    }
    part[0] = part[1] = part[2] = part[3] = 0.0;
    for (int n = 1; n < NN; ++n) {
        part[0] += fnode[n];
        part[1] += dfl[n][kDirDiam];
        part[2] += dfl[n][kDirTf];
        part[3] += dfl[n][kDirPsi];
    }
    // local gradient columns
    for (int col = 0; col < L.stride; ++col) {
        double gsum = 0.0;
        if (col < AWE_NX) {
            for (int n = 1; n < NN; ++n) gsum += C[n] * inv_h_tf * dfl[n][AWE_NX + col];
        } else if (col < AWE_NX + AWE_NU) {
            for (int n = 1; n < NN; ++n) gsum += dfl[n][2 * AWE_NX + col - AWE_NX];
        } else if (col >= 2 * AWE_NX + AWE_NU + AWE_NZ) {
            const int q = col - (2 * AWE_NX + AWE_NU + AWE_NZ);
            const int r = 1 + q / (AWE_NX + AWE_NZ), e = q % (AWE_NX + AWE_NZ);
            if (e < AWE_NX) {
                gsum = dfl[r][e];
                for (int n = 1; n < NN; ++n)
                    if (n != r) gsum += C[r * NN + n] * inv_h_tf * dfl[n][AWE_NX + e];
            } else {
                gsum = dfl[r][kDirZ];
            }
        }
        grad[base + col] = gsum;
    }
    // CCS values through the gather list
    double scl[64];
    scl[0] = 1.0;
    for (int i = 1; i <= NN * NN; ++i) scl[i] = C[i - 1] * inv_h_tf;
    for (size_t q = 0; q < T.kconst.size(); ++q) scl[1 + NN * NN + q] = T.kconst[q];
    const int* sg = &T.seg[(size_t)k * kSegs * 3];
    const unsigned* gl = &T.glist[T.glist_off[k]];
    for (int s = 0; s < kSegs; ++s) {
        const int g0 = sg[3 * s], len = sg[3 * s + 1], lo = sg[3 * s + 2];
        for (int i = 0; i < len; ++i) {
            const unsigned e = gl[lo + i];
            jac[g0 + i] = scl[e >> 16] * tang[e & 0xffffu];
        }
    }
}

// Hessian of sigma f + lam^T g restricted to one interval: local CCS slots and the interval's
// share of the global-global entries (mirrors ap2_hess_kernel)
void hess_interval(const Ap2Tables& T, const Ap2HessTables& HT, int k, const double* V, const double* P,
                   double sigma, const double* lam, double* H, double* gpart, std::vector<double>& tang,
                   std::vector<double>& wn, std::vector<double>& hd) {
    const Layout& L = T.lay;
    const ColorTabs& ct = T.ct;
    const HessTabs& ht = HT.ht;
    const int d = T.d, NN = d + 1;
    const double* C = T.dcoll.C;
    const double* cst = T.cst.data();
    const double* th = P + L.n_v + AWE_NW + AWE_NCOST;
    const double* cost = P + L.n_v + AWE_NW;
    const double* wts = P + L.n_v;
    const double* vref = P;
    const int base = L.v_int0 + k * L.stride;
    const double* vt = V;
    const double tf = vt[1];
    const double h = 1.0 / T.n_k;
    const double inv_h_tf = 1.0 / h / tf;
    const double inv_tf = 1.0 / tf;
    const double psi = vt[2 + kPhiPsi];
    auto toff = [&](int n) { return n == 0 ? 0 : ct.tsize[0] + (n - 1) * ct.tsize[1]; };
    node_values(T, k, V, wn);

    // first-order pass (tangents of the beta / power rows and of the xdot directions)
    tang.assign((size_t)T.tang_total + 1, 0.0);
    double gval[8][kGvalStride];
    for (int n = 0; n < NN; ++n) {
        const int kind = n > 0;
        CpuIn in{&wn[n * 64], &ct, kind, n > 0 ? C[n * NN + n] * inv_h_tf : 0.0, inv_tf};
        CpuSink sink{&tang[toff(n)], gval[n], &ct, kind};
        DN gamma(vt[2 + kPhiGamma]);
        for (int c = 0; c < kHalf; ++c) gamma.d[c] = ((ct.seedA[kind][c] >> kDirGamma) & 1ull) ? 1.0 : 0.0;
        awe::ap2_node<DN>(in, gamma, th, cst, sink, n == 0);
    }
    const double w_track = cost[kCostTracking] / cst[AWE_C_NORM_TRACKING];
    const double w_xdot = cost[kCostXdotRegularisation] / cst[AWE_C_NORM_XDOT_REG];
    const double w_ureg = cost[kCostURegularisation] / cst[AWE_C_NORM_U_REG];
    const double w_fict = cost[kCostFictitious] / cst[AWE_C_NORM_FICTITIOUS];
    const double w_theta = cost[kCostThetaRegularisation] / cst[AWE_C_NORM_THETA_REG];

    // row weights mu per node
    double mu[8][kHRows + 1];
    for (int n = 0; n < NN; ++n) {
        for (int r = 0; r <= kHRows; ++r) mu[n][r] = 0.0;
        if (n == 0) {
            for (int r = 0; r < kRowPower; ++r) mu[n][r] = lam[k * L.rows + r];
        } else {
            const double wj = T.dcoll.w[n - 1];
            for (int r = 0; r < AWE_N_EQ; ++r) mu[n][r] = lam[k * L.rows + AWE_N_EQ + AWE_N_INEQ + (n - 1) * AWE_N_EQ + r];
            const double cb = cost[kCostBeta] * wj / cst[AWE_C_NORM_BETA];
            const double cp = -cost[kCostPower] * wj / (double)T.n_k;
            mu[n][kRowPower] = sigma * (1.0 - psi) * cp;
            mu[n][kRowBeta] = sigma * 2.0 * cb * gval[n][kRowBeta];
        }
    }
    // direction-pair Hessian of every node: colour-pair hyper-dual passes
    const int hoff1 = ht.npairs[0];
    hd.assign((size_t)ht.npairs[0] + d * ht.npairs[1], 0.0);
    auto hoff = [&](int n) { return n == 0 ? 0 : hoff1 + (n - 1) * ht.npairs[1]; };
    for (int n = 0; n < NN; ++n) {
        const int kind = n > 0;
        for (int t = 0; t < ht.ntask[kind]; ++t) {
            const int task = HT.tasks[ht.task_off[kind] + t];
            const int c1 = task & 0xff, c2 = task >> 8;
            CpuHIn in{&wn[n * 64], &ct, kind, c1, c2, n > 0 ? C[n * NN + n] * inv_h_tf : 0.0, inv_tf};
            CpuHSink sink{&hd[hoff(n)], &ht, mu[n], kind, c1, c2};
            const double g1 = ((ct.seedA[kind][c1] >> kDirGamma) & 1ull) ? 1.0 : 0.0;
            const double g2 = ((ct.seedA[kind][c2] >> kDirGamma) & 1ull) ? 1.0 : 0.0;
            awe::ap2_node<awe::HDual>(in, awe::HDual(vt[2 + kPhiGamma], g1, g2, 0.0), th, cst, sink, n == 0);
        }
    }
    // objective terms at the Radau nodes, in direction space; map terms G
    double G[8][AWE_NX] = {}, GT[8] = {};
    for (int n = 1; n < NN; ++n) {
        const int j = n - 1;
        const double wj = T.dcoll.w[j];
        const double* w = &wn[n * 64];
        const double* rb = vref + base;
        const double* rcx = rb + 2 * AWE_NX + AWE_NU + AWE_NZ + j * (AWE_NX + AWE_NZ);
        const double cxx = C[n * NN + n] * inv_h_tf;
        const double* tp = &tang[toff(n)];
        double* hn = &hd[hoff(n)];
        auto addp = [&](int p, int q, double v) { hn[ht.pidx[1][p][q]] += sigma * v; };
        const double cb = cost[kCostBeta] * wj / cst[AWE_C_NORM_BETA];
        const double cp = -cost[kCostPower] * wj / (double)T.n_k;
        double tfsum = 0.0;
        for (int i = 0; i < AWE_NX; ++i) {
            const double ai = wts[i] * w_track, bi = wts[AWE_NX + i] * w_xdot, xd = w[AWE_NX + i];
            addp(i, i, 2.0 * wj * psi * ai + cxx * cxx * 2.0 * wj * bi);
            addp(i, AWE_NX + i, cxx * 2.0 * wj * bi);
            addp(i, kDirTf, cxx * (-xd * inv_tf) * 2.0 * wj * bi);
            addp(AWE_NX + i, AWE_NX + i, 2.0 * wj * bi);
            addp(AWE_NX + i, kDirTf, (-xd * inv_tf) * 2.0 * wj * bi);
            addp(i, kDirPsi, 2.0 * wj * ai * (w[i] - rcx[i]));
            tfsum += (xd * inv_tf) * (xd * inv_tf) * 2.0 * wj * bi;
        }
        addp(kDirTf, kDirTf, tfsum);
        for (int i = 0; i < AWE_NU; ++i)
            addp(2 * AWE_NX + i, 2 * AWE_NX + i, 2.0 * wj * wts[2 * AWE_NX + i] * (i < 6 ? w_fict : w_ureg));
        {
            const double az = wts[kDirZ] * w_track;
            addp(kDirZ, kDirZ, 2.0 * wj * psi * az);
            addp(kDirZ, kDirPsi, 2.0 * wj * az * (w[kDirZ] - rcx[AWE_NX]));
            addp(kDirDiam, kDirDiam, 2.0 * wj * wts[kDirDiam] * w_theta);
        }
        for (int p = 0; p <= kDirGamma; ++p) {
            if (ct.obj_power[p] >= 0) addp(p, kDirPsi, -cp * tp[ct.obj_power[p]]);
            if (ct.obj_beta[p] < 0) continue;
            for (int q = p; q <= kDirGamma; ++q)
                if (ct.obj_beta[q] >= 0) addp(p, q, 2.0 * cb * tp[ct.obj_beta[p]] * tp[ct.obj_beta[q]]);
        }
        // gradient of the node Lagrangian w.r.t. xdot_i (rows + objective)
        for (int i = 0; i < AWE_NX; ++i) {
            const int dir = AWE_NX + i, c = ct.dcolor[1][dir];
            double gi = sigma * wj * 2.0 * wts[dir] * w_xdot * w[dir];
            if (c >= 0) {
                const unsigned long long m = ct.dmask[1][dir], cm = ct.cmask[1][c];
                for (int r = 0; r < kHRows; ++r)
                    if ((m >> r) & 1ull) gi += mu[n][r] * tp[ct.off[1][c] + __builtin_popcountll(cm & ((1ull << r) - 1ull))];
            }
            G[n][i] = gi;
            GT[n] += gi * 2.0 * w[dir] * inv_tf * inv_tf;
        }
    }
    // V-space entries
    double scl[64];
    scl[0] = 1.0;
    for (int i = 1; i <= NN * NN; ++i) scl[i] = C[i - 1] * inv_h_tf;
    const int ng = (int)HT.gslot.size();
    const int nloc = HT.nslot[k];
    for (int e = 0; e < nloc + ng; ++e) {
        const int ei = HT.ent_off[k] + e;
        double v = 0.0;
        for (int t = HT.term_off[ei]; t < HT.term_off[ei + 1]; ++t) {
            const unsigned term = HT.terms[t];
            const int type = term >> 30, n = (term >> 27) & 7;
            if (type == kHTypeA) {
                v += scl[(term >> 7) & 127] * scl[term & 127] * hd[hoff(n) + ((term >> 14) & 8191)];
            } else if (type == kHTypeB) {
                const int i = (term >> 22) & 31, r = (term >> 19) & 7;
                v += G[n][i] * (-C[r * NN + n] * inv_h_tf * inv_tf);
            } else {
                v += GT[n];
            }
        }
        if (e < nloc) H[HT.slot0[k] + e] = v;
        else gpart[e - nloc] = v;
    }
}

void finalize(const Ap2Tables& T, const double* V, const double* P, const double* part, double* f,
              double* g, double* grad) {
    const Layout& L = T.lay;
    const double* cost = P + L.n_v + AWE_NW;
    const double* vref = P;
    double s[kNPartial] = {0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < T.n_k; ++k)
        for (int c = 0; c < kNPartial; ++c) s[c] += part[k * kNPartial + c];
    const double tf = V[1], tf_ref = vref[1];
    const int last = L.v_int0 + (T.n_k - 1) * L.stride + 2 * AWE_NX + AWE_NU + AWE_NZ +
                     (T.d - 1) * (AWE_NX + AWE_NZ);
    for (int q = 0; q < AWE_NX; ++q) {
        const int i = kPeriodicOrder[q];
        g[T.n_k * L.rows + q] = V[L.v_int0 + i] - V[last + i];
    }
    const int phi_cost_map[AWE_NPHI] = {3, 6, 4, 5, 7, 8, 9};
    double fh = 0.0;
    for (int i = 0; i < AWE_NPHI; ++i) fh += cost[phi_cost_map[i]] * V[AWE_NTH + i];
    *f = s[0] + cost[kCostTf] * (tf - tf_ref) * (tf - tf_ref) + fh;
    grad[0] = s[1];
    grad[1] = s[2] + cost[kCostTf] * 2.0 * (tf - tf_ref);
    for (int i = 0; i < AWE_NPHI; ++i) grad[AWE_NTH + i] = cost[phi_cost_map[i]] + (i == kPhiPsi ? s[3] : 0.0);
    for (int i = 0; i < AWE_NXI; ++i) grad[AWE_NTH + AWE_NPHI + i] = 0.0;
    for (int i = 0; i < AWE_NX; ++i) grad[L.v_int0 + T.n_k * L.stride + i] = 0.0;
}

// one node of the shared model with a dense Jacobian: direction c of the pass seeds input base + c
struct NodeIn {
    const double* w;
    int base;
    DN operator()(int i) const {
        DN r(w[i]);
        if (i >= base && i < base + kHalf) r.d[i - base] = 1.0;
        return r;
    }
};

struct NodeSinkDense {
    double* rows;   // [kGvalStride]
    double* jac;    // [kGvalStride][AWE_NW], row-major
    int base;
    void emit(int r, const DN& v) {
        rows[r] = v.v;
        for (int c = 0; c < kHalf && base + c < AWE_NW; ++c) jac[r * AWE_NW + base + c] = v.d[c];
    }
    void eq_row(int r, const DN& v) { emit(r, v); }
    void ineq_row(int r, const DN& v) { emit(AWE_N_EQ + r, v); }
    void power(const DN& v) { emit(kRowPower, v); }
    void beta(const DN& v) { emit(kRowBeta, v); }
};

}  // namespace

extern "C" {

const char* ap2cpu_last_error(void) { return g_err.c_str(); }

// Model rows of one node (24 eq, 9 ineq, power, beta; kGvalStride doubles) and their Jacobian
// w.r.t. the 59 scaled node variables, for model-level known-answer tests (integration of the
// DAE).  theta0 in the flat AWE_TH_* layout; the phi-gamma embedding factor is `gamma`.
int ap2cpu_node(void* hv, const double* w_sc, const double* theta0, double gamma, double* rows,
                double* jac) {
    const Ap2Tables& T = static_cast<Handle*>(hv)->t;
    const double* cst = T.cst.data();
    std::memset(jac, 0, sizeof(double) * kGvalStride * AWE_NW);
    for (int base = 0; base < AWE_NW; base += kHalf) {
        NodeIn in{w_sc, base};
        NodeSinkDense sink{rows, jac, base};
        awe::ap2_node<DN>(in, DN(gamma), theta0, cst, sink, true);
    }
    return AWE_OK;
}

int ap2cpu_create(int n_k, int d, const double* consts, int n_consts, void** out) {
    if (!out || !consts) { g_err = "null argument"; return AWE_ERR_ARG; }
    if (d < 1 || d > 7) { g_err = "bad d"; return AWE_ERR_ARG; }
    auto* h = new Handle();
    int rc = build_ap2_tables(n_k, d, consts, n_consts, h->t, g_err);
    if (rc) { delete h; return rc; }
    *out = h;
    return AWE_OK;
}

int ap2cpu_sizes(void* hv, int* n_v, int* n_g, int* n_p, int* nnz) {
    const Ap2Tables& T = static_cast<Handle*>(hv)->t;
    *n_v = T.lay.n_v; *n_g = T.lay.n_g; *n_p = T.lay.n_p; *nnz = T.nnz;
    return AWE_OK;
}

int ap2cpu_sparsity(void* hv, int* colind, int* row) {
    const Ap2Tables& T = static_cast<Handle*>(hv)->t;
    std::memcpy(colind, T.colind.data(), sizeof(int) * T.colind.size());
    std::memcpy(row, T.row.data(), sizeof(int) * T.row.size());
    return AWE_OK;
}

// batch instances, instance-major arrays as in awe_eval_nlp; nthreads <= 0: OpenMP default
int ap2cpu_eval_nlp(void* hv, int batch, const double* V, const double* P, double* f, double* g,
                    double* grad, double* jac, int nthreads) {
    const Ap2Tables& T = static_cast<Handle*>(hv)->t;
    const Layout& L = T.lay;
    std::vector<double> part((size_t)batch * T.n_k * kNPartial);
    const int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#pragma omp parallel num_threads(nt)
    {
        std::vector<double> tang, wn;
#pragma omp for schedule(static)
        for (long t = 0; t < (long)batch * T.n_k; ++t) {
            const int b = (int)(t / T.n_k), k = (int)(t % T.n_k);
            eval_interval(T, k, V + (size_t)b * L.n_v, P + (size_t)b * L.n_p, g + (size_t)b * L.n_g,
                          grad + (size_t)b * L.n_v, jac + (size_t)b * T.nnz,
                          &part[((size_t)b * T.n_k + k) * kNPartial], tang, wn);
        }
#pragma omp for schedule(static)
        for (int b = 0; b < batch; ++b)
            finalize(T, V + (size_t)b * L.n_v, P + (size_t)b * L.n_p, &part[(size_t)b * T.n_k * kNPartial],
                     f + b, g + (size_t)b * L.n_g, grad + (size_t)b * L.n_v);
    }
    return AWE_OK;
}

void ap2cpu_destroy(void* hv) { delete static_cast<Handle*>(hv); }

int ap2cpu_hess_init(void* hv, int* nnz) {
    Handle* h = static_cast<Handle*>(hv);
    if (h->ht.nnz == 0) {
        int rc = build_hess_tables(h->t, h->ht, g_err);
        if (rc) return rc;
    }
    *nnz = h->ht.nnz;
    return AWE_OK;
}

int ap2cpu_hess_sparsity(void* hv, int* colind, int* row) {
    const Ap2HessTables& H = static_cast<Handle*>(hv)->ht;
    std::memcpy(colind, H.colind.data(), sizeof(int) * H.colind.size());
    std::memcpy(row, H.row.data(), sizeof(int) * H.row.size());
    return AWE_OK;
}

// upper-triangular CCS values of the Hessian of sigma f + lam^T g for each instance
int ap2cpu_eval_hess(void* hv, int batch, const double* V, const double* P, const double* sigma,
                     const double* lam, double* H, int nthreads) {
    Handle* hd = static_cast<Handle*>(hv);
    const Ap2Tables& T = hd->t;
    const Ap2HessTables& HT = hd->ht;
    if (HT.nnz == 0) { g_err = "call ap2cpu_hess_init first"; return AWE_ERR_ARG; }
    const Layout& L = T.lay;
    const int ng = (int)HT.gslot.size();
    std::vector<double> gpart((size_t)batch * T.n_k * ng);
    const int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#pragma omp parallel num_threads(nt)
    {
        std::vector<double> tang, wn, hdir;
#pragma omp for schedule(dynamic)
        for (long t = 0; t < (long)batch * T.n_k; ++t) {
            const int b = (int)(t / T.n_k), k = (int)(t % T.n_k);
            hess_interval(T, HT, k, V + (size_t)b * L.n_v, P + (size_t)b * L.n_p, sigma[b],
                          lam + (size_t)b * L.n_g, H + (size_t)b * HT.nnz, &gpart[((size_t)b * T.n_k + k) * ng],
                          tang, wn, hdir);
        }
#pragma omp for schedule(static)
        for (int b = 0; b < batch; ++b) {
            const double* P_b = P + (size_t)b * L.n_p;
            const double c_tf = P_b[L.n_v + AWE_NW + kCostTf];
            const int itf = L.theta(1);
            for (int g = 0; g < ng; ++g) {
                double v = 0.0;
                for (int k = 0; k < T.n_k; ++k) v += gpart[((size_t)b * T.n_k + k) * ng + g];
                const int slot = HT.gslot[g];
                if (HT.row[slot] == itf && slot >= HT.colind[itf] && slot < HT.colind[itf + 1])
                    v += sigma[b] * 2.0 * c_tf;
                H[(size_t)b * HT.nnz + slot] = v;
            }
        }
    }
    return AWE_OK;
}

}  // extern "C"
