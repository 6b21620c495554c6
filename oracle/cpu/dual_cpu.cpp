// CPU port of the dual-kite evaluator (awebox_amd/csrc/awedual.hip) -- TEST AND BASELINE
// INFRASTRUCTURE, never used by the product.
//
// The same algorithm on the host: the shared node model (dual_model.hpp) and host tables
// (dual_tables.hpp: colouring, CCS pattern, gather list), compressed forward mode with one Dual
// evaluation per (node, colour), the objective directional derivatives, the gradient assembly
// through the collocation polynomial and the gather-list J values; OpenMP over (instance,
// interval).  Two uses:
//   * tests compare it with the independent oracle (oracle/multikite_oracle.py), so the kernel's
//     colouring / gather / objective logic is exercised without a GPU;
//   * bench.py times it as the config-3 CPU baseline (kind "port").
// Sub-models are evaluated inline (no preaccumulation), so results agree with the GPU to rounding.
#include <omp.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "dual_model.hpp"
#include "dual_tables.hpp"

namespace {

using namespace dlt;
thread_local std::string g_err;

// objective constants (kNPart, kCost*, kPhiCost, kPhiPsi): dual_tables.hpp

struct Handle {
    Tables t;
    std::vector<double> cst;
};

struct In {
    const double* w;
    const int8_t* col;
    int lane;
    double cxx, tfl;
    awe::Dual operator()(int i) const {
        double t = (col[i] == lane) ? 1.0 : 0.0;
        if (i >= ADL_NX && i < 2 * ADL_NX) {
            if (col[i - ADL_NX] == lane) t += cxx;
            t += tfl * w[i];
        }
        return awe::Dual(w[i], t);
    }
};

struct Sink {
    double* tp;
    double* gv;
    Mask m;
    bool c0;
    void emit(int r, const awe::Dual& v) {
        if (c0) gv[r] = v.v;
        if (m.has(r)) tp[m.below(r)] = v.d;
    }
    void eq_row(int r, const awe::Dual& v) { emit(r, v); }
    void ineq_row(int r, const awe::Dual& v) { emit(ADL_N_EQ + r, v); }
    void power(const awe::Dual& v) { emit(kRowPower, v); }
    void beta(int k, const awe::Dual& v) { emit(kRowBeta0 + k, v); }
};

double time_period(const double* V, const Layout& L) {
    if (!L.single) return V[1];
    return V[1] * L.nk_reelout / L.n_k + V[2] * (L.n_k - L.nk_reelout) / L.n_k;
}

void interval(const Handle& h, const double* V, const double* P, int k, double* g, double* grad, double* jac,
              double* part) {
    const Tables& T = h.t;
    const Layout& L = T.lay;
    const ColorTabs& ct = T.ct;
    const double* cst = h.cst.data();
    const int D = L.d, NN = D + 1;
    const int STRIDE = L.stride, nthv = L.n_thv;
    const int base = L.v_int0 + k * STRIDE;
    std::vector<double> vloc(ADL_NTHV + 7 + STRIDE + ADL_NX, 0.0), rloc(ADL_NTHV + STRIDE, 0.0);
    for (int i = 0; i < nthv; ++i) { vloc[i] = V[i]; rloc[i] = P[i]; }
    for (int i = 0; i < 7; ++i) vloc[ADL_NTHV + i] = V[nthv + i];
    for (int i = 0; i < STRIDE + ADL_NX; ++i) vloc[ADL_NTHV + 7 + i] = V[base + i];
    for (int i = 0; i < STRIDE; ++i) rloc[ADL_NTHV + i] = P[base + i];
    const double* wts = P + L.n_v;
    const double* cost = P + L.n_v + ADL_NW;
    const double* th = P + L.n_v + ADL_NW + 20;
    const double psi = vloc[ADL_NTHV + kPhiPsi];
    double wef[ADL_NW], wtr[ADL_NW];
    for (int i = 0; i < ADL_NW; ++i) {
        int ci;
        double nrm;
        bool track = false;
        if (i < ADL_NX || (i >= 119 && i < 122)) { ci = kCostTracking; nrm = cst[ADL_C_NORM_TRACKING]; track = true; }
        else if (i < 2 * ADL_NX) { ci = kCostXdotRegularisation; nrm = cst[ADL_C_NORM_XDOT_REG]; }
        else if (i < 119) {
            const int u = i - 100;
            const bool fict = (u % 9) < 6 && u < 18;
            ci = fict ? kCostFictitious : kCostURegularisation;
            nrm = cst[fict ? ADL_C_NORM_FICTITIOUS : ADL_C_NORM_U_REG];
        } else { ci = kCostThetaRegularisation; nrm = cst[ADL_C_NORM_THETA_REG]; }
        double we = wts[i] * cost[ci] / nrm;
        if (i == awe::dl::kTf) we = 0.0;
        wef[i] = we;
        wtr[i] = track ? psi * we : we;
    }
    const int tfi = L.single ? (k < L.nk_reelout ? 1 : 2) : 1;
    const double tf = vloc[tfi];
    const double ihtf = (double)L.n_k / tf;
    const auto& C = T.coll.C;   // C[j][r] = l_j'(tau_r)
    const double* xk = vloc.data() + ADL_NTHV + 7;
    const double* uk = xk + ADL_NX;
    const double* xdk = uk + ADL_NU;
    const double* zk = xdk + ADL_NX;
    const double* coll = zk + ADL_NZ;
    const double* xk1 = coll + D * (ADL_NX + ADL_NZ);
    auto Xv = [&](int r, int i) { return r == 0 ? xk[i] : coll[(r - 1) * (ADL_NX + ADL_NZ) + i]; };
    auto node_theta = [&](const double* tv, int t) { return t == 1 ? tv[tfi] : (L.single ? tv[t == 0 ? 0 : t + 1] : tv[t]); };
    std::vector<double> wn(NN * 128, 0.0), rn(D * ADL_NW, 0.0);
    for (int n = 0; n < NN; ++n)
        for (int i = 0; i < 127; ++i) {
            double val = 0.0;
            if (i < ADL_NX) val = Xv(n, i);
            else if (i < 2 * ADL_NX) {
                if (n == 0) val = xdk[i - ADL_NX];
                else {
                    double s = 0.0;
                    for (int r = 0; r < NN; ++r) s += C[r][n] * Xv(r, i - ADL_NX);
                    val = s * ihtf;
                }
            } else if (i < 2 * ADL_NX + ADL_NU) val = uk[i - 2 * ADL_NX];
            else if (i < 2 * ADL_NX + ADL_NU + ADL_NZ) {
                const int z = i - (2 * ADL_NX + ADL_NU);
                val = n == 0 ? zk[z] : coll[(n - 1) * (ADL_NX + ADL_NZ) + ADL_NX + z];
            } else if (i < ADL_NW) val = node_theta(vloc.data(), i - (2 * ADL_NX + ADL_NU + ADL_NZ));
            else val = vloc[ADL_NTHV];
            wn[n * 128 + i] = val;
        }
    for (int j = 0; j < D; ++j)
        for (int i = 0; i < ADL_NW; ++i) {
            const double* rl = rloc.data() + ADL_NTHV;
            double val;
            if (i < ADL_NX) val = rl[2 * ADL_NX + ADL_NU + ADL_NZ + j * (ADL_NX + ADL_NZ) + i];
            else if (i < 2 * ADL_NX) val = 0.0;
            else if (i < 2 * ADL_NX + ADL_NU) val = rl[ADL_NX + (i - 2 * ADL_NX)];
            else if (i < 2 * ADL_NX + ADL_NU + ADL_NZ)
                val = rl[2 * ADL_NX + ADL_NU + ADL_NZ + j * (ADL_NX + ADL_NZ) + ADL_NX + (i - (2 * ADL_NX + ADL_NU))];
            else val = node_theta(rloc.data(), i - (2 * ADL_NX + ADL_NU + ADL_NZ));
            rn[j * ADL_NW + i] = val;
        }
    // ---- model pass: one Dual evaluation per (node, colour) --------------------------------
    std::vector<double> tang(T.tang_total, 0.0), gval(NN * kGvalStride, 0.0);
    for (int n = 0; n < NN; ++n) {
        const int kind = n > 0;
        const int toff = n == 0 ? 0 : ct.tsize[0] + (n - 1) * ct.tsize[1];
        for (int c = 0; c < ct.ncol[kind]; ++c) {
            In in{&wn[n * 128], ct.col[kind], c, n > 0 ? C[n][n] * ihtf : 0.0,
                  (n > 0 && ct.col[1][awe::dl::kTf] == c) ? -1.0 / tf : 0.0};
            Mask m;
            m.lo = ct.cm_lo[kind][c];
            m.hi = ct.cm_hi[kind][c];
            Sink sink{&tang[toff + ct.off[kind][c]], &gval[n * kGvalStride], m, c == 0};
            awe::dual_node<awe::Dual>(in, awe::Dual(wn[n * 128 + 126], ct.col[kind][126] == c ? 1.0 : 0.0), th, cst,
                                      sink, n == 0);
        }
    }
    // ---- objective directional derivatives -------------------------------------------------------
    const double Tp = time_period(V, L);
    const double cb = cost[kCostBeta] / cst[ADL_C_NORM_BETA];
    std::vector<double> obj(D * 128, 0.0), fterm(D * 128, 0.0);
    for (int j = 0; j < D; ++j) {
        const int n = j + 1;
        const double wq = T.coll.w[j];
        const double* wv = &wn[n * 128];
        const double* rv = &rn[j * ADL_NW];
        const double cxx = C[n][n] * ihtf;
        const int toff = ct.tsize[0] + (n - 1) * ct.tsize[1];
        for (int dir = 0; dir < 127; ++dir) {
            double acc = 0.0;
            if (dir < ADL_NX) acc = 2.0 * wq * (wtr[dir] * (wv[dir] - rv[dir]) + wtr[ADL_NX + dir] * wv[ADL_NX + dir] * cxx);
            else if (dir < 2 * ADL_NX) acc = 2.0 * wq * wtr[dir] * wv[dir];
            else if (dir == awe::dl::kTf) {
                for (int i = 0; i < ADL_NX; ++i) acc -= 2.0 * wq * wtr[ADL_NX + i] * wv[ADL_NX + i] * wv[ADL_NX + i] / tf;
            } else if (dir < ADL_NW) acc = 2.0 * wq * wtr[dir] * (wv[dir] - rv[dir]);
            if (dir < ADL_NW) {
                const double e = wv[dir] - rv[dir];
                fterm[j * 128 + dir] = wq * wef[dir] * e * e;
            }
            const int tp = ct.obj_tang[dir][0];
            if (tp >= 0) acc += (1.0 - psi) * (-cost[kCostPower]) * (tf / L.n_k) * wq / Tp * tang[toff + tp];
            for (int kk = 0; kk < 2; ++kk) {
                const int tb = ct.obj_tang[dir][1 + kk];
                if (tb >= 0) acc += 2.0 * wq * cb * gval[n * kGvalStride + kRowBeta0 + kk] * tang[toff + tb];
            }
            obj[j * 128 + dir] = acc;
        }
    }
    {
        double tr = 0.0, ot = 0.0, A = 0.0, pd[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j = 0; j < D; ++j) {
            const int n = j + 1;
            const double wq = T.coll.w[j];
            for (int i = 0; i < ADL_NW; ++i) {
                const bool track = i < ADL_NX || (i >= 119 && i < 122);
                if (track) tr += fterm[j * 128 + i]; else ot += fterm[j * 128 + i];
            }
            const double* gv = &gval[n * kGvalStride];
            ot += wq * cb * (gv[kRowBeta0] * gv[kRowBeta0] + gv[kRowBeta0 + 1] * gv[kRowBeta0 + 1]);
            A += wq * gv[kRowPower] / L.n_k;
            for (int q = 0; q < 4; ++q) pd[q] += obj[j * 128 + 122 + q];
        }
        part[0] = tr; part[1] = ot; part[2] = A;
        for (int q = 0; q < 4; ++q) part[3 + q] = pd[q];
        part[7] = 0.0;
    }
    // ---- gradient of the interval's columns -------------------------------------------------------
    for (int c = 0; c < STRIDE; ++c) {
        double gr = 0.0;
        if (c < ADL_NX) {
            for (int m = 1; m < NN; ++m) gr += obj[(m - 1) * 128 + ADL_NX + c] * C[0][m] * ihtf;
        } else if (c < ADL_NX + ADL_NU) {
            for (int m = 1; m < NN; ++m) gr += obj[(m - 1) * 128 + 2 * ADL_NX + (c - ADL_NX)];
        } else if (c >= 2 * ADL_NX + ADL_NU + ADL_NZ) {
            const int q = c - (2 * ADL_NX + ADL_NU + ADL_NZ);
            const int j = q / (ADL_NX + ADL_NZ), e = q % (ADL_NX + ADL_NZ), n = j + 1;
            if (e < ADL_NX) {
                gr = obj[j * 128 + e];
                for (int m = 1; m < NN; ++m)
                    if (m != n) gr += obj[(m - 1) * 128 + ADL_NX + e] * C[n][m] * ihtf;
            } else gr = obj[j * 128 + 2 * ADL_NX + ADL_NU + (e - ADL_NX)];
        }
        grad[base + c] = gr;
    }
    if (k == L.n_k - 1)
        for (int c = 0; c < ADL_NX; ++c) grad[base + STRIDE + c] = 0.0;
    // ---- g rows -----------------------------------------------------------------------------------
    const int ROWS = L.rows;
    for (int r = 0; r < ROWS; ++r) {
        double val;
        if (r < ADL_N_EQ + ADL_N_INEQ) val = gval[r];
        else if (r < ADL_N_EQ + ADL_N_INEQ + D * ADL_N_EQ) {
            const int q = r - (ADL_N_EQ + ADL_N_INEQ);
            val = gval[(1 + q / ADL_N_EQ) * kGvalStride + q % ADL_N_EQ];
        } else {
            const int i = r - (ADL_N_EQ + ADL_N_INEQ + D * ADL_N_EQ);
            double s = 0.0;
            for (int rr = 0; rr < NN; ++rr) s += T.coll.D[rr] * Xv(rr, i);
            val = xk1[i] - s;
        }
        g[k * ROWS + r] = val;
    }
    // ---- J_g values --------------------------------------------------------------------------------
    for (int e = T.goff[k]; e < T.goff[k + 1]; ++e) {
        const uint32_t cd = T.gcode[e];
        const uint32_t kind = cd >> 29;
        const int rr = (cd >> 25) & 15, n = (cd >> 21) & 15, idx = cd & ((1u << 21) - 1u);
        double val;
        if (kind == kKindTang) val = tang[idx];
        else if (kind == kKindTangPoly) val = tang[idx] * (C[rr][n] * ihtf);
        else val = T.kconst[idx];
        jac[T.gslot[e]] = val;
    }
}

void finalize(const Handle& h, const double* V, const double* P, const double* part, double* f, double* g,
              double* grad) {
    const Layout& L = h.t.lay;
    const double* cst = h.cst.data();
    const double* cost = P + L.n_v + ADL_NW;
    const int nthv = L.n_thv;
    double tr = 0.0, ot = 0.0, e_end = 0.0, A0 = 0.0, A1 = 0.0, pdt = 0.0, pls = 0.0, pds = 0.0, ptf0 = 0.0, ptf1 = 0.0;
    for (int k = 0; k < L.n_k; ++k) {
        const double* q = part + (size_t)k * kNPart;
        const bool ph1 = L.single && k >= L.nk_reelout;
        tr += q[0];
        ot += q[1];
        e_end += V[ph1 ? 2 : 1] * q[2];
        if (ph1) { A1 += q[2]; ptf1 += q[4]; } else { A0 += q[2]; ptf0 += q[4]; }
        pdt += q[3]; pls += q[5]; pds += q[6];
    }
    const double T = time_period(V, L), Tref = time_period(P, L);
    const double psi = V[nthv + kPhiPsi];
    const double cp = cost[kCostPower], ctf = cost[kCostTf];
    const double f_power = -cp * e_end / T;
    double fv = psi * tr + (1.0 - psi) * f_power + ot + ctf * (T - Tref) * (T - Tref);
    for (int i = 0; i < 7; ++i) fv += cost[kPhiCost[i]] * V[nthv + i];
    *f = fv;
    const double n0 = L.single ? (double)L.nk_reelout / L.n_k : 1.0, n1 = L.single ? (double)(L.n_k - L.nk_reelout) / L.n_k : 0.0;
    grad[0] = pdt;
    grad[1] = ptf0 + (1.0 - psi) * (-cp) * (A0 * T - e_end * n0) / (T * T) + 2.0 * ctf * (T - Tref) * n0;
    if (L.single) {
        grad[2] = ptf1 + (1.0 - psi) * (-cp) * (A1 * T - e_end * n1) / (T * T) + 2.0 * ctf * (T - Tref) * n1;
        grad[3] = pls;
        grad[4] = pds;
    } else {
        grad[2] = pls;
        grad[3] = pds;
    }
    for (int i = 0; i < 7; ++i) grad[nthv + i] = cost[kPhiCost[i]] + (i == kPhiPsi ? tr - f_power : 0.0);
    grad[nthv + 7] = grad[nthv + 8] = 0.0;
    if (L.single) {
        const double frac = cst[ADL_C_PHASE_FIX_REELOUT];
        g[L.g_tf()] = (T - cst[ADL_C_TF_UB]) / frac;
        g[L.g_tf() + 1] = (cst[ADL_C_TF_LB] - T) / frac;
    }
    static const int kOrder[ADL_NX] = {24, 25, 26, 45, 46, 47, 49, 3, 4, 5, 9, 10, 11, 30, 31, 32, 48,
                                       12, 13, 14, 33, 34, 35, 0, 1, 2, 6, 7, 8, 27, 28, 29,
                                       15, 16, 17, 18, 19, 20, 21, 22, 23, 36, 37, 38, 39, 40, 41, 42, 43, 44};
    const int x0 = L.x(0, 0), xT = L.coll_x(L.n_k - 1, L.d - 1, 0);
    for (int i = 0; i < ADL_NX; ++i) g[L.g_periodic() + i] = V[x0 + kOrder[i]] - V[xT + kOrder[i]];
}

}  // namespace

extern "C" {

const char* dualcpu_last_error(void) { return g_err.c_str(); }

int dualcpu_create(int n_k, int d, const double* consts, int n_consts, void** out) {
    auto* h = new Handle();
    if (build_tables(n_k, d, consts, n_consts, h->t, g_err)) {
        delete h;
        return 1;
    }
    h->cst.assign(consts, consts + n_consts);
    *out = h;
    return 0;
}

int dualcpu_sizes(void* hv, int* n_v, int* n_g, int* n_p, int* nnz) {
    const Handle* h = (const Handle*)hv;
    *n_v = h->t.lay.n_v; *n_g = h->t.lay.n_g; *n_p = h->t.lay.n_p; *nnz = (int)h->t.row.size();
    return 0;
}

int dualcpu_sparsity(void* hv, int* colind, int* row) {
    const Handle* h = (const Handle*)hv;
    std::memcpy(colind, h->t.colind.data(), sizeof(int) * h->t.colind.size());
    std::memcpy(row, h->t.row.data(), sizeof(int) * h->t.row.size());
    return 0;
}

int dualcpu_eval_nlp(void* hv, int batch, const double* V, const double* P, double* f, double* g, double* grad,
                     double* jac, int threads) {
    const Handle* h = (const Handle*)hv;
    const Layout& L = h->t.lay;
    const size_t nnz = h->t.row.size();
    std::vector<double> part((size_t)batch * L.n_k * kNPart);
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for collapse(2) schedule(dynamic, 1)
    for (int b = 0; b < batch; ++b)
        for (int k = 0; k < L.n_k; ++k)
            interval(*h, V + (size_t)b * L.n_v, P + (size_t)b * L.n_p, k, g + (size_t)b * L.n_g, grad + (size_t)b * L.n_v,
                     jac + (size_t)b * nnz, part.data() + ((size_t)b * L.n_k + k) * kNPart);
    for (int b = 0; b < batch; ++b)
        finalize(*h, V + (size_t)b * L.n_v, P + (size_t)b * L.n_p, part.data() + (size_t)b * L.n_k * kNPart, f + b,
                 g + (size_t)b * L.n_g, grad + (size_t)b * L.n_v);
    return 0;
}

void dualcpu_destroy(void* hv) { delete (Handle*)hv; }

}  // extern "C"
