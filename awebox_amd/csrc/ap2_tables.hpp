// Host-side tables of the AP2 collocation evaluator, shared by the HIP library (awegpu.hip) and
// the CPU port used as the CPU baseline (oracle/cpu/ap2_cpu.cpp).
//
//   * collocation coefficients (collocation.py:67-200) and the V / g layout
//     (var_struct.py:39-97, constraints.py:48-145);
//   * structural row masks of the node model, obtained by instantiating ap2_node on the
//     dependency-bitmask scalar (what CasADi's symbolic sparsity propagation provides);
//   * the greedy colouring of the seed directions (compressed forward mode);
//   * the CCS pattern of J_g and, for every CCS slot, where its value comes from (gather list).
// Plain C++: no HIP types, compiles with g++ as well as hipcc.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/awegpu.h"
#include "ap2_model.hpp"

namespace awt {

constexpr int kMaxD = 9;
constexpr int kHalf = 32;        // lanes per node in the model pass (compressed directions)
constexpr int kDirs = 64;        // seed directions (lane = direction in the scatter pass)
constexpr int kDirZ = 56, kDirDiam = 57, kDirTf = 58, kDirGamma = 59, kDirPsi = 60;
constexpr int kRowPower = AWE_N_EQ + AWE_N_INEQ;       // 33: power integrand (objective)
constexpr int kRowBeta = kRowPower + 1;                // 34: side slip (objective)
constexpr int kGvalStride = 36;
constexpr unsigned long long kJRows = (1ull << kRowPower) - 1ull;
constexpr int kSegs = 4;
constexpr int kMaxConst = 8;         // CCS runs per interval: local columns, diam_t, t_f, gamma
constexpr int kPhiGamma = 0, kPhiPsi = 3;
constexpr int kCostTracking = 0, kCostURegularisation = 1, kCostXdotRegularisation = 2,
              kCostGamma = 3, kCostPsi = 5, kCostFictitious = 10, kCostPower = 11, kCostTf = 13,
              kCostThetaRegularisation = 14, kCostBeta = 18;
constexpr int kNPartial = 4;    // per interval: f, df/d diam_t, df/d t_f, df/d psi

constexpr int kPreStride = 28;
// Radau IIA nodes (what casadi::collocation_points returns, collocation.py:76)
constexpr long double kRadau[kMaxD + 1][kMaxD] = {
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

inline Coll make_coll(int d) {
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
constexpr int kPeriodicOrder[AWE_NX] = {18, 19, 20, 22, 3, 4, 5, 21, 6, 7, 8, 0, 1, 2,
                                     9, 10, 11, 12, 13, 14, 15, 16, 17};

// Compressed-direction tables (host colouring, see build_tables).  kind 0 = shooting node,
// kind 1 = Radau node.  Direction numbering (lane of the scatter pass): 0..58 node variables
// (at a Radau node: 0..22 state x_i with its own xdot_i, 23..45 xdot_i into the other
// polynomial columns, 58 = t_f through every xdot_i), 59 phi.gamma, 60 phi.psi (objective only).
struct ColorTabs {
    unsigned long long seedA[2][kHalf];   // colour seeds node variable i (bit i) / gamma (bit 59)
    unsigned int seedXD[2][kHalf];        // colour carries the xdot-direction of state i
    unsigned long long cmask[2][kHalf];   // rows (0..34) the colour produces
    int off[2][kHalf];                    // colour's first entry in the node's tangent buffer
    int tf_color[2];
    unsigned long long dmask[2][kDirs];   // rows of each direction
    int dcolor[2][kDirs];                 // colour of each direction, -1 if it has no rows
    int tsize[2];                         // tangent-buffer entries per node
    int obj_beta[kDirs];                  // Radau node: tangent-buffer index of the beta row of
    int obj_power[kDirs];                 // each direction, and of its power row (-1: none)
};

// Everything derived on the host from (n_k, d, consts).
struct Ap2Tables {
    int n_k = 0, d = 0;
    Layout lay{1, 1};
    Coll coll{};
    DevColl dcoll{};
    std::vector<double> cst;
    std::vector<int> colind, row;   // CCS pattern of J_g
    int nnz = 0;
    ColorTabs ct{};
    std::vector<int> seg;           // [n_k][kSegs][3] global CCS slot, length, list offset
    std::vector<unsigned> glist;    // per CCS slot: tangent index | scale index << 16
    std::vector<int> glist_off;     // [n_k] first list entry of each interval
    int tang_total = 0;             // tangent-buffer entries (+1 slot holding 1.0)
    int nscale = 0;                 // gather scales: 1, (d+1)^2 polynomial, constants
    std::vector<double> kconst;     // values of constant J entries
};

// structural dependency of every model output on the 59 node variables + gamma (bit 59)
struct DepIn {
    awe::Dep operator()(int i) const { return awe::Dep::bit(i); }
};

struct ModelMasks {
    unsigned long long eq[AWE_N_EQ], ineq[AWE_N_INEQ], pw, bt;
};

inline void model_masks(const double* cst, ModelMasks& mm) {
    std::vector<double> th(AWE_NTHETA0, 1.0);   // values are irrelevant for the structure
    DepIn in;
    awe::NodeResult<awe::Dep> res;
    awe::ap2_node<awe::Dep>(in, awe::Dep::bit(kDirGamma), th.data(), cst, res, true);
    for (int r = 0; r < AWE_N_EQ; ++r) mm.eq[r] = res.eq[r].m;
    for (int r = 0; r < AWE_N_INEQ; ++r) mm.ineq[r] = res.ineq[r].m;
    mm.pw = res.pw.m;
    mm.bt = res.bt.m;
}

// CPU-only: collocation coefficients, structural masks of the node model, the colouring of the
// seed directions, the CCS pattern of J_g and the kernel's LDS/CCS index tables.
inline int build_ap2_tables(int n_k, int d, const double* consts, int n_consts, Ap2Tables& T,
                            std::string& err) {
    auto fail = [&](int code, const char* msg) { err = msg; return code; };
    Ap2Tables* h = &T;
    h->n_k = n_k; h->d = d;
    h->lay = Layout(n_k, d);
    h->coll = make_coll(d);
    for (int j = 0; j <= d; ++j)
        for (int r = 0; r <= d; ++r) h->dcoll.C[j * (d + 1) + r] = h->coll.C[j][r];
    for (int j = 0; j <= d; ++j) h->dcoll.D[j] = h->coll.D[j];
    for (int j = 0; j < d; ++j) h->dcoll.w[j] = h->coll.w[j];
    h->cst.assign(consts, consts + n_consts);
    const Layout& L = h->lay;
    const Coll& cl = h->coll;
    const int NN = d + 1;

    // ---- direction row masks ------------------------------------------------------------
    ModelMasks mm;
    model_masks(h->cst.data(), mm);
    auto rows_of = [&](int var, int kind) {
        unsigned long long m = 0;
        for (int r = 0; r < AWE_N_EQ; ++r) if ((mm.eq[r] >> var) & 1ull) m |= 1ull << r;
        if (kind == 0) {
            for (int r = 0; r < AWE_N_INEQ; ++r)
                if ((mm.ineq[r] >> var) & 1ull) m |= 1ull << (AWE_N_EQ + r);
        } else {
            if ((mm.pw >> var) & 1ull) m |= 1ull << kRowPower;
            if ((mm.bt >> var) & 1ull) m |= 1ull << kRowBeta;
        }
        return m;
    };
    ColorTabs ct;
    std::memset(&ct, 0, sizeof(ct));
    for (int dir = 0; dir <= kDirGamma; ++dir) ct.dmask[0][dir] = rows_of(dir, 0);
    for (int dir = 0; dir <= kDirGamma; ++dir) {
        unsigned long long m = rows_of(dir, 1);
        if (dir < AWE_NX) m |= rows_of(AWE_NX + dir, 1);
        if (dir == kDirTf)
            for (int i = 0; i < AWE_NX; ++i) m |= rows_of(AWE_NX + i, 1);
        ct.dmask[1][dir] = m;
    }

    // ---- greedy colouring: directions with disjoint row sets share a lane ----------------
    for (int kind = 0; kind < 2; ++kind) {
        std::vector<int> order;
        for (int dir = 0; dir < kDirs; ++dir) {
            ct.dcolor[kind][dir] = -1;
            if (ct.dmask[kind][dir]) order.push_back(dir);
        }
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
            return __builtin_popcountll(ct.dmask[kind][x]) > __builtin_popcountll(ct.dmask[kind][y]);
        });
        std::vector<unsigned long long> cm;
        for (int dir : order) {
            const unsigned long long m = ct.dmask[kind][dir];
            size_t c = 0;
            while (c < cm.size() && (cm[c] & m)) ++c;
            if (c == cm.size()) cm.push_back(0ull);
            cm[c] |= m;
            ct.dcolor[kind][dir] = (int)c;
        }
        if (cm.size() > (size_t)kHalf) return fail(AWE_ERR_ARG, "internal: more than 32 colours");
        ct.tf_color[kind] = -1;
        int off = 0;
        for (int c = 0; c < kHalf; ++c) {
            ct.cmask[kind][c] = c < (int)cm.size() ? cm[c] : 0ull;
            ct.off[kind][c] = off;
            off += __builtin_popcountll(ct.cmask[kind][c]);
        }
        ct.tsize[kind] = off;
        for (int dir = 0; dir < kDirs; ++dir) {
            const int c = ct.dcolor[kind][dir];
            if (c < 0) continue;
            if (kind == 1 && dir >= AWE_NX && dir < 2 * AWE_NX) {
                ct.seedXD[kind][c] |= 1u << (dir - AWE_NX);
            } else {
                ct.seedA[kind][c] |= 1ull << dir;
                if (kind == 1 && dir == kDirTf) ct.tf_color[kind] = c;
            }
        }
    }
    for (int dir = 0; dir < kDirs; ++dir) {
        ct.obj_beta[dir] = ct.obj_power[dir] = -1;
        const int c = ct.dcolor[1][dir];
        if (c < 0) continue;
        const unsigned long long m = ct.dmask[1][dir], cm = ct.cmask[1][c];
        if ((m >> kRowBeta) & 1ull)
            ct.obj_beta[dir] = ct.off[1][c] + __builtin_popcountll(cm & ((1ull << kRowBeta) - 1ull));
        if ((m >> kRowPower) & 1ull)
            ct.obj_power[dir] = ct.off[1][c] + __builtin_popcountll(cm & ((1ull << kRowPower) - 1ull));
    }
    h->tang_total = ct.tsize[0] + d * ct.tsize[1];
    {   // the tangent buffer doubles as sub-model scratch [NN][n_el][7][6] + [NN][n_el][4]
        const int n_el = (int)h->cst[AWE_C_N_ELEMENTS];
        if (n_el < 1 || n_el > 64) return fail(AWE_ERR_ARG, "tether elements must be in 1..64");
        h->tang_total = std::max(h->tang_total, NN * n_el * (7 * 6 + 4));
    }

    // ---- target columns of each (k, node, direction) ------------------------------------
    auto dir_cols = [&](int k, int node, int dir, std::vector<int>& cols) {
        cols.clear();
        if (dir == kDirGamma) { cols.push_back(L.phi(kPhiGamma)); return; }
        if (dir >= 2 * AWE_NX + AWE_NU + AWE_NZ) {
            cols.push_back(L.theta(dir - (2 * AWE_NX + AWE_NU + AWE_NZ)));
            return;
        }
        if (dir >= 2 * AWE_NX && dir < 2 * AWE_NX + AWE_NU) { cols.push_back(L.u(k, dir - 2 * AWE_NX)); return; }
        if (node == 0) {
            if (dir < AWE_NX) cols.push_back(L.x(k, dir));
            else if (dir < 2 * AWE_NX) cols.push_back(L.xdot(k, dir - AWE_NX));
            else cols.push_back(L.z(k));
            return;
        }
        if (dir < AWE_NX) { cols.push_back(L.coll_x(k, node - 1, dir)); return; }
        if (dir < 2 * AWE_NX) {
            for (int r = 0; r < NN; ++r) if (r != node) cols.push_back(L.X(k, r, dir - AWE_NX));
            return;
        }
        cols.push_back(L.coll_z(k, node - 1));
    };
    auto node_row0 = [&](int k, int node) { return node == 0 ? L.g_shoot(k) : L.g_coll(k, node - 1); };

    // ---- triplets -----------------------------------------------------------------------
    std::vector<std::pair<int, int>> trip;   // (col, row)
    trip.reserve(200000);
    std::vector<int> cols;
    for (int k = 0; k < n_k; ++k) {
        for (int node = 0; node < NN; ++node)
            for (int dir = 0; dir < kDirs; ++dir) {
                const unsigned long long m = ct.dmask[node > 0][dir] & kJRows;
                if (!m) continue;
                dir_cols(k, node, dir, cols);
                for (int c : cols)
                    for (int r = 0; r < kRowPower; ++r)
                        if ((m >> r) & 1ull) trip.emplace_back(c, node_row0(k, node) + r);
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

    // ---- per-interval CCS runs and their LDS image ---------------------------------------
    // run 0: every entry of the interval's own columns x[k] .. coll_var[k] (the last interval
    // also owns the terminal x[n_k] columns); runs 1-3: the interval's rows of the global
    // columns diam_t, t_f and phi.gamma
    std::vector<int> seg((size_t)n_k * kSegs * 3, 0);
    const int gcols[kSegs - 1] = {L.theta(0), L.theta(1), L.phi(kPhiGamma)};
    for (int k = 0; k < n_k; ++k) {
        int* s = &seg[(size_t)k * kSegs * 3];
        const int lo = h->colind[L.x(k, 0)];
        const int hi = (k == n_k - 1) ? h->nnz : h->colind[L.x(k + 1, 0)];
        s[0] = lo; s[1] = hi - lo; s[2] = 0;
        int off = hi - lo;
        for (int q = 0; q < kSegs - 1; ++q) {
            const int col = gcols[q];
            auto b = h->row.begin() + h->colind[col], e = h->row.begin() + h->colind[col + 1];
            const int a0 = (int)(std::lower_bound(b, e, k * L.rows) - h->row.begin());
            const int a1 = (int)(std::lower_bound(b, e, (k + 1) * L.rows) - h->row.begin());
            s[3 * (q + 1)] = a0; s[3 * (q + 1) + 1] = a1 - a0; s[3 * (q + 1) + 2] = off;
            off += a1 - a0;
        }
    }
    auto lds_of = [&](int k, int slot) -> int {
        const int* s = &seg[(size_t)k * kSegs * 3];
        for (int q = 0; q < kSegs; ++q)
            if (slot >= s[3 * q] && slot < s[3 * q] + s[3 * q + 1]) return s[3 * q + 2] + slot - s[3 * q];
        return -1;
    };
    int bad = 0;
    {   // every CCS slot belongs to exactly one interval run
        std::vector<int> cover(h->nnz, 0);
        for (int k = 0; k < n_k; ++k)
            for (int q = 0; q < kSegs; ++q) {
                const int* s = &seg[((size_t)k * kSegs + q) * 3];
                for (int i = 0; i < s[1]; ++i) cover[s[0] + i]++;
            }
        for (int i = 0; i < h->nnz; ++i) if (cover[i] != 1) ++bad;
    }

    // ---- gather list: for every CCS slot of every interval, where its value comes from -------
    std::vector<int> list_off(n_k + 1, 0);
    for (int k = 0; k < n_k; ++k) {
        const int* s = &seg[(size_t)k * kSegs * 3];
        int total = 0;
        for (int q = 0; q < kSegs; ++q) total += s[3 * q + 1];
        list_off[k + 1] = list_off[k] + total;
    }
    const unsigned kUnset = 0xffffffffu;
    std::vector<unsigned> glist(list_off[n_k], kUnset);
    const int nn2 = NN * NN;
    auto put = [&](int k, int slot, int src, int scale) {
        const int q = lds_of(k, slot);
        if (q < 0 || src < 0 || src > 0xffff || scale > 0xffff) { ++bad; return; }
        unsigned& e = glist[list_off[k] + q];
        if (e != kUnset) ++bad;
        e = (unsigned)src | ((unsigned)scale << 16);
    };
    auto toff = [&](int node) { return node == 0 ? 0 : ct.tsize[0] + (node - 1) * ct.tsize[1]; };
    for (int k = 0; k < n_k; ++k)
        for (int node = 0; node < NN; ++node) {
            const int kind = node > 0;
            for (int dir = 0; dir < kDirs; ++dir) {
                const unsigned long long m = ct.dmask[kind][dir] & kJRows;
                if (!m) continue;
                const int c = ct.dcolor[kind][dir];
                const unsigned long long cm = ct.cmask[kind][c];
                const bool xd = node > 0 && dir >= AWE_NX && dir < 2 * AWE_NX;
                dir_cols(k, node, dir, cols);
                std::vector<int> rr_of;   // polynomial node of each target (xdot directions)
                for (int r = 0; r < NN; ++r) if (r != node) rr_of.push_back(r);
                const int g0 = node_row0(k, node);
                for (size_t t = 0; t < cols.size(); ++t)
                    for (int r = 0; r < kRowPower; ++r) {
                        if (!((m >> r) & 1ull)) continue;
                        const int src = toff(node) + ct.off[kind][c] +
                                        __builtin_popcountll(cm & ((1ull << r) - 1ull));
                        const int scale = xd ? 1 + rr_of[t] * NN + node : 0;
                        put(k, find(cols[t], g0 + r), src, scale);
                    }
            }
        }
    // ---- constant entries: continuity (+1, -D_r) and periodicity (+1, -1) ------------------
    std::vector<double>& kc = h->kconst;
    kc.clear();
    auto add_const = [&](int col, int rw, double val) {
        const int slot = find(col, rw);
        size_t q = 0;
        while (q < kc.size() && kc[q] != val) ++q;
        if (q == kc.size()) kc.push_back(val);
        for (int k = 0; k < n_k; ++k)
            if (lds_of(k, slot) >= 0) { put(k, slot, h->tang_total, 1 + nn2 + (int)q); return; }
        ++bad;
    };
    for (int k = 0; k < n_k; ++k)
        for (int i = 0; i < AWE_NX; ++i) {
            add_const(L.x(k + 1, i), L.g_cont(k) + i, 1.0);
            for (int r = 0; r < NN; ++r)
                if (cl.D[r] != 0.0) add_const(L.X(k, r, i), L.g_cont(k) + i, -cl.D[r]);
        }
    for (int i = 0; i < AWE_NX; ++i) {
        add_const(L.x(0, kPeriodicOrder[i]), L.g_periodic() + i, 1.0);
        add_const(last + kPeriodicOrder[i], L.g_periodic() + i, -1.0);
    }
    if ((int)kc.size() > kMaxConst) return fail(AWE_ERR_ARG, "internal: too many constant entries");
    h->nscale = 1 + nn2 + (int)kc.size();
    if (h->nscale > 64) return fail(AWE_ERR_ARG, "internal: scale table exceeds 64 entries");
    // every slot of every interval run has exactly one source
    for (unsigned e : glist) if (e == kUnset) ++bad;
    if (bad) return fail(AWE_ERR_ARG, "internal: inconsistent sparsity tables");
    T.glist.swap(glist);
    T.glist_off.assign(list_off.begin(), list_off.end() - 1);
    T.seg.swap(seg);
    T.ct = ct;
    return AWE_OK;
}


// =========================================================================================
// Hessian of the Lagrangian (nlp_hess_l)
// =========================================================================================

// Structural second-order dependency: d = variables the value depends on, h[i] bit j = the value
// has a (possibly) nonzero second derivative in (i, j).  Propagated through the node model like
// Dep; what CasADi's symbolic Hessian sparsity provides in the reference.
struct HDep {
    unsigned long long d = 0;
    unsigned long long h[64] = {};
    HDep() = default;
    HDep(double) {}
    static HDep var(int i) { HDep x; x.d = 1ull << i; return x; }
};
inline void hdep_cross(HDep& r, unsigned long long a, unsigned long long b) {
    for (int i = 0; i < 64; ++i) {
        if ((a >> i) & 1ull) r.h[i] |= b;
        if ((b >> i) & 1ull) r.h[i] |= a;
    }
}
inline HDep hdep_lin(const HDep& x, const HDep& y) {
    HDep r; r.d = x.d | y.d;
    for (int i = 0; i < 64; ++i) r.h[i] = x.h[i] | y.h[i];
    return r;
}
inline HDep hdep_nl(const HDep& x) { HDep r = x; hdep_cross(r, x.d, x.d); return r; }
inline HDep operator+(const HDep& x, const HDep& y) { return hdep_lin(x, y); }
inline HDep operator-(const HDep& x, const HDep& y) { return hdep_lin(x, y); }
inline HDep operator-(const HDep& x) { return x; }
inline HDep operator*(const HDep& x, const HDep& y) { HDep r = hdep_lin(x, y); hdep_cross(r, x.d, y.d); return r; }
inline HDep operator/(const HDep& x, const HDep& y) {
    HDep r = hdep_lin(x, y); hdep_cross(r, x.d, y.d); hdep_cross(r, y.d, y.d); return r;
}
inline HDep operator+(const HDep& x, double) { return x; }
inline HDep operator+(double, const HDep& y) { return y; }
inline HDep operator-(const HDep& x, double) { return x; }
inline HDep operator-(double, const HDep& y) { return y; }
inline HDep operator*(const HDep& x, double) { return x; }
inline HDep operator*(double, const HDep& y) { return y; }
inline HDep operator/(const HDep& x, double) { return x; }
inline HDep operator/(double, const HDep& y) { return hdep_nl(y); }
inline HDep sqrt(const HDep& x) { return hdep_nl(x); }
inline HDep exp(const HDep& x) { return hdep_nl(x); }
inline HDep log(const HDep& x) { return hdep_nl(x); }

constexpr int kHRows = 35;              // node rows incl. power (33) and beta (34)
constexpr int kHTypeA = 0, kHTypeB = 1, kHTypeC = 2;

// Gather term of one V-space Hessian entry (bits 31..30 type):
//   A: scale[sa] scale[sb] Hdir_n[pidx]          n 27..29, pidx 14..26, sa 7..13, sb 0..6
//   B: G[n][i] (-C[r][n] / (h tf^2))              n 27..29, i 22..26, r 19..21
//   C: sum_i G[n][i] 2 xdot_i / tf^2  (t_f, t_f)  n 27..29
inline unsigned hterm_a(int n, int pidx, int sa, int sb) {
    return ((unsigned)kHTypeA << 30) | ((unsigned)n << 27) | ((unsigned)pidx << 14) | ((unsigned)sa << 7) | (unsigned)sb;
}
inline unsigned hterm_b(int n, int i, int r) {
    return ((unsigned)kHTypeB << 30) | ((unsigned)n << 27) | ((unsigned)i << 22) | ((unsigned)r << 19);
}
inline unsigned hterm_c(int n) { return ((unsigned)kHTypeC << 30) | ((unsigned)n << 27); }

struct HessTabs {                       // device-visible part
    int npairs[2];                      // direction pairs per node kind
    short pidx[2][kDirs][kDirs];        // compact index of the (unordered) direction pair, -1
    signed char pdir[2][kHalf][kHRows + 1];   // direction of colour c that owns row r, -1
    int ntask[2];
    int task_off[2];                    // offsets into the task list (c1 | c2 << 8)
};

struct Ap2HessTables {
    HessTabs ht{};
    std::vector<int> tasks;             // per kind: colour pairs c1 <= c2
    std::vector<int> colind, row;       // upper-triangular CCS of the V-space Hessian
    int nnz = 0;
    std::vector<int> slot0, nslot;      // [n_k] the interval's contiguous CCS range
    std::vector<int> gslot;             // CCS slots of the global-global entries
    std::vector<int> ent_off;           // [n_k + 1] entries of each interval (local slots, then globals)
    std::vector<int> term_off;          // [n_entries + 1] into terms
    std::vector<unsigned> terms;
    std::vector<short> task_target;     // [task][kHRows + 1]: pair index a row feeds, -1
    int max_pairs = 0;
};

// V columns (with gather-scale index) that direction `dir` of node `node` of interval k feeds
inline void direction_columns(const Layout& L, int d, int k, int node, int dir,
                              std::vector<std::pair<int, int>>& cols) {
    const int NN = d + 1;
    cols.clear();
    if (dir == kDirPsi) { cols.emplace_back(L.phi(kPhiPsi), 0); return; }
    if (dir == kDirGamma) { cols.emplace_back(L.phi(kPhiGamma), 0); return; }
    if (dir >= 2 * AWE_NX + AWE_NU + AWE_NZ) { cols.emplace_back(L.theta(dir - (2 * AWE_NX + AWE_NU + AWE_NZ)), 0); return; }
    if (dir >= 2 * AWE_NX && dir < 2 * AWE_NX + AWE_NU) { cols.emplace_back(L.u(k, dir - 2 * AWE_NX), 0); return; }
    if (node == 0) {
        if (dir < AWE_NX) cols.emplace_back(L.x(k, dir), 0);
        else if (dir < 2 * AWE_NX) cols.emplace_back(L.xdot(k, dir - AWE_NX), 0);
        else cols.emplace_back(L.z(k), 0);
        return;
    }
    if (dir < AWE_NX) { cols.emplace_back(L.coll_x(k, node - 1, dir), 0); return; }
    if (dir < 2 * AWE_NX) {
        for (int r = 0; r < NN; ++r)
            if (r != node) cols.emplace_back(L.X(k, r, dir - AWE_NX), 1 + r * NN + node);
        return;
    }
    cols.emplace_back(L.coll_z(k, node - 1), 0);
}

inline int build_hess_tables(const Ap2Tables& T, Ap2HessTables& H, std::string& err) {
    const Layout& L = T.lay;
    const ColorTabs& ct = T.ct;
    const int n_k = T.n_k, d = T.d, NN = d + 1;
    HessTabs& ht = H.ht;
    std::memset(&ht, 0, sizeof(ht));
    std::memset(ht.pidx, 0xff, sizeof(ht.pidx));
    std::memset(ht.pdir, 0xff, sizeof(ht.pdir));

    // ---- second-order structure of every node row, over the node variables + gamma ---------
    struct HSink {
        HDep rows[kHRows];
        void eq_row(int r, const HDep& v) { rows[r] = v; }
        void ineq_row(int r, const HDep& v) { rows[AWE_N_EQ + r] = v; }
        void power(const HDep& v) { rows[kRowPower] = v; }
        void beta(const HDep& v) { rows[kRowBeta] = v; }
    };
    struct HIn { HDep operator()(int i) const { return HDep::var(i); } };
    std::vector<double> th(AWE_NTHETA0, 1.0);
    HSink hs;
    awe::ap2_node<HDep>(HIn{}, HDep::var(kDirGamma), th.data(), T.cst.data(), hs, true);

    // node variables each direction seeds
    auto dvars = [&](int kind, int dir) {
        unsigned long long m = 0;
        if (dir > kDirGamma) return m;
        if (kind == 0) return 1ull << dir;
        if (dir < AWE_NX) return (1ull << dir) | (1ull << (AWE_NX + dir));
        if (dir == kDirTf) {
            for (int i = 0; i < AWE_NX; ++i) m |= 1ull << (AWE_NX + i);
            return m;
        }
        return 1ull << dir;
    };
    auto row_used = [&](int kind, int r) {
        if (kind == 0) return r < kRowPower;
        return r < AWE_N_EQ || r == kRowPower || r == kRowBeta;
    };
    auto interacts = [&](int r, unsigned long long va, unsigned long long vb) {
        for (int u = 0; u < 64; ++u)
            if (((va >> u) & 1ull) && (hs.rows[r].h[u] & vb)) return true;
        return false;
    };
    std::vector<std::vector<std::pair<int, int>>> pairs(2);
    std::vector<std::vector<char>> has(2, std::vector<char>(kDirs * kDirs, 0));
    auto add_pair = [&](int kind, int p, int q) {
        if (p > q) std::swap(p, q);
        if (!has[kind][p * kDirs + q]) { has[kind][p * kDirs + q] = 1; pairs[kind].emplace_back(p, q); }
    };
    std::vector<int> task_set[2];
    for (int kind = 0; kind < 2; ++kind) {
        std::vector<char> tk(kHalf * kHalf, 0);
        for (int r = 0; r < kHRows; ++r) {
            if (!row_used(kind, r)) continue;
            for (int p = 0; p <= kDirGamma; ++p)
                for (int q = p; q <= kDirGamma; ++q) {
                    const unsigned long long vp = dvars(kind, p), vq = dvars(kind, q);
                    if (!vp || !vq || !interacts(r, vp, vq)) continue;
                    const int cp = ct.dcolor[kind][p], cq = ct.dcolor[kind][q];
                    if (cp < 0 || cq < 0 || !((ct.dmask[kind][p] >> r) & 1ull) || !((ct.dmask[kind][q] >> r) & 1ull)) {
                        err = "internal: Hessian structure outside the first-order pattern";
                        return AWE_ERR_ARG;
                    }
                    add_pair(kind, p, q);
                    tk[std::min(cp, cq) * kHalf + std::max(cp, cq)] = 1;
                }
        }
        for (int c1 = 0; c1 < kHalf; ++c1)
            for (int c2 = c1; c2 < kHalf; ++c2)
                if (tk[c1 * kHalf + c2]) task_set[kind].push_back(c1 | (c2 << 8));
    }
    // objective terms at Radau nodes (objective.py; see the kernel's objective Hessian pass)
    {
        const int kind = 1;
        for (int i = 0; i < AWE_NX; ++i) {
            add_pair(kind, i, i);
            add_pair(kind, i, AWE_NX + i);
            add_pair(kind, i, kDirTf);
            add_pair(kind, AWE_NX + i, AWE_NX + i);
            add_pair(kind, AWE_NX + i, kDirTf);
            add_pair(kind, i, kDirPsi);
        }
        add_pair(kind, kDirTf, kDirTf);
        for (int i = 2 * AWE_NX; i <= kDirDiam; ++i) add_pair(kind, i, i);
        add_pair(kind, kDirZ, kDirPsi);
        std::vector<int> bdirs, pdirs;
        for (int p = 0; p <= kDirGamma; ++p) {
            if ((ct.dmask[1][p] >> kRowBeta) & 1ull) bdirs.push_back(p);
            if ((ct.dmask[1][p] >> kRowPower) & 1ull) pdirs.push_back(p);
        }
        for (size_t a = 0; a < bdirs.size(); ++a)
            for (size_t b = a; b < bdirs.size(); ++b) add_pair(kind, bdirs[a], bdirs[b]);
        for (int p : pdirs) add_pair(kind, p, kDirPsi);
    }
    for (int kind = 0; kind < 2; ++kind) {
        std::sort(pairs[kind].begin(), pairs[kind].end());
        ht.npairs[kind] = (int)pairs[kind].size();
        if (ht.npairs[kind] >= 8192) { err = "internal: too many Hessian direction pairs"; return AWE_ERR_ARG; }
        for (int i = 0; i < ht.npairs[kind]; ++i) {
            const int p = pairs[kind][i].first, q = pairs[kind][i].second;
            ht.pidx[kind][p][q] = ht.pidx[kind][q][p] = (short)i;
        }
        for (int dir = 0; dir < kDirs; ++dir) {
            const int c = ct.dcolor[kind][dir];
            if (c < 0) continue;
            for (int r = 0; r < kHRows; ++r)
                if ((ct.dmask[kind][dir] >> r) & 1ull) ht.pdir[kind][c][r] = (signed char)dir;
        }
        ht.task_off[kind] = (int)H.tasks.size();
        ht.ntask[kind] = (int)task_set[kind].size();
        H.tasks.insert(H.tasks.end(), task_set[kind].begin(), task_set[kind].end());
    }
    H.max_pairs = std::max(ht.npairs[0], ht.npairs[1]);
    // per task and row: the direction pair its mixed second derivative belongs to
    H.task_target.assign(H.tasks.size() * (kHRows + 1), (short)-1);
    for (int kind = 0; kind < 2; ++kind)
        for (int t = 0; t < ht.ntask[kind]; ++t) {
            const int task = H.tasks[ht.task_off[kind] + t], c1 = task & 0xff, c2 = task >> 8;
            for (int r = 0; r < kHRows; ++r) {
                if (!row_used(kind, r)) continue;
                const int p = ht.pdir[kind][c1][r], q = ht.pdir[kind][c2][r];
                if (p < 0 || q < 0) continue;
                H.task_target[(size_t)(ht.task_off[kind] + t) * (kHRows + 1) + r] = ht.pidx[kind][p][q];
            }
        }

    // ---- V-space entries and their gather terms ----------------------------------------------
    auto is_global = [&](int col) { return col < L.v_int0; };
    std::vector<std::pair<long long, unsigned>> ent;   // (key = col * n_v + row, term), with the interval
    std::vector<int> ent_k;
    std::vector<std::pair<int, int>> ca, cb;
    const int itf = L.theta(1);
    for (int k = 0; k < n_k; ++k)
        for (int node = 0; node < NN; ++node) {
            const int kind = node > 0;
            for (const auto& pq : pairs[kind]) {
                const int p = pq.first, q = pq.second;
                const int pi = ht.pidx[kind][p][q];
                direction_columns(L, d, k, node, p, ca);
                direction_columns(L, d, k, node, q, cb);
                for (size_t a = 0; a < ca.size(); ++a)
                    for (size_t b = (p == q ? a : 0); b < cb.size(); ++b) {
                        int r0 = ca[a].first, c0 = cb[b].first, sa = ca[a].second, sb = cb[b].second;
                        if (r0 > c0) { std::swap(r0, c0); std::swap(sa, sb); }
                        ent.emplace_back((long long)c0 * L.n_v + r0, hterm_a(node, pi, sa, sb));
                        ent_k.push_back(k);
                    }
            }
            if (node == 0) continue;
            for (int i = 0; i < AWE_NX; ++i)
                for (int r = 0; r < NN; ++r) {
                    const int col = L.X(k, r, i);
                    ent.emplace_back((long long)col * L.n_v + itf, hterm_b(node, i, r));
                    ent_k.push_back(k);
                }
            ent.emplace_back((long long)itf * L.n_v + itf, hterm_c(node));
            ent_k.push_back(k);
        }
    // CCS pattern (upper triangle, column-major) and per-interval slot ranges
    std::vector<long long> keys;
    keys.reserve(ent.size());
    for (auto& e : ent) keys.push_back(e.first);
    keys.push_back((long long)itf * L.n_v + itf);            // time cost (t_f, t_f)
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    H.nnz = (int)keys.size();
    H.colind.assign(L.n_v + 1, 0);
    H.row.resize(H.nnz);
    for (int i = 0; i < H.nnz; ++i) {
        H.colind[keys[i] / L.n_v + 1]++;
        H.row[i] = (int)(keys[i] % L.n_v);
    }
    for (int c = 0; c < L.n_v; ++c) H.colind[c + 1] += H.colind[c];
    auto slot_of = [&](long long key) {
        return (int)(std::lower_bound(keys.begin(), keys.end(), key) - keys.begin());
    };
    for (int c = 0; c < L.v_int0; ++c)
        for (int s = H.colind[c]; s < H.colind[c + 1]; ++s) H.gslot.push_back(s);
    const int ng = (int)H.gslot.size();
    H.slot0.resize(n_k);
    H.nslot.resize(n_k);
    for (int k = 0; k < n_k; ++k) {
        H.slot0[k] = H.colind[L.x(k, 0)];
        H.nslot[k] = (k == n_k - 1 ? H.nnz : H.colind[L.x(k + 1, 0)]) - H.slot0[k];
    }
    // terms per (interval, entry): entries 0..nslot-1 are the local slots, then ng globals
    std::vector<std::vector<unsigned>> bucket;
    H.ent_off.assign(n_k + 1, 0);
    for (int k = 0; k < n_k; ++k) H.ent_off[k + 1] = H.ent_off[k] + H.nslot[k] + ng;
    bucket.resize(H.ent_off[n_k]);
    for (size_t e = 0; e < ent.size(); ++e) {
        const int k = ent_k[e];
        const int slot = slot_of(ent[e].first);
        const int col = (int)(ent[e].first / L.n_v);
        int idx;
        if (is_global(col)) {
            idx = (int)(std::find(H.gslot.begin(), H.gslot.end(), slot) - H.gslot.begin());
            idx += H.nslot[k];
        } else {
            idx = slot - H.slot0[k];
            if (idx < 0 || idx >= H.nslot[k]) { err = "internal: Hessian entry outside its interval"; return AWE_ERR_ARG; }
        }
        bucket[H.ent_off[k] + idx].push_back(ent[e].second);
    }
    H.term_off.assign(bucket.size() + 1, 0);
    for (size_t i = 0; i < bucket.size(); ++i) {
        H.term_off[i + 1] = H.term_off[i] + (int)bucket[i].size();
        H.terms.insert(H.terms.end(), bucket[i].begin(), bucket[i].end());
    }
    return AWE_OK;
}

}  // namespace awt
