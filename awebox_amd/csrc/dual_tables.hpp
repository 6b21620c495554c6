// Host-side tables of the multi-kite evaluator (awedual.hip).  Plain C++ (g++ and hipcc).
//
//   * the NLP layout with the single_reelout phase fix (var_struct.py:39-115: V.theta =
//     [diam_t, t_f(2), l_s, diam_s]; constraints.py:48-170: per interval [shooting 53, path 19,
//     collocation d x 53, continuity 50], then periodic 50 and the two t_f bound rows);
//   * structural row masks of dual_node (instantiated on the 128-bit dependency scalar Dep2);
//   * compressed forward mode: the 127 seed directions of a node (126 node variables + phi.gamma)
//     are greedily coloured (Curtis-Powell-Reid) into <= 64 groups with disjoint row sets, so one
//     64-lane wavefront recovers a node's whole Jacobian block;
//   * the CCS pattern of J_g and, per CCS slot, where its value comes from (gather list).
//
// Directions.  Shooting node (kind 0): direction i seeds node variable i (126 = phi.gamma).
// Radau node n (kind 1): direction i < 50 seeds state x_i together with xdot_i += C[n][n]/(h tf)
// (its column is the collocation variable X_{n,i}); direction 50 + i seeds xdot_i alone (the
// columns X_{r,i}, r != n, get that tangent times C[r][n]/(h tf)); direction 123 seeds t_f and
// every xdot_i with -xdot_i/tf (collocation.py:202-258); the others seed their variable.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/awedual.h"
#include "ap2_tables.hpp"      // awt::Coll / make_coll
#include "dual_model.hpp"

namespace dlt {

constexpr int kDirs = 127;
constexpr int kLanes = 64;
constexpr int kRowPower = ADL_N_EQ + ADL_N_INEQ;   // 72
constexpr int kRowBeta0 = kRowPower + 1;           // 73, 74
constexpr int kNRows = kRowBeta0 + ADL_NKITES;     // 75
constexpr int kGvalStride = 76;
constexpr int kMaxConst = 16;

// objective (objective.py): partial sums per interval -- tracking, other, power integral A_k,
// d/d diam_t, t_f, l_s, diam_s -- and the cost-vector indices of P's cost entries
constexpr int kNPart = 8;
constexpr int kCostTracking = 0, kCostURegularisation = 1, kCostXdotRegularisation = 2, kCostFictitious = 10,
              kCostPower = 11, kCostTf = 13, kCostThetaRegularisation = 14, kCostBeta = 18;
constexpr int kPhiCost[7] = {3, 6, 4, 5, 7, 8, 9};   // cost index of phi = [gamma tau iota psi eta nu upsilon]
constexpr int kPhiPsi = 3;
// periodicity rows in the sorted order of the x names (operation.py:245-266): state index of each row
constexpr int kPeriodicOrder[ADL_NX] = {24, 25, 26, 45, 46, 47, 49, 3,  4,  5,  9,  10, 11, 30, 31, 32, 48,
                                        12, 13, 14, 33, 34, 35, 0,  1,  2,  6,  7,  8,  27, 28, 29,
                                        15, 16, 17, 18, 19, 20, 21, 22, 23, 36, 37, 38, 39, 40, 41, 42, 43, 44};

struct Mask {
    uint64_t lo = 0, hi = 0;
    bool has(int r) const { return r < 64 ? ((lo >> r) & 1u) : ((hi >> (r - 64)) & 1u); }
    void set(int r) { if (r < 64) lo |= (uint64_t)1 << r; else hi |= (uint64_t)1 << (r - 64); }
    bool any() const { return lo || hi; }
    bool meets(const Mask& o) const { return (lo & o.lo) || (hi & o.hi); }
    void merge(const Mask& o) { lo |= o.lo; hi |= o.hi; }
    int count() const { return __builtin_popcountll(lo) + __builtin_popcountll(hi); }
    int below(int r) const {   // number of set rows < r
        if (r < 64) return __builtin_popcountll(lo & (((uint64_t)1 << r) - 1u));
        return __builtin_popcountll(lo) + __builtin_popcountll(hi & (((uint64_t)1 << (r - 64)) - 1u));
    }
};

struct Layout {
    int n_k = 0, d = 0, nk_reelout = 0, single = 1, n_thv = ADL_NTHV;
    int stride = 0, v_int0 = 0, n_v = 0, rows = 0, n_g = 0, n_p = 0;
    void init(int nk, int dd, int nkr, int sgl) {
        n_k = nk; d = dd; nk_reelout = nkr; single = sgl;
        n_thv = sgl ? ADL_NTHV : ADL_NTH;
        stride = 2 * ADL_NX + ADL_NU + ADL_NZ + dd * (ADL_NX + ADL_NZ);
        v_int0 = n_thv + 7 + 2;
        n_v = v_int0 + nk * stride + ADL_NX;
        rows = ADL_N_EQ + ADL_N_INEQ + dd * ADL_N_EQ + ADL_NX;
        n_g = nk * rows + ADL_NX + (sgl ? 2 : 0);
        n_p = n_v + ADL_NW + 20 + AWE_NTHETA0;
    }
    int th_diam_t() const { return 0; }
    int th_tf(int k) const { return single ? (k < nk_reelout ? 1 : 2) : 1; }
    int th_ls() const { return single ? 3 : 2; }
    int th_diam_s() const { return single ? 4 : 3; }
    int phi(int i) const { return n_thv + i; }
    int x(int k, int i) const { return v_int0 + k * stride + i; }
    int u(int k, int i) const { return v_int0 + k * stride + ADL_NX + i; }
    int xdot(int k, int i) const { return v_int0 + k * stride + ADL_NX + ADL_NU + i; }
    int z(int k, int i) const { return v_int0 + k * stride + 2 * ADL_NX + ADL_NU + i; }
    int coll_x(int k, int j, int i) const {
        return v_int0 + k * stride + 2 * ADL_NX + ADL_NU + ADL_NZ + j * (ADL_NX + ADL_NZ) + i;
    }
    int coll_z(int k, int j, int i) const { return coll_x(k, j, 0) + ADL_NX + i; }
    int X(int k, int r, int i) const { return r == 0 ? x(k, i) : coll_x(k, r - 1, i); }
    int g_shoot(int k) const { return k * rows; }
    int g_coll(int k, int j) const { return k * rows + ADL_N_EQ + ADL_N_INEQ + j * ADL_N_EQ; }
    int g_cont(int k) const { return k * rows + ADL_N_EQ + ADL_N_INEQ + d * ADL_N_EQ; }
    int g_periodic() const { return n_k * rows; }
    int g_tf() const { return n_k * rows + ADL_NX; }
};

// device-visible colouring tables
struct ColorTabs {
    int8_t col[2][128];         // colour of each direction (-1: no rows)
    uint64_t cm_lo[2][kLanes];  // rows produced by each colour
    uint64_t cm_hi[2][kLanes];
    int off[2][kLanes];         // first tangent-buffer entry of each colour (node-relative)
    int ncol[2];
    int tsize[2];               // tangent-buffer entries per node
    int obj_tang[kDirs][3];     // Radau node: node-relative tangent index of the power / beta2 /
                                // beta3 rows of each direction, -1 if structurally zero
};

// gather code: kind (bits 29..31) | r (25..28) | n (21..24) | payload (0..20)
constexpr uint32_t kKindTang = 0, kKindTangPoly = 1, kKindConst = 2;
inline uint32_t gcode(uint32_t kind, int r, int n, int payload) {
    return (kind << 29) | ((uint32_t)r << 25) | ((uint32_t)n << 21) | (uint32_t)payload;
}

struct Tables {
    Layout lay;
    awt::Coll coll{};
    ColorTabs ct{};
    Mask dmask[2][kDirs];
    std::vector<int> colind, row;
    std::vector<int> goff, gslot;
    std::vector<uint32_t> gcode;
    std::vector<double> kconst;
    int tang_total = 0;
};

struct DepSink {
    awe::Dep2 rows[kNRows];
    void eq_row(int r, const awe::Dep2& v) { rows[r] = v; }
    void ineq_row(int r, const awe::Dep2& v) { rows[ADL_N_EQ + r] = v; }
    void power(const awe::Dep2& v) { rows[kRowPower] = v; }
    void beta(int k, const awe::Dep2& v) { rows[kRowBeta0 + k] = v; }
};
struct DepIn {
    awe::Dep2 operator()(int i) const { return awe::Dep2::bit(i); }
};

inline int build_tables(int n_k, int d, const double* consts, int n_consts, Tables& T, std::string& err) {
    auto fail = [&](const char* m) { err = m; return 1; };
    if (n_consts != ADL_NCONST) return fail("consts must have ADL_NCONST entries");
    if (n_k < 1 || d < 1 || d > 5) return fail("need n_k >= 1 and 1 <= d <= 5");
    if (consts[ADL_C_N_K] != (double)n_k || consts[ADL_C_D] != (double)d)
        return fail("consts[ADL_C_N_K], consts[ADL_C_D] disagree with n_k, d");
    const int nkr = (int)consts[ADL_C_NK_REELOUT];
    const int sgl = consts[ADL_C_SINGLE_REELOUT] != 0.0;
    if (sgl && (nkr < 1 || nkr >= n_k)) return fail("single_reelout needs 1 <= nk_reelout < n_k");
    const int n_el = (int)consts[ADL_C_N_ELEMENTS];
    if (n_el < 1 || n_el > 64) return fail("tether elements must be in 1..64");
    T.lay.init(n_k, d, sgl ? nkr : n_k, sgl);
    T.coll = awt::make_coll(d);
    const Layout& L = T.lay;
    const int NN = d + 1;

    // ---- structural row masks of the node model ------------------------------------------
    Mask vrows[kDirs];   // rows of each node variable (+ gamma)
    {
        std::vector<double> th(AWE_NTHETA0, 1.0);
        DepSink s;
        awe::dual_node<awe::Dep2>(DepIn{}, awe::Dep2::bit(awe::dl::kGamma), th.data(), consts, s, true);
        for (int r = 0; r < kNRows; ++r)
            for (int v = 0; v < kDirs; ++v)
                if (s.rows[r].has(v)) vrows[v].set(r);
    }
    auto restrict_kind = [&](Mask m, int kind) {
        Mask o;
        for (int r = 0; r < kNRows; ++r) {
            if (!m.has(r)) continue;
            const bool eq = r < ADL_N_EQ, ineq = r >= ADL_N_EQ && r < kRowPower, obj = r >= kRowPower;
            if (eq || (kind == 0 && ineq) || (kind == 1 && obj)) o.set(r);
        }
        return o;
    };
    ColorTabs& ct = T.ct;
    std::memset(&ct, 0, sizeof(ct));
    for (int dir = 0; dir < kDirs; ++dir) {
        T.dmask[0][dir] = restrict_kind(vrows[dir], 0);
        Mask m = vrows[dir];
        if (dir < ADL_NX) m.merge(vrows[ADL_NX + dir]);
        if (dir == awe::dl::kTf)
            for (int i = 0; i < ADL_NX; ++i) m.merge(vrows[ADL_NX + i]);
        T.dmask[1][dir] = restrict_kind(m, 1);
    }
    for (int kind = 0; kind < 2; ++kind) {
        std::vector<int> order;
        for (int dir = 0; dir < 128; ++dir) ct.col[kind][dir] = -1;
        for (int dir = 0; dir < kDirs; ++dir)
            if (T.dmask[kind][dir].any()) order.push_back(dir);
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
            return T.dmask[kind][a].count() > T.dmask[kind][b].count();
        });
        std::vector<Mask> cm;
        for (int dir : order) {
            const Mask& m = T.dmask[kind][dir];
            size_t c = 0;
            while (c < cm.size() && cm[c].meets(m)) ++c;
            if (c == cm.size()) cm.push_back(Mask{});
            cm[c].merge(m);
            ct.col[kind][dir] = (int8_t)c;
        }
        if (cm.size() > (size_t)kLanes) return fail("internal: more than 64 colours");
        ct.ncol[kind] = (int)cm.size();
        int off = 0;
        for (int c = 0; c < kLanes; ++c) {
            const Mask m = c < (int)cm.size() ? cm[c] : Mask{};
            ct.cm_lo[kind][c] = m.lo;
            ct.cm_hi[kind][c] = m.hi;
            ct.off[kind][c] = off;
            off += m.count();
        }
        ct.tsize[kind] = off;
    }
    auto tidx = [&](int kind, int dir, int r) -> int {   // node-relative tangent index
        const int c = ct.col[kind][dir];
        if (c < 0 || !T.dmask[kind][dir].has(r)) return -1;
        Mask m;
        m.lo = ct.cm_lo[kind][c];
        m.hi = ct.cm_hi[kind][c];
        return ct.off[kind][c] + m.below(r);
    };
    for (int dir = 0; dir < kDirs; ++dir)
        for (int q = 0; q < 3; ++q) ct.obj_tang[dir][q] = tidx(1, dir, kRowPower + q);
    T.tang_total = ct.tsize[0] + d * ct.tsize[1];
    auto toff = [&](int n) { return n == 0 ? 0 : ct.tsize[0] + (n - 1) * ct.tsize[1]; };

    // ---- triplets (col, row, owner interval, code) ----------------------------------------
    std::vector<std::tuple<int, int, int, uint32_t>> trip;
    trip.reserve((size_t)n_k * 8000);
    auto& kc = T.kconst;
    kc.clear();
    auto kidx = [&](double v) -> int {
        for (size_t q = 0; q < kc.size(); ++q)
            if (kc[q] == v) return (int)q;
        kc.push_back(v);
        return (int)kc.size() - 1;
    };
    for (int k = 0; k < n_k; ++k) {
        for (int n = 0; n < NN; ++n) {
            const int kind = n > 0;
            const int g0 = n == 0 ? L.g_shoot(k) : L.g_coll(k, n - 1);
            for (int dir = 0; dir < kDirs; ++dir) {
                const Mask& m = T.dmask[kind][dir];
                for (int r = 0; r < kRowPower; ++r) {
                    if (!m.has(r)) continue;
                    const int src = toff(n) + tidx(kind, dir, r);
                    const uint32_t code = gcode(kKindTang, 0, 0, src);
                    const int grow = g0 + r;
                    if (dir == awe::dl::kGamma) { trip.emplace_back(L.phi(0), grow, k, code); continue; }
                    if (dir >= 2 * ADL_NX + ADL_NU + ADL_NZ) {            // theta
                        const int t = dir - (2 * ADL_NX + ADL_NU + ADL_NZ);
                        const int col = t == 0 ? L.th_diam_t() : t == 1 ? L.th_tf(k) : t == 2 ? L.th_ls() : L.th_diam_s();
                        trip.emplace_back(col, grow, k, code);
                        continue;
                    }
                    if (dir >= 2 * ADL_NX && dir < 2 * ADL_NX + ADL_NU) {
                        trip.emplace_back(L.u(k, dir - 2 * ADL_NX), grow, k, code);
                        continue;
                    }
                    if (dir >= 2 * ADL_NX + ADL_NU) {                     // z
                        const int i = dir - (2 * ADL_NX + ADL_NU);
                        trip.emplace_back(n == 0 ? L.z(k, i) : L.coll_z(k, n - 1, i), grow, k, code);
                        continue;
                    }
                    if (n == 0) {
                        trip.emplace_back(dir < ADL_NX ? L.x(k, dir) : L.xdot(k, dir - ADL_NX), grow, k, code);
                        continue;
                    }
                    if (dir < ADL_NX) { trip.emplace_back(L.coll_x(k, n - 1, dir), grow, k, code); continue; }
                    for (int rr = 0; rr < NN; ++rr)
                        if (rr != n)
                            trip.emplace_back(L.X(k, rr, dir - ADL_NX), grow, k, gcode(kKindTangPoly, rr, n, src));
                }
            }
        }
        for (int i = 0; i < ADL_NX; ++i) {   // continuity x[k+1] - sum_r D_r X_{k,r}
            const int grow = L.g_cont(k) + i;
            trip.emplace_back(L.x(k + 1, i), grow, k, gcode(kKindConst, 0, 0, kidx(1.0)));
            for (int rr = 0; rr < NN; ++rr)
                if (T.coll.D[rr] != 0.0)
                    trip.emplace_back(L.X(k, rr, i), grow, k, gcode(kKindConst, 0, 0, kidx(-T.coll.D[rr])));
        }
    }
    {   // periodicity (sorted x names, operation.py:245-266) and the t_f bounds (constraints.py:148-170)
        static const char* names[] = {"q10", "dq10", "q21", "dq21", "omega21", "r21", "delta21",
                                      "q31", "dq31", "omega31", "r31", "delta31", "l_t", "dl_t"};
        static const int sizes[] = {3, 3, 3, 3, 3, 9, 3, 3, 3, 3, 9, 3, 1, 1};
        std::vector<std::pair<std::string, int>> ent;
        int pos = 0;
        for (int e = 0; e < 14; ++e) { ent.emplace_back(names[e], pos); pos += sizes[e]; }
        std::vector<int> size_of(14);
        std::vector<int> idx(14);
        for (int e = 0; e < 14; ++e) idx[e] = e;
        std::sort(idx.begin(), idx.end(), [&](int a, int b) { return ent[a].first < ent[b].first; });
        int row = L.g_periodic();
        const int last = n_k - 1;
        for (int e : idx)
            for (int i = 0; i < sizes[e]; ++i, ++row) {
                trip.emplace_back(L.x(0, ent[e].second + i), row, last, gcode(kKindConst, 0, 0, kidx(1.0)));
                trip.emplace_back(L.coll_x(last, d - 1, ent[e].second + i), row, last, gcode(kKindConst, 0, 0, kidx(-1.0)));
            }
        if (sgl) {
            const double frac = consts[ADL_C_PHASE_FIX_REELOUT];
            const double a0 = (double)nkr / n_k / frac, a1 = (double)(n_k - nkr) / n_k / frac;
            trip.emplace_back(1, L.g_tf(), last, gcode(kKindConst, 0, 0, kidx(a0)));
            trip.emplace_back(2, L.g_tf(), last, gcode(kKindConst, 0, 0, kidx(a1)));
            trip.emplace_back(1, L.g_tf() + 1, last, gcode(kKindConst, 0, 0, kidx(-a0)));
            trip.emplace_back(2, L.g_tf() + 1, last, gcode(kKindConst, 0, 0, kidx(-a1)));
        }
    }
    if ((int)kc.size() > kMaxConst) return fail("internal: too many constant J entries");
    std::sort(trip.begin(), trip.end(), [](const auto& a, const auto& b) {
        return std::get<0>(a) != std::get<0>(b) ? std::get<0>(a) < std::get<0>(b) : std::get<1>(a) < std::get<1>(b);
    });
    for (size_t e = 1; e < trip.size(); ++e)
        if (std::get<0>(trip[e]) == std::get<0>(trip[e - 1]) && std::get<1>(trip[e]) == std::get<1>(trip[e - 1]))
            return fail("internal: duplicate J entry");
    T.colind.assign(L.n_v + 1, 0);
    T.row.resize(trip.size());
    for (size_t e = 0; e < trip.size(); ++e) {
        T.colind[std::get<0>(trip[e]) + 1]++;
        T.row[e] = std::get<1>(trip[e]);
    }
    for (int c = 0; c < L.n_v; ++c) T.colind[c + 1] += T.colind[c];
    std::vector<std::vector<std::pair<int, uint32_t>>> per(n_k);
    for (size_t e = 0; e < trip.size(); ++e) per[std::get<2>(trip[e])].emplace_back((int)e, std::get<3>(trip[e]));
    T.goff.assign(n_k + 1, 0);
    T.gslot.clear();
    T.gcode.clear();
    for (int k = 0; k < n_k; ++k) {
        for (auto& pe : per[k]) {
            T.gslot.push_back(pe.first);
            T.gcode.push_back(pe.second);
        }
        T.goff[k + 1] = (int)T.gslot.size();
    }
    return 0;
}

}  // namespace dlt
