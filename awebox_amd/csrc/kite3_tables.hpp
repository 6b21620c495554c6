// Host-side tables of the tracking-MPC evaluator (3-DOF kite, awempc.hip).  Plain C++.
//
//   * the MPC NLP layout: V (var_struct.py:39-115) and g = [initial conditions (operation.py:
//     303-326)] + per interval [shooting 12, path 2, collocation d x 12, continuity 11]
//     (constraints.py:48-145, 210-373);
//   * structural row masks of the node model (kite3_node on the dependency-bitmask scalar);
//   * the CCS pattern of J_g and, per CCS slot, where its value comes from (gather list).
//
// Directions of the model pass (one lane each, 32 per node; no colouring is needed for 31
// node variables): at the shooting node, lane l seeds node variable l (31 = phi.gamma).  At a
// Radau node n, lane i < 11 seeds the state x_i together with xdot_i += C[n][n] / (h tf) (so it
// yields the derivative with respect to the collocation variable X_{n,i}), lanes 11..21 seed xdot_i
// alone (the derivative with respect to X_{r,i}, r != n, is that tangent times C[r][n] / (h tf)),
// lanes 22..29 seed u, z, diam_t, lane 30 seeds t_f through every xdot_i (-xdot_i / tf), lane 31
// seeds phi.gamma.
#pragma once

#include <algorithm>
#include <cstdint>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/awempc.h"
#include "ap2_tables.hpp"       // awt::Coll / make_coll / DevColl (radau coefficients)
#include "kite3_model.hpp"

namespace k3t {

constexpr int kLanes = 32;
constexpr int kRowsPerNode = K3_N_EQ + K3_N_INEQ;     // 14 (only the shooting node has ineq rows)
constexpr int kDirTf = 30, kDirGamma = 31;
// gather code: kind (bits 29..31) | r (25..28) | n (21..24) | tangent index (0..20)
constexpr uint32_t kKindTang = 0, kKindTangPoly = 1, kKindOne = 2, kKindMinusD = 3;

inline uint32_t code(uint32_t kind, int r, int n, int idx) {
    return (kind << 29) | ((uint32_t)r << 25) | ((uint32_t)n << 21) | (uint32_t)idx;
}
inline int tang_index(int n, int row, int lane) { return (n * kRowsPerNode + row) * kLanes + lane; }

struct Layout {
    int n_k = 0, d = 0, stride = 0, v_int0 = 0, n_v = 0, rows = 0, n_g = 0, n_p = 0;
    void init(int nk, int dd) {
        n_k = nk;
        d = dd;
        stride = K3_NX + K3_NU + K3_NX + K3_NZ + dd * (K3_NX + K3_NZ);
        v_int0 = K3_NTH + K3_NPHI + K3_NXI;
        n_v = v_int0 + nk * stride + K3_NX;
        rows = K3_N_EQ + K3_N_INEQ + dd * K3_N_EQ + K3_NX;
        n_g = K3_NX + nk * rows;
        n_p = K3_NX + n_v + 1 + K3_NX + K3_NU + K3_NX;
    }
    int x(int k, int i) const { return v_int0 + k * stride + i; }
    int u(int k, int i) const { return v_int0 + k * stride + K3_NX + i; }
    int xdot(int k, int i) const { return v_int0 + k * stride + K3_NX + K3_NU + i; }
    int z(int k) const { return v_int0 + k * stride + 2 * K3_NX + K3_NU; }
    int coll_x(int k, int j, int i) const {
        return v_int0 + k * stride + 2 * K3_NX + K3_NU + K3_NZ + j * (K3_NX + K3_NZ) + i;
    }
    int coll_z(int k, int j) const {
        return v_int0 + k * stride + 2 * K3_NX + K3_NU + K3_NZ + j * (K3_NX + K3_NZ) + K3_NX;
    }
    // X_{k,r}: r = 0 -> x[k], r >= 1 -> coll_x[k][r-1]
    int X(int k, int r, int i) const { return r == 0 ? x(k, i) : coll_x(k, r - 1, i); }
    int g_shoot(int k) const { return K3_NX + k * rows; }
    int g_coll(int k, int j) const { return K3_NX + k * rows + K3_N_EQ + K3_N_INEQ + j * K3_N_EQ; }
    int g_cont(int k) const { return K3_NX + k * rows + K3_N_EQ + K3_N_INEQ + d * K3_N_EQ; }
};

struct Tables {
    Layout lay;
    awt::Coll coll;
    uint32_t eq_mask[K3_N_EQ], ineq_mask[K3_N_INEQ];   // bits 0..30 node variables, 31 gamma
    std::vector<int> colind, row;                        // CCS of J_g
    std::vector<int> goff;                               // [n_k + 1] gather-list offsets per interval
    std::vector<int> gslot;                              // CCS slot
    std::vector<uint32_t> gcode;                         // value source
};

struct DepSink {
    awe::Dep eq[K3_N_EQ], ineq[K3_N_INEQ];
    void eq_row(int r, const awe::Dep& v) { eq[r] = v; }
    void ineq_row(int r, const awe::Dep& v) { ineq[r] = v; }
};
struct DepIn {
    awe::Dep operator()(int i) const { return awe::Dep::bit(i); }
};

inline int build_tables(int n_k, int d, const double* consts, int n_consts, Tables& T, std::string& err) {
    if (n_consts != K3_NCONST) { err = "consts must have K3_NCONST entries"; return 1; }
    if (n_k < 1 || d < 1 || d > 5) { err = "need n_k >= 1 and 1 <= d <= 5"; return 1; }
    T.lay.init(n_k, d);
    T.coll = awt::make_coll(d);
    {
        DepSink s;
        awe::kite3_node<awe::Dep>(DepIn{}, awe::Dep::bit(kDirGamma), 5.0, consts, s, true);
        for (int r = 0; r < K3_N_EQ; ++r) T.eq_mask[r] = (uint32_t)s.eq[r].m;
        for (int r = 0; r < K3_N_INEQ; ++r) T.ineq_mask[r] = (uint32_t)s.ineq[r].m;
    }
    const Layout& L = T.lay;
    const int NN = d + 1;
    constexpr uint32_t kXdotBits = ((1u << K3_NX) - 1u) << K3_NX;
    // triplets (col, row, owner interval, code)
    std::vector<std::tuple<int, int, int, uint32_t>> trip;
    auto add = [&](int col, int row, int owner, uint32_t c) { trip.emplace_back(col, row, owner, c); };
    for (int i = 0; i < K3_NX; ++i) add(L.x(0, i), i, 0, code(kKindOne, 0, 0, 0));   // initial rows
    for (int k = 0; k < n_k; ++k) {
        // ---- shooting node: rows g_shoot .. +13 (eq then ineq), directions = node variables
        for (int r = 0; r < kRowsPerNode; ++r) {
            const uint32_t m = r < K3_N_EQ ? T.eq_mask[r] : T.ineq_mask[r - K3_N_EQ];
            const int grow = L.g_shoot(k) + r;
            for (int l = 0; l < kLanes; ++l) {
                if (!((m >> l) & 1u)) continue;
                const uint32_t c = code(kKindTang, 0, 0, tang_index(0, r, l));
                if (l < K3_NX) add(L.x(k, l), grow, k, c);
                else if (l < 2 * K3_NX) add(L.xdot(k, l - K3_NX), grow, k, c);
                else if (l < 2 * K3_NX + K3_NU) add(L.u(k, l - 2 * K3_NX), grow, k, c);
                else if (l == 2 * K3_NX + K3_NU) add(L.z(k), grow, k, c);
                else if (l == kDirGamma) add(K3_NTH + 0, grow, k, c);       // phi.gamma
                else add(l - (2 * K3_NX + K3_NU + K3_NZ), grow, k, c);       // theta
            }
        }
        // ---- Radau nodes n = 1..d
        for (int n = 1; n < NN; ++n) {
            for (int r = 0; r < K3_N_EQ; ++r) {
                const uint32_t m = T.eq_mask[r];
                const int grow = L.g_coll(k, n - 1) + r;
                for (int i = 0; i < K3_NX; ++i) {
                    // own column X_{n,i}
                    if (((m >> i) & 1u) || ((m >> (K3_NX + i)) & 1u))
                        add(L.X(k, n, i), grow, k, code(kKindTang, 0, 0, tang_index(n, r, i)));
                    // the other polynomial columns X_{rr,i} through xdot_i
                    if ((m >> (K3_NX + i)) & 1u)
                        for (int rr = 0; rr < NN; ++rr)
                            if (rr != n)
                                add(L.X(k, rr, i), grow, k, code(kKindTangPoly, rr, n, tang_index(n, r, K3_NX + i)));
                }
                for (int j = 0; j < K3_NU; ++j)
                    if ((m >> (2 * K3_NX + j)) & 1u)
                        add(L.u(k, j), grow, k, code(kKindTang, 0, 0, tang_index(n, r, 2 * K3_NX + j)));
                if ((m >> (2 * K3_NX + K3_NU)) & 1u)
                    add(L.coll_z(k, n - 1), grow, k, code(kKindTang, 0, 0, tang_index(n, r, 2 * K3_NX + K3_NU)));
                if ((m >> 29) & 1u) add(0, grow, k, code(kKindTang, 0, 0, tang_index(n, r, 29)));      // diam_t
                if ((m & kXdotBits) || ((m >> kDirTf) & 1u))
                    add(1, grow, k, code(kKindTang, 0, 0, tang_index(n, r, kDirTf)));                 // t_f
                if ((m >> kDirGamma) & 1u) add(K3_NTH + 0, grow, k, code(kKindTang, 0, 0, tang_index(n, r, kDirGamma)));
            }
        }
        // ---- continuity x[k+1] - sum_r D_r X_{k,r}
        for (int i = 0; i < K3_NX; ++i) {
            const int grow = L.g_cont(k) + i;
            add(L.x(k + 1, i), grow, k, code(kKindOne, 0, 0, 0));
            for (int rr = 0; rr < NN; ++rr) add(L.X(k, rr, i), grow, k, code(kKindMinusD, rr, 0, 0));
        }
    }
    std::sort(trip.begin(), trip.end(), [](const auto& a, const auto& b) {
        return std::get<0>(a) != std::get<0>(b) ? std::get<0>(a) < std::get<0>(b) : std::get<1>(a) < std::get<1>(b);
    });
    for (size_t e = 1; e < trip.size(); ++e)
        if (std::get<0>(trip[e]) == std::get<0>(trip[e - 1]) && std::get<1>(trip[e]) == std::get<1>(trip[e - 1])) {
            err = "duplicate J entry";
            return 1;
        }
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

}  // namespace k3t
