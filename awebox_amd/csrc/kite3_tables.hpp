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

// =========================================================================================
// Hessian of the Lagrangian (nlp_hess_l of the MPC NLP, pmpc.py:193-217 with IPOPT's exact
// Hessian, default.py:323).  The constraints' second derivatives come from the node model in
// hyper-dual arithmetic, one task per direction pair (p, q) that is structurally nonzero (HDep over
// the 32 directions of the first-order pass, kite3 needs no colouring); the initial-condition and
// continuity rows are linear.  Directions map to V columns exactly as in the first-order gather
// list, so the V-space entry (a, b) of node n is s_a s_b Hdir_n(p_a, p_b) with s = 1 or the
// polynomial scale C[r][n] / (h tf); xdot's second-order dependence on t_f adds
// G_n,i d2 xdot_i / dV dV with G_n,i = sum_r mu_r dF_r / dxdot_i (first-order tasks, e2 = 0).
// The tracking cost (pmpc.py:304-358) is a diagonal quadratic in V.
// =========================================================================================
constexpr int kHTA = 0, kHTB = 1, kHTC = 2, kHTD = 3;   // term types (bits 31..30)
constexpr int kGTask = 255;                            // q of a first-order task
// A: scl[sa] scl[sb] hd_n[t]        n 27..29, t 14..26, sa 7..13, sb 0..6
// B: G_n,i (-C[r][n] / (h tf^2))     n, i 22..26, r 19..21        (t_f, X_{r,i})
// C: G_n,i 2 xdot_i / tf^2           n, i 22..26                   (t_f, t_f)
// D: sigma 2 (tracking weight)       n, sub 22..23 (0 coll x, 1 coll z, 2 u), i 17..21
inline unsigned hta(int n, int t, int sa, int sb) {
    return ((unsigned)kHTA << 30) | ((unsigned)n << 27) | ((unsigned)t << 14) | ((unsigned)sa << 7) | (unsigned)sb;
}
inline unsigned htb(int n, int i, int r) {
    return ((unsigned)kHTB << 30) | ((unsigned)n << 27) | ((unsigned)i << 22) | ((unsigned)r << 19);
}
inline unsigned htc(int n, int i) { return ((unsigned)kHTC << 30) | ((unsigned)n << 27) | ((unsigned)i << 22); }
inline unsigned htd(int n, int sub, int i) {
    return ((unsigned)kHTD << 30) | ((unsigned)n << 27) | ((unsigned)sub << 22) | ((unsigned)i << 17);
}

struct HessTables {
    int ntask[2] = {0, 0}, task_off[2] = {0, 0}, npair1 = 0;   // kind 1: npair1 pair tasks, then K3_NX G tasks
    std::vector<int> task;              // p | q << 8, per kind
    std::vector<int> colind, row;       // upper-triangular CCS of the V-space Hessian
    int nnz = 0;
    std::vector<int> slot0, nslot;      // [n_k] contiguous local slots of interval k
    std::vector<int> gslot;             // slots of the global-global entries (theta, phi)
    std::vector<int> xnslot;            // slots of the terminal (x[N], x[N]) diagonal
    std::vector<int> ent_off;           // [n_k + 1]: entries of interval k = nslot[k] local + globals
    std::vector<int> term_off;
    std::vector<unsigned> terms;
};

// node variables each direction seeds (shooting node: itself; Radau node: a state direction
// also moves its xdot, the t_f direction moves every xdot)
inline uint32_t hdir_vars(int kind, int dir) {
    if (dir == kGTask) return 0u;
    if (kind == 0) return 1u << dir;
    if (dir < K3_NX) return (1u << dir) | (1u << (K3_NX + dir));
    if (dir == kDirTf) return ((1u << K3_NX) - 1u) << K3_NX;
    return 1u << dir;
}

// V columns (with scale index: 0 -> 1, 1 + r NN + n -> C[r][n] / (h tf)) direction `dir` of node
// `n` of interval k feeds (the first-order gather list's columns)
inline void hdir_columns(const Layout& L, int k, int n, int dir, std::vector<std::pair<int, int>>& cols) {
    const int NN = L.d + 1;
    cols.clear();
    if (dir == kDirGamma) { cols.emplace_back(K3_NTH + 0, 0); return; }
    if (dir >= 2 * K3_NX + K3_NU + K3_NZ) { cols.emplace_back(dir - (2 * K3_NX + K3_NU + K3_NZ), 0); return; }
    if (dir >= 2 * K3_NX && dir < 2 * K3_NX + K3_NU) { cols.emplace_back(L.u(k, dir - 2 * K3_NX), 0); return; }
    if (n == 0) {
        if (dir < K3_NX) cols.emplace_back(L.x(k, dir), 0);
        else if (dir < 2 * K3_NX) cols.emplace_back(L.xdot(k, dir - K3_NX), 0);
        else cols.emplace_back(L.z(k), 0);
        return;
    }
    if (dir < K3_NX) { cols.emplace_back(L.coll_x(k, n - 1, dir), 0); return; }
    if (dir < 2 * K3_NX) {
        for (int r = 0; r < NN; ++r)
            if (r != n) cols.emplace_back(L.X(k, r, dir - K3_NX), 1 + r * NN + n);
        return;
    }
    cols.emplace_back(L.coll_z(k, n - 1), 0);
}

}  // namespace k3t

namespace awt {
inline HDep sin(const HDep& x) { return hdep_nl(x); }
inline HDep cos(const HDep& x) { return hdep_nl(x); }
}  // namespace awt

namespace k3t {

inline int build_hess_tables(const Tables& T, const double* consts, HessTables& H, std::string& err) {
    const Layout& L = T.lay;
    const int n_k = L.n_k, d = L.d, NN = d + 1;
    struct HSink {
        awt::HDep rows[kRowsPerNode];
        void eq_row(int r, const awt::HDep& v) { rows[r] = v; }
        void ineq_row(int r, const awt::HDep& v) { rows[K3_N_EQ + r] = v; }
    };
    struct HIn { awt::HDep operator()(int i) const { return awt::HDep::var(i); } };
    HSink hs;
    awe::kite3_node<awt::HDep>(HIn{}, awt::HDep::var(kDirGamma), 5.0, consts, hs, true);
    auto interacts = [&](int r, uint32_t va, uint32_t vb) {
        for (int u = 0; u < 32; ++u)
            if (((va >> u) & 1u) && (hs.rows[r].h[u] & (unsigned long long)vb)) return true;
        return false;
    };
    H.task.clear();
    for (int kind = 0; kind < 2; ++kind) {
        H.task_off[kind] = (int)H.task.size();
        const int nrows = kind == 0 ? kRowsPerNode : K3_N_EQ;
        for (int p = 0; p < kLanes; ++p)
            for (int q = p; q < kLanes; ++q) {
                const uint32_t vp = hdir_vars(kind, p), vq = hdir_vars(kind, q);
                bool nz = false;
                for (int r = 0; r < nrows && !nz; ++r) nz = interacts(r, vp, vq);
                if (nz) H.task.push_back(p | (q << 8));
            }
        if (kind == 1) {
            H.npair1 = (int)H.task.size() - H.task_off[1];
            for (int i = 0; i < K3_NX; ++i) H.task.push_back((K3_NX + i) | (kGTask << 8));
        }
        H.ntask[kind] = (int)H.task.size() - H.task_off[kind];
    }
    if (H.ntask[0] >= 8192 || H.ntask[1] >= 8192) { err = "internal: too many Hessian tasks"; return 1; }

    // ---- V-space entries and their terms -------------------------------------------------------
    const int itf = 1;                                  // V index of theta.t_f
    std::vector<std::pair<long long, unsigned>> ent;    // (key = col n_v + row, term)
    std::vector<int> ent_k;
    std::vector<std::pair<int, int>> ca, cb;
    auto add = [&](int k, int r0, int c0, unsigned term) {
        if (r0 > c0) std::swap(r0, c0);
        ent.emplace_back((long long)c0 * L.n_v + r0, term);
        ent_k.push_back(k);
    };
    for (int k = 0; k < n_k; ++k) {
        for (int n = 0; n < NN; ++n) {
            const int kind = n > 0;
            const int np = kind == 0 ? H.ntask[0] : H.npair1;
            for (int t = 0; t < np; ++t) {
                const int pq = H.task[H.task_off[kind] + t], p = pq & 0xff, q = pq >> 8;
                hdir_columns(L, k, n, p, ca);
                hdir_columns(L, k, n, q, cb);
                for (size_t a = 0; a < ca.size(); ++a)
                    for (size_t b = (p == q ? a : 0); b < cb.size(); ++b) {
                        int r0 = ca[a].first, c0 = cb[b].first, sa = ca[a].second, sb = cb[b].second;
                        if (r0 > c0) { std::swap(r0, c0); std::swap(sa, sb); }
                        add(k, r0, c0, hta(n, t, sa, sb));
                    }
            }
            if (n == 0) continue;
            for (int i = 0; i < K3_NX; ++i) {
                for (int r = 0; r < NN; ++r) add(k, itf, L.X(k, r, i), htb(n, i, r));
                add(k, itf, itf, htc(n, i));
                add(k, L.coll_x(k, n - 1, i), L.coll_x(k, n - 1, i), htd(n, 0, i));
            }
            add(k, L.coll_z(k, n - 1), L.coll_z(k, n - 1), htd(n, 1, 0));
        }
        for (int i = 0; i < K3_NU; ++i) add(k, L.u(k, i), L.u(k, i), htd(0, 2, i));
    }
    std::vector<long long> keys;
    keys.reserve(ent.size() + K3_NX);
    for (auto& e : ent) keys.push_back(e.first);
    for (int i = 0; i < K3_NX; ++i) keys.push_back((long long)L.x(n_k, i) * L.n_v + L.x(n_k, i));   // terminal cost
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
    auto slot_of = [&](long long key) { return (int)(std::lower_bound(keys.begin(), keys.end(), key) - keys.begin()); };
    H.gslot.clear();
    for (int c = 0; c < L.v_int0; ++c)
        for (int s = H.colind[c]; s < H.colind[c + 1]; ++s) H.gslot.push_back(s);
    H.xnslot.clear();
    for (int i = 0; i < K3_NX; ++i) H.xnslot.push_back(slot_of((long long)L.x(n_k, i) * L.n_v + L.x(n_k, i)));
    const int ng = (int)H.gslot.size();
    H.slot0.resize(n_k);
    H.nslot.resize(n_k);
    for (int k = 0; k < n_k; ++k) {
        H.slot0[k] = H.colind[L.x(k, 0)];
        H.nslot[k] = H.colind[L.x(k + 1, 0)] - H.slot0[k];
    }
    // every x[N] slot is a terminal diagonal entry (finalize kernel)
    if (H.colind[L.n_v] - H.colind[L.x(n_k, 0)] != K3_NX) { err = "internal: x[N] Hessian columns"; return 1; }
    std::vector<std::vector<unsigned>> bucket;
    H.ent_off.assign(n_k + 1, 0);
    for (int k = 0; k < n_k; ++k) H.ent_off[k + 1] = H.ent_off[k] + H.nslot[k] + ng;
    bucket.resize(H.ent_off[n_k]);
    for (size_t e = 0; e < ent.size(); ++e) {
        const int k = ent_k[e];
        const int slot = slot_of(ent[e].first);
        const int col = (int)(ent[e].first / L.n_v);
        int idx;
        if (col < L.v_int0) {
            idx = (int)(std::find(H.gslot.begin(), H.gslot.end(), slot) - H.gslot.begin()) + H.nslot[k];
        } else {
            idx = slot - H.slot0[k];
            if (idx < 0 || idx >= H.nslot[k]) { err = "internal: Hessian entry outside its interval"; return 1; }
        }
        bucket[H.ent_off[k] + idx].push_back(ent[e].second);
    }
    H.term_off.assign(bucket.size() + 1, 0);
    H.terms.clear();
    for (size_t i = 0; i < bucket.size(); ++i) {
        H.term_off[i + 1] = H.term_off[i] + (int)bucket[i].size();
        H.terms.insert(H.terms.end(), bucket[i].begin(), bucket[i].end());
    }
    return 0;
}

}  // namespace k3t
