// Host-side tables of the multi-kite Hessian kernel (awedual.hip, dual_hess_kernel): the exact
// Hessian of the Lagrangian sigma f + lam^T g (nlp_hess_l; awebox's default IPOPT setting
// hessian_approximation = 'exact', opts/default.py:323, preparation.py:272-273).  Plain C++.
//
// The design of the AP2 Hessian (ap2_tables.hpp, build_hess_tables) at the 127-direction node:
//   * a second-order dependency scalar (HDep2: first-order mask + per-variable second-order
//     masks over 128 inputs) run through dual_node gives, for every node row, the pairs of node
//     variables with a possibly nonzero mixed second derivative;
//   * the Jacobian colouring separates those rows, so a hyper-dual evaluation with e1 along
//     colour c1 and e2 along colour c2 gives, for each row r, d2F_r / dp dq where p, q are the
//     unique directions of c1, c2 that row r depends on: one (node, colour pair) task per thread
//     accumulates mu_r d2F_r into a compact direction-pair Hessian with no conflicts;
//   * two virtual directions carry the objective's global couplings that no node variable
//     seeds: phi.psi (tracking vs power homotopy) and, with single_reelout, the t_f of the
//     OTHER phase (the power cost is divided by the phase-fixed period T = n0 tf0 + n1 tf1,
//     ocp_outputs.py:118-140);
//   * a gather list maps direction pairs to the upper-triangular CCS of the V-space Hessian
//     (xdot directions of a Radau node feed every collocation column X_r with C[r][n]/(h tf)),
//     plus the second-order terms of xdot = C X / (h tf) in t_f (types B and C below).
#pragma once

#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "dual_tables.hpp"

namespace dlt {

// ---- structural second-order dependency over <= 128 node inputs (host only) -----------------
struct HDep2 {
    Mask d;
    Mask h[128];
    HDep2() = default;
    HDep2(double) {}
    static HDep2 var(int i) { HDep2 x; x.d.set(i); return x; }
};
inline void hdep2_cross(HDep2& r, const Mask& a, const Mask& b) {
    for (int i = 0; i < 128; ++i) {
        if (a.has(i)) r.h[i].merge(b);
        if (b.has(i)) r.h[i].merge(a);
    }
}
inline HDep2 hdep2_lin(const HDep2& x, const HDep2& y) {
    HDep2 r;
    r.d = x.d;
    r.d.merge(y.d);
    for (int i = 0; i < 128; ++i) { r.h[i] = x.h[i]; r.h[i].merge(y.h[i]); }
    return r;
}
inline HDep2 hdep2_nl(const HDep2& x) { HDep2 r = x; hdep2_cross(r, x.d, x.d); return r; }
inline HDep2 operator+(const HDep2& x, const HDep2& y) { return hdep2_lin(x, y); }
inline HDep2 operator-(const HDep2& x, const HDep2& y) { return hdep2_lin(x, y); }
inline HDep2 operator-(const HDep2& x) { return x; }
inline HDep2 operator*(const HDep2& x, const HDep2& y) { HDep2 r = hdep2_lin(x, y); hdep2_cross(r, x.d, y.d); return r; }
inline HDep2 operator/(const HDep2& x, const HDep2& y) {
    HDep2 r = hdep2_lin(x, y); hdep2_cross(r, x.d, y.d); hdep2_cross(r, y.d, y.d); return r;
}
inline HDep2 operator+(const HDep2& x, double) { return x; }
inline HDep2 operator+(double, const HDep2& y) { return y; }
inline HDep2 operator-(const HDep2& x, double) { return x; }
inline HDep2 operator-(double, const HDep2& y) { return y; }
inline HDep2 operator*(const HDep2& x, double) { return x; }
inline HDep2 operator*(double, const HDep2& y) { return y; }
inline HDep2 operator/(const HDep2& x, double) { return x; }
inline HDep2 operator/(double, const HDep2& y) { return hdep2_nl(y); }
inline HDep2 sqrt(const HDep2& x) { return hdep2_nl(x); }
inline HDep2 exp(const HDep2& x) { return hdep2_nl(x); }
inline HDep2 log(const HDep2& x) { return hdep2_nl(x); }

// Hessian directions: the 127 node directions (126 node variables + phi.gamma), then
constexpr int kHDirPsi = 127;        // phi.psi (objective only)
constexpr int kHDirTfOther = 128;    // t_f of the other phase (objective only, single_reelout)
constexpr int kHDirs = 129;
constexpr int kHRowStride = kNRows + 1;   // 76: row targets per task
constexpr int kHTypeA = 0, kHTypeB = 1, kHTypeC = 2;

// Gather term of one V-space Hessian entry (bits 31..30 type):
//   A: scl[sa] scl[sb] hd_n[pidx]                       n 27..29, pidx 14..26, sa 7..13, sb 0..6
//   B: G[n][i] (-C[r][n] n_k / tf^2)   (X_r,i ; t_f)    n 27..29, i 21..26, r 18..20
//   C: sum_i G[n][i] 2 xdot_i / tf^2   (t_f ; t_f)      n 27..29
// scl[0] = 1, scl[1 + r NN + n] = C[r][n] n_k / tf.
inline unsigned dterm_a(int n, int pidx, int sa, int sb) {
    return ((unsigned)kHTypeA << 30) | ((unsigned)n << 27) | ((unsigned)pidx << 14) | ((unsigned)sa << 7) | (unsigned)sb;
}
inline unsigned dterm_b(int n, int i, int r) {
    return ((unsigned)kHTypeB << 30) | ((unsigned)n << 27) | ((unsigned)i << 21) | ((unsigned)r << 18);
}
inline unsigned dterm_c(int n) { return ((unsigned)kHTypeC << 30) | ((unsigned)n << 27); }

struct DHessTabs {                           // device-visible part
    int npairs[2];                           // direction pairs per node kind
    int ntask[2];
    int task_off[2];                         // into the task list (c1 | c2 << 8)
    short pidx[2][kHDirs][kHDirs];           // compact index of the unordered direction pair, -1
    uint64_t dm_lo[2][128], dm_hi[2][128];   // rows of each direction (first-order masks)
};

struct DualHessTables {
    DHessTabs ht{};
    std::vector<int> tasks;
    std::vector<short> task_target;          // [task][kHRowStride]: pair index a row feeds, -1
    std::vector<int> colind, row;            // upper-triangular CCS of the V-space Hessian
    int nnz = 0;
    std::vector<int> slot0, nslot;           // [n_k] the interval's contiguous CCS range
    std::vector<int> gslot;                  // CCS slots of the global-global entries
    std::vector<int> gcol, grow;             // their (column, row)
    std::vector<int> ent_off;                // [n_k + 1] entries of each interval (local, then globals)
    std::vector<int> term_off;               // [n_entries + 1] into terms
    std::vector<unsigned> terms;
    int max_pairs = 0;
};

// V columns (with scale index) that direction `dir` of node `node` of interval k feeds
inline void dual_direction_columns(const Layout& L, int d, int k, int node, int dir,
                                   std::vector<std::pair<int, int>>& cols) {
    const int NN = d + 1;
    cols.clear();
    if (dir == kHDirPsi) { cols.emplace_back(L.phi(3), 0); return; }
    if (dir == kHDirTfOther) {
        if (L.single) cols.emplace_back(L.th_tf(k) == 1 ? 2 : 1, 0);
        return;
    }
    if (dir == awe::dl::kGamma) { cols.emplace_back(L.phi(0), 0); return; }
    if (dir >= 2 * ADL_NX + ADL_NU + ADL_NZ) {
        const int t = dir - (2 * ADL_NX + ADL_NU + ADL_NZ);
        cols.emplace_back(t == 0 ? L.th_diam_t() : t == 1 ? L.th_tf(k) : t == 2 ? L.th_ls() : L.th_diam_s(), 0);
        return;
    }
    if (dir >= 2 * ADL_NX && dir < 2 * ADL_NX + ADL_NU) { cols.emplace_back(L.u(k, dir - 2 * ADL_NX), 0); return; }
    if (dir >= 2 * ADL_NX + ADL_NU) {
        const int i = dir - (2 * ADL_NX + ADL_NU);
        cols.emplace_back(node == 0 ? L.z(k, i) : L.coll_z(k, node - 1, i), 0);
        return;
    }
    if (node == 0) {
        cols.emplace_back(dir < ADL_NX ? L.x(k, dir) : L.xdot(k, dir - ADL_NX), 0);
        return;
    }
    if (dir < ADL_NX) { cols.emplace_back(L.coll_x(k, node - 1, dir), 0); return; }
    for (int r = 0; r < NN; ++r)
        if (r != node) cols.emplace_back(L.X(k, r, dir - ADL_NX), 1 + r * NN + node);
}

inline int build_dual_hess_tables(const Tables& T, const double* consts, DualHessTables& H, std::string& err) {
    const Layout& L = T.lay;
    const ColorTabs& ct = T.ct;
    const int n_k = L.n_k, d = L.d, NN = d + 1;
    DHessTabs& ht = H.ht;
    std::memset(&ht, 0, sizeof(ht));
    std::memset(ht.pidx, 0xff, sizeof(ht.pidx));
    using awe::dl::kTf;

    // ---- second-order structure of every node row ------------------------------------------
    struct HSink {
        HDep2 rows[kNRows];
        void eq_row(int r, const HDep2& v) { rows[r] = v; }
        void ineq_row(int r, const HDep2& v) { rows[ADL_N_EQ + r] = v; }
        void power(const HDep2& v) { rows[kRowPower] = v; }
        void beta(int k, const HDep2& v) { rows[kRowBeta0 + k] = v; }
    };
    struct HIn { HDep2 operator()(int i) const { return HDep2::var(i); } };
    std::vector<double> th(AWE_NTHETA0, 1.0);
    auto* hs = new HSink();
    awe::dual_node<HDep2>(HIn{}, HDep2::var(awe::dl::kGamma), th.data(), consts, *hs, true);

    auto dvars = [&](int kind, int dir) {   // node variables a direction seeds
        Mask m;
        if (dir >= kDirs) return m;
        m.set(dir);
        if (kind == 1 && dir < ADL_NX) m.set(ADL_NX + dir);
        if (kind == 1 && dir == kTf)
            for (int i = 0; i < ADL_NX; ++i) m.set(ADL_NX + i);
        return m;
    };
    auto row_used = [&](int kind, int r) {
        if (kind == 0) return r < kRowPower;
        return r < ADL_N_EQ || r >= kRowPower;
    };
    auto interacts = [&](int r, const Mask& va, const Mask& vb) {
        for (int u = 0; u < 128; ++u)
            if (va.has(u) && hs->rows[r].h[u].meets(vb)) return true;
        return false;
    };
    std::vector<std::vector<std::pair<int, int>>> pairs(2);
    std::vector<std::vector<char>> has(2, std::vector<char>(kHDirs * kHDirs, 0));
    auto add_pair = [&](int kind, int p, int q) {
        if (p > q) std::swap(p, q);
        if (!has[kind][p * kHDirs + q]) { has[kind][p * kHDirs + q] = 1; pairs[kind].emplace_back(p, q); }
    };
    std::vector<int> task_set[2];
    for (int kind = 0; kind < 2; ++kind) {
        std::vector<Mask> dv(kDirs);
        for (int p = 0; p < kDirs; ++p) dv[p] = dvars(kind, p);
        std::vector<char> tk(kLanes * kLanes, 0);
        for (int r = 0; r < kNRows; ++r) {
            if (!row_used(kind, r)) continue;
            for (int p = 0; p < kDirs; ++p) {
                if (!T.dmask[kind][p].has(r)) continue;
                for (int q = p; q < kDirs; ++q) {
                    if (!T.dmask[kind][q].has(r) || !interacts(r, dv[p], dv[q])) continue;
                    const int cp = ct.col[kind][p], cq = ct.col[kind][q];
                    if (cp < 0 || cq < 0) {
                        err = "internal: Hessian structure outside the first-order pattern";
                        delete hs;
                        return 1;
                    }
                    add_pair(kind, p, q);
                    tk[std::min(cp, cq) * kLanes + std::max(cp, cq)] = 1;
                }
            }
        }
        for (int c1 = 0; c1 < kLanes; ++c1)
            for (int c2 = c1; c2 < kLanes; ++c2)
                if (tk[c1 * kLanes + c2]) task_set[kind].push_back(c1 | (c2 << 8));
    }
    delete hs;
    // objective terms at the Radau nodes (the kernel's objective pass; objective.py:45-544)
    {
        const int kind = 1;
        for (int i = 0; i < ADL_NX; ++i) {
            add_pair(kind, i, i);
            add_pair(kind, i, ADL_NX + i);
            add_pair(kind, i, kTf);
            add_pair(kind, ADL_NX + i, ADL_NX + i);
            add_pair(kind, ADL_NX + i, kTf);
            add_pair(kind, i, kHDirPsi);
        }
        add_pair(kind, kTf, kTf);
        for (int p = 2 * ADL_NX; p < ADL_NW; ++p) add_pair(kind, p, p);
        for (int p = 2 * ADL_NX + ADL_NU; p < 2 * ADL_NX + ADL_NU + ADL_NZ; ++p) add_pair(kind, p, kHDirPsi);
        std::vector<int> bdirs, pdirs;
        for (int p = 0; p < kDirs; ++p) {
            if (T.dmask[1][p].has(kRowBeta0) || T.dmask[1][p].has(kRowBeta0 + 1)) bdirs.push_back(p);
            if (T.dmask[1][p].has(kRowPower)) pdirs.push_back(p);
        }
        for (size_t a = 0; a < bdirs.size(); ++a)
            for (size_t b = a; b < bdirs.size(); ++b) add_pair(kind, bdirs[a], bdirs[b]);
        for (int p : pdirs) {
            add_pair(kind, p, kHDirPsi);
            add_pair(kind, p, kTf);
            if (L.single) add_pair(kind, p, kHDirTfOther);
        }
    }
    for (int kind = 0; kind < 2; ++kind) {
        std::sort(pairs[kind].begin(), pairs[kind].end());
        ht.npairs[kind] = (int)pairs[kind].size();
        if (ht.npairs[kind] >= 8192) { err = "internal: too many Hessian direction pairs"; return 1; }
        for (int i = 0; i < ht.npairs[kind]; ++i) {
            const int p = pairs[kind][i].first, q = pairs[kind][i].second;
            ht.pidx[kind][p][q] = ht.pidx[kind][q][p] = (short)i;
        }
        for (int dir = 0; dir < kDirs; ++dir) {
            ht.dm_lo[kind][dir] = T.dmask[kind][dir].lo;
            ht.dm_hi[kind][dir] = T.dmask[kind][dir].hi;
        }
        ht.task_off[kind] = (int)H.tasks.size();
        ht.ntask[kind] = (int)task_set[kind].size();
        H.tasks.insert(H.tasks.end(), task_set[kind].begin(), task_set[kind].end());
    }
    H.max_pairs = std::max(ht.npairs[0], ht.npairs[1]);
    // per task and row: the direction pair its mixed second derivative belongs to
    int pdir[2][kLanes][kNRows];
    std::memset(pdir, 0xff, sizeof(pdir));
    for (int kind = 0; kind < 2; ++kind)
        for (int dir = 0; dir < kDirs; ++dir) {
            const int c = ct.col[kind][dir];
            if (c < 0) continue;
            for (int r = 0; r < kNRows; ++r)
                if (T.dmask[kind][dir].has(r)) pdir[kind][c][r] = dir;
        }
    H.task_target.assign(H.tasks.size() * kHRowStride, (short)-1);
    for (int kind = 0; kind < 2; ++kind)
        for (int t = 0; t < ht.ntask[kind]; ++t) {
            const int task = H.tasks[ht.task_off[kind] + t], c1 = task & 0xff, c2 = task >> 8;
            for (int r = 0; r < kNRows; ++r) {
                if (!row_used(kind, r)) continue;
                const int p = pdir[kind][c1][r], q = pdir[kind][c2][r];
                if (p < 0 || q < 0) continue;
                H.task_target[(size_t)(ht.task_off[kind] + t) * kHRowStride + r] = ht.pidx[kind][p][q];
            }
        }

    // ---- V-space entries and their gather terms ----------------------------------------------
    auto is_global = [&](int col) { return col < L.v_int0; };
    std::vector<std::pair<long long, unsigned>> ent;   // (key = col * n_v + row, term)
    std::vector<int> ent_k;
    std::vector<std::pair<int, int>> ca, cb;
    for (int k = 0; k < n_k; ++k) {
        const int itf = L.th_tf(k);
        for (int node = 0; node < NN; ++node) {
            const int kind = node > 0;
            for (const auto& pq : pairs[kind]) {
                const int p = pq.first, q = pq.second;
                const int pi = ht.pidx[kind][p][q];
                dual_direction_columns(L, d, k, node, p, ca);
                dual_direction_columns(L, d, k, node, q, cb);
                for (size_t a = 0; a < ca.size(); ++a)
                    for (size_t b = (p == q ? a : 0); b < cb.size(); ++b) {
                        int r0 = ca[a].first, c0 = cb[b].first, sa = ca[a].second, sb = cb[b].second;
                        if (r0 > c0) { std::swap(r0, c0); std::swap(sa, sb); }
                        ent.emplace_back((long long)c0 * L.n_v + r0, dterm_a(node, pi, sa, sb));
                        ent_k.push_back(k);
                    }
            }
            if (node == 0) continue;
            for (int i = 0; i < ADL_NX; ++i)
                for (int r = 0; r < NN; ++r) {
                    ent.emplace_back((long long)L.X(k, r, i) * L.n_v + itf, dterm_b(node, i, r));
                    ent_k.push_back(k);
                }
            ent.emplace_back((long long)itf * L.n_v + itf, dterm_c(node));
            ent_k.push_back(k);
        }
    }
    // CCS pattern (upper triangle, column-major): plus the period-coupled global entries of the
    // power and time costs, (t_f_i, t_f_j) and (psi, t_f_i)
    std::vector<long long> keys;
    keys.reserve(ent.size() + 8);
    for (auto& e : ent) keys.push_back(e.first);
    const int ntf = L.single ? 2 : 1;
    for (int i = 0; i < ntf; ++i) {
        for (int j = i; j < ntf; ++j) keys.push_back((long long)(1 + j) * L.n_v + (1 + i));
        keys.push_back((long long)L.phi(3) * L.n_v + (1 + i));
    }
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
        for (int s = H.colind[c]; s < H.colind[c + 1]; ++s) {
            H.gslot.push_back(s);
            H.gcol.push_back(c);
            H.grow.push_back(H.row[s]);
        }
    const int ng = (int)H.gslot.size();
    H.slot0.resize(n_k);
    H.nslot.resize(n_k);
    for (int k = 0; k < n_k; ++k) {
        H.slot0[k] = H.colind[L.x(k, 0)];
        H.nslot[k] = (k == n_k - 1 ? H.nnz : H.colind[L.x(k + 1, 0)]) - H.slot0[k];
    }
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
            idx = (int)(std::find(H.gslot.begin(), H.gslot.end(), slot) - H.gslot.begin()) + H.nslot[k];
        } else {
            idx = slot - H.slot0[k];
            if (idx < 0 || idx >= H.nslot[k]) { err = "internal: Hessian entry outside its interval"; return 1; }
        }
        bucket[H.ent_off[k] + idx].push_back(ent[e].second);
    }
    H.term_off.assign(bucket.size() + 1, 0);
    for (size_t i = 0; i < bucket.size(); ++i) {
        H.term_off[i + 1] = H.term_off[i] + (int)bucket[i].size();
        H.terms.insert(H.terms.end(), bucket[i].begin(), bucket[i].end());
    }
    return 0;
}

}  // namespace dlt
