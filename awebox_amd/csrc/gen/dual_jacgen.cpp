// Build-time generator of the dual-kite node-Jacobian code (awebox_amd/csrc/dual_nodejac.gen.hpp).
//
//   dual_jacgen <consts file> <output header>
//
// Traces dual_node (dual_model.hpp) on the symbolic scalar of gen/sym.hpp for the two node kinds of
// the collocation scheme (shooting node: 53 model equalities + 19 path inequalities; Radau node: 53
// equalities + the power integrand and the two side slips the objective needs), differentiates the
// tape along the 127 seed directions of dual_tables.hpp (at a Radau node direction i < 50 seeds x_i
// and xdot_i = C[n][n] / (h t_f), direction 50 + i seeds xdot_i, direction 123 carries d/d t_f through
// every xdot_i = -xdot_i / t_f, direction 126 is phi.gamma), and writes one straight-line function
// per kind that stores the node's row values and every entry of the first-order pattern
// (Tables::dmask), plus the table that maps (row, direction) to the tangent slot.  At the Radau node
// it also stores the power and side-slip values and the directional derivatives of the node's beta
// and power objective terms ex2 (beta_2^2 + beta_3^2) + ex3 p (objective.py:390-421, the (1 - psi)
// power cost over the phase-fixed period).  This is what CasADi's SX jacobian + code generation
// produce for the reference's nlp_jac_g of the dual-kite NLP (preparation.py:366-400,
// examples/dual_kites_power_curve.py), restricted to one node.
//
// The parameters theta0 and the model constants enter as run-time loads (th[i], cst[i]); only the
// integer structure read from them (tether elements, stability-derivative table lengths) is fixed at
// generation time and written out, so that adl_create can check it.
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../dual_tables.hpp"
#include "sym.hpp"

namespace {

using awe::Op;
using awe::Sym;
using namespace dlt;

constexpr int kRows = kRowPower;              // 72 rows with tangent slots: 53 eq + 19 ineq

struct RowSink {
    int rows[kNRows];
    RowSink() { for (int& r : rows) r = -1; }
    void eq_row(int r, const Sym& v) { rows[r] = v.id; }
    void ineq_row(int r, const Sym& v) { rows[ADL_N_EQ + r] = v.id; }
    void power(const Sym& v) { rows[kRowPower] = v.id; }
    void beta(int k, const Sym& v) { rows[kRowBeta0 + k] = v.id; }
};

struct SymIn {
    const Sym* w;
    Sym operator()(int i) const { return w[i]; }
};

struct KindOut {
    std::vector<std::string> group;          // one function body per row group
    std::vector<awe::EmitStats> group_stats;
    awe::EmitStats st;
    std::vector<short> tan_idx;   // [kRows][kDirs]
};

// Row groups: the node's outputs split by kite -- group k (0, 1) takes kite k's rows (DCM,
// rotation, translation and holonomic rows of its secondary tether, its path inequalities, its side
// slip), group 2 the rest (node 1's translation and the main holonomic row, the trivial kinematics,
// anticollision, the power integrand).  Each group is its own function body that recomputes the
// values it needs, so that three wavefronts evaluate one node side by side and each keeps about one
// kite's working set in registers (one body for all rows peaks at ~490 live doubles).
constexpr int kGroups = 7;
const bool kSplitKites = std::getenv("AWE_DUAL_SPLIT_KITES") != nullptr;
int row_group(int r) {
    using namespace awe::dl;
    if (r < 0) return 2;
    for (int k = 0; k < ADL_NKITES; ++k) {
        if (r >= ADL_N_EQ) {
            const int q = r - ADL_N_EQ;
            if (q == irow_force(k) || q == irow_force(k) + 1 || q == irow_airspeed(k) || q == irow_airspeed(k) + 1 ||
                (q >= irow_valid(k) && q < irow_valid(k) + 4) || q == irow_yaw(k))
                return k;
            continue;
        }
        if ((r >= row_trans(k) && r < row_trans(k) + 3) || r == row_hol(k) || (r >= row_rot(k) && r < row_rot(k) + 3) ||
            (r >= row_dcm(k) && r < row_dcm(k) + 9))
            return k;
    }
    return r < ADL_N_EQ && r >= kRowTrans1 && r < kRowTrans1 + 3 ? 2 : 3;
}

std::vector<int> ko_dbp_dirs;     // directions of the Radau node's dbp entries, in order

// traces the node (kite 3 first when first_kite = 1) and emits the bodies of the row groups `want`
KindOut generate(int kind, const std::vector<double>& cst, const Tables& T, int first_kite, const std::vector<int>& want,
                 int slot_base_in) {
    awe::Tape tape;
    awe::active_tape() = &tape;
    std::vector<Sym> w(kDirs), th(AWE_NTHETA0), cs(cst.size());
    for (int i = 0; i < kDirs; ++i) w[i] = Sym::of(tape.leaf(Op::Input, i));
    for (int i = 0; i < AWE_NTHETA0; ++i) th[i] = Sym::of(tape.leaf(Op::Th, i));
    for (size_t i = 0; i < cst.size(); ++i) cs[i] = Sym::of(tape.leaf(Op::Cs, (int)i, cst[i]));
    const int ex_cxx = tape.leaf(Op::Extra, 0), ex_inv_tf = tape.leaf(Op::Extra, 1);
    RowSink sink;
    awe::dual_node<Sym>(SymIn{w.data()}, w[awe::dl::kGamma], th.data(), cs.data(), sink, kind == 0,
                        awe::DualInlineSubmodels(), first_kite);
    // the Radau node's objective terms, one per row group: ex2 beta_2^2, ex2 beta_3^2, ex3 p
    int objt[kGroups] = {-1, -1, -1, -1, -1, -1, -1};
    if (kind == 1) {
        const Sym cb = Sym::of(tape.leaf(Op::Extra, 2)), cpp = Sym::of(tape.leaf(Op::Extra, 3));
        for (int k = 0; k < ADL_NKITES; ++k) {
            const Sym bk = Sym::of(sink.rows[kRowBeta0 + k]);
            objt[k] = (cb * (bk * bk)).id;
        }
        objt[3] = (cpp * Sym::of(sink.rows[kRowPower])).id;
    }
    const int n0 = (int)tape.n.size();
    const int one = tape.cnst(1.0);
    auto seed = [&](int i) -> awe::SparseGrad {
        if (kind == 1 && i >= ADL_NX && i < 2 * ADL_NX) {
            // xdot_s = sum_r C[r][n] X_r / (h t_f): d/d(dir s) = C[n][n] / (h t_f), d/d(dir 50 + s) = 1,
            // d/d t_f = -xdot_s / t_f
            const int s = i - ADL_NX;
            const int dtf = tape.mul(tape.neg(w[i].id), ex_inv_tf);
            return {{s, ex_cxx}, {i, one}, {awe::dl::kTf, dtf}};
        }
        return {{i, one}};
    };
    std::vector<awe::SparseGrad> G = awe::forward_grads(tape, n0, seed);

    const int nrows = kind == 0 ? kRows : ADL_N_EQ;
    std::vector<awe::Store> stores;
    const int zero = tape.cnst(0.0);
    for (int r = 0; r < nrows; ++r) {
        const int v = sink.rows[r];
        if (v < 0) { std::fprintf(stderr, "row %d not produced\n", r); std::exit(1); }
        stores.push_back({v, 0, r, -1});
        for (auto& e : G[v])
            if (!T.dmask[kind][e.first].has(r)) {
                std::fprintf(stderr, "kind %d row %d: derivative along direction %d outside the pattern\n", kind, r,
                             e.first);
                std::exit(1);
            }
        for (int dir = 0; dir < kDirs; ++dir) {
            if (!T.dmask[kind][dir].has(r)) continue;
            int node = zero;
            for (auto& e : G[v]) if (e.first == dir) node = e.second;
            stores.push_back({node, 1, r, dir});
        }
    }
    std::vector<int> store_group;                  // row group of every store
    for (auto& st : stores) store_group.push_back(row_group(st.row));
    // tangents of a group split in two direction ranges of equal counts: node 1's translation rows
    // (group 2 -> 2, 4), and with kSplitKites each kite's rows (0 -> 0, 5; 1 -> 1, 6)
    auto split = [&](int from, int to) {
        std::vector<int> per_dir(kDirs, 0);
        int total = 0;
        for (size_t i = 0; i < stores.size(); ++i)
            if (store_group[i] == from && stores[i].kind == 1) { per_dir[stores[i].dir]++; total++; }
        std::vector<int> half(kDirs, 0);
        for (int dir = 0, acc = 0; dir < kDirs; ++dir) { half[dir] = 2 * acc >= total; acc += per_dir[dir]; }
        for (size_t i = 0; i < stores.size(); ++i)
            if (store_group[i] == from && stores[i].kind == 1 && half[stores[i].dir]) store_group[i] = to;
    };
    split(2, 4);
    if (kSplitKites) {
        split(0, 5);
        split(1, 6);
    }
    if (kind == 1) {   // power and side slips (obv), tangents of the node's objective terms (dbp)
        stores.push_back({sink.rows[kRowPower], 3, 0, -1});
        store_group.push_back(3);
        for (int k = 0; k < ADL_NKITES; ++k) {
            stores.push_back({sink.rows[kRowBeta0 + k], 3, 1 + k, -1});
            store_group.push_back(k);
        }
        for (int grp : want) {
            if (objt[grp] < 0) continue;
            std::vector<std::pair<int, int>> dg(G[objt[grp]].begin(), G[objt[grp]].end());
            std::sort(dg.begin(), dg.end());
            for (auto& e : dg) {
                if (e.first >= awe::dl::kGamma) continue;   // phi.gamma: no beta / power dependence
                stores.push_back({e.second, 2, -1, (int)ko_dbp_dirs.size()});
                store_group.push_back(grp);
                ko_dbp_dirs.push_back(e.first);
            }
        }
    }
    KindOut ko;
    ko.tan_idx.assign(kRows * kDirs, -1);
    ko.group.assign(kGroups, std::string());
    ko.group_stats.assign(kGroups, awe::EmitStats());
    int slot_base = slot_base_in;
    for (int grp : want) {
        std::vector<awe::Store> part;
        for (size_t i = 0; i < stores.size(); ++i)
            if (store_group[i] == grp) part.push_back(stores[i]);
        awe::EmitStats st;
        const int before = slot_base;
        ko.group[grp] = awe::emit(tape, part, st, true, 32, false, slot_base);
        ko.group_stats[grp] = st;
        slot_base = before + st.n_tan;
        ko.st.ops += st.ops; ko.st.flops += st.flops; ko.st.transcendental += st.transcendental;
        ko.st.loads += st.loads; ko.st.n_tan += st.n_tan; ko.st.n_zero_tan += st.n_zero_tan;
        ko.st.max_live = std::max(ko.st.max_live, st.max_live);
        for (auto& s : part)
            if (s.kind == 1) ko.tan_idx[s.row * kDirs + s.dir] = (short)s.slot;
    }
    awe::active_tape() = nullptr;
    return ko;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: dual_jacgen <consts file> <output header>\n");
        return 2;
    }
    std::vector<double> cst;
    {
        std::ifstream f(argv[1]);
        double x;
        while (f >> x) cst.push_back(x);
    }
    if ((int)cst.size() != ADL_NCONST) {
        std::fprintf(stderr, "expected %d constants, read %zu\n", ADL_NCONST, cst.size());
        return 2;
    }
    Tables T;
    std::string err;
    if (build_tables((int)cst[ADL_C_N_K], (int)cst[ADL_C_D], cst.data(), (int)cst.size(), T, err)) {
        std::fprintf(stderr, "tables: %s\n", err.c_str());
        return 1;
    }
    // groups 0 and 2 from the trace in the model's order, group 1 (kite 3) from the trace with kite 3
    // first; slots numbered group after group, dbp entries kite 2, node 1, kite 3
    auto gen_kind = [&](int kind) {
        KindOut a = generate(kind, cst, T, 0, {0, 5}, 0);
        const int na = a.group_stats[0].n_tan + a.group_stats[5].n_tan;
        KindOut c = generate(kind, cst, T, 1, {1, 6}, na);
        const int nc = c.group_stats[1].n_tan + c.group_stats[6].n_tan;
        KindOut b = generate(kind, cst, T, 0, {2, 4, 3}, na + nc);
        KindOut o = a;
        for (KindOut* x : {&c, &b})
            for (int g = 0; g < kGroups; ++g)
                if (!x->group[g].empty()) { o.group[g] = x->group[g]; o.group_stats[g] = x->group_stats[g]; }
        for (int i = 0; i < kRows * kDirs; ++i) {
            if (c.tan_idx[i] >= 0) o.tan_idx[i] = c.tan_idx[i];
            if (b.tan_idx[i] >= 0) o.tan_idx[i] = b.tan_idx[i];
        }
        o.st = awe::EmitStats();
        for (int g = 0; g < kGroups; ++g) {
            const awe::EmitStats& st = o.group_stats[g];
            o.st.ops += st.ops; o.st.flops += st.flops; o.st.transcendental += st.transcendental;
            o.st.loads += st.loads; o.st.n_tan += st.n_tan; o.st.n_zero_tan += st.n_zero_tan;
            o.st.max_live = std::max(o.st.max_live, st.max_live);
        }
        return o;
    };
    KindOut ks = gen_kind(0), kr = gen_kind(1);
    // wavefront roles: kite 2's rows, kite 3's rows, node 1's translation rows along the first half
    // of their directions, then the second half and the remaining rows (groups 4 and 3, each in its
    // own scope: both come from one trace, so their statement names repeat)
    const std::vector<std::vector<int>> role_groups =
        kSplitKites ? std::vector<std::vector<int>>{{0}, {5}, {1}, {6}, {2}, {4, 3}}
                    : std::vector<std::vector<int>>{{0}, {1}, {2}, {4, 3}};
    auto bodies = [&](const KindOut& k) {
        std::string b;
        for (size_t r = 0; r < role_groups.size(); ++r) {
            b += std::string(r ? "    else " : "    ") + "if constexpr (G == " + std::to_string(r) + ") {\n";
            for (int g : role_groups[r]) b += "    {\n" + k.group[g] + "    }\n";
            b += "    }\n";
        }
        return b;
    };
    auto role_ops = [&](const KindOut& k, size_t r) {
        int ops = 0;
        for (int g : role_groups[r]) ops += k.group_stats[g].ops;
        return ops;
    };

    std::ostringstream o;
    o << "// GENERATED by awebox_amd/csrc/gen/dual_jacgen.cpp from dual_model.hpp -- do not edit.\n"
         "// Straight-line value + sparse forward-mode Jacobian of one dual-kite collocation node along\n"
         "// the evaluator's 127 seed directions (see the generator's header comment).\n"
         "#pragma once\n\n#include \"scalar.hpp\"\n\n"
         "// scheduling fence: keeps the register allocator to the emitted (pressure-scheduled) order\n"
         "#if defined(__HIP_DEVICE_COMPILE__)\n#define AWE_GEN_FENCE() __builtin_amdgcn_sched_barrier(0)\n"
         "#else\n#define AWE_GEN_FENCE() ((void)0)\n#endif\n\nnamespace awe_dgen {\n\n";
    o << "// integer structure of the model constants the code was generated for (adl_create checks it)\n";
    o << "constexpr int kNElements = " << (int)cst[ADL_C_N_ELEMENTS] << ";\n";
    o << "constexpr int kSdLen[54] = {";
    for (int i = 0; i < 54; ++i) o << (i ? ", " : "") << (int)cst[ADL_C_SD_LEN + i];
    o << "};\n";
    o << "// tangent slots per node kind (0 shooting, 1 Radau): one per J_g pattern entry of the node's rows\n";
    o << "constexpr int kNTan[2] = {" << ks.st.n_tan << ", " << kr.st.n_tan << "};\n";
    o << "// algorithmic operations per node kind: adds/muls/reciprocals, transcendental calls\n";
    o << "constexpr int kFlops[2] = {" << ks.st.flops << ", " << kr.st.flops << "};\n";
    o << "constexpr int kTranscendental[2] = {" << ks.st.transcendental << ", " << kr.st.transcendental << "};\n";
    o << "// dbp[i] of the Radau node is the derivative along seed direction kDbpDir[i]\n";
    o << "constexpr int kNDbp = " << ko_dbp_dirs.size() << ";\n";
    o << "constexpr int kDbpDir[" << std::max<size_t>(1, ko_dbp_dirs.size()) << "] = {";
    for (size_t i = 0; i < ko_dbp_dirs.size(); ++i) o << (i ? ", " : "") << ko_dbp_dirs[i];
    o << "};\n";
    std::vector<int> th_row(AWE_NTHETA0, -1);
    int n_th = 0;
    std::vector<const std::string*> all_bodies;
    for (const KindOut* k : {&ks, &kr})
        for (auto& b : k->group) all_bodies.push_back(&b);
    for (const std::string* b : all_bodies)
        for (size_t p = b->find("th["); p != std::string::npos; p = b->find("th[", p + 3)) {
            if (p > 0 && (std::isalnum((unsigned char)(*b)[p - 1]) || (*b)[p - 1] == '_')) continue;
            const int i = std::atoi(b->c_str() + p + 3);
            if (i >= 0 && i < AWE_NTHETA0 && th_row[i] < 0) th_row[i] = 0;
        }
    for (int i = 0; i < AWE_NTHETA0; ++i) if (th_row[i] == 0) th_row[i] = n_th++;
    o << "// theta0 entries read by the node code: kThRow[i] is the compact row of th[i] (-1: unused)\n";
    o << "constexpr int kNThUsed = " << n_th << ";\n";
    o << "constexpr short kThRow[" << AWE_NTHETA0 << "] = {";
    for (int i = 0; i < AWE_NTHETA0; ++i) o << (i ? "," : "") << th_row[i];
    o << "};\n";
    o << "// tangent slot of (row, direction), -1 outside the pattern\n";
    o << "constexpr short kTanIdx[2][" << kRows << "][" << kDirs << "] = {\n";
    for (const KindOut* k : {&ks, &kr}) {
        o << "  {\n";
        for (int r = 0; r < kRows; ++r) {
            o << "    {";
            for (int d = 0; d < kDirs; ++d) o << (d ? "," : "") << k->tan_idx[r * kDirs + d];
            o << "},\n";
        }
        o << "  },\n";
    }
    o << "};\n\n";
    o << "// shooting node: val[0..71] = 53 equalities + 19 path inequalities\n";
    o << "// in(i): node variable i (126 = phi.gamma); th[i] theta0; tan[s]: an accessor that sends slot s\n"
         "// to its J_g entries\n";
    o << "// G: wavefront role (0, 1: the rows of kite 2, 3 of the architecture; 2, 3: node 1's translation rows\n"
         "// along two halves of their directions; 3 also the main holonomic and trivial rows, anticollision, power)\n";
    o << "constexpr int kRoles = " << role_groups.size() << ";\n";
    o << "// generated operations per (node kind, role)\n";
    o << "constexpr int kRoleOps[2][" << role_groups.size() << "] = {";
    for (const KindOut* k : {&ks, &kr}) {
        o << (k == &ks ? "{" : ", {");
        for (size_t r = 0; r < role_groups.size(); ++r) o << (r ? ", " : "") << role_ops(*k, r);
        o << "}";
    }
    o << "};\n";
    o << "template <int TS, int G, class In, class Th, class Val, class Tan>\nAWE_HD void dual_node_shoot(const In& in, "
         "Th th, const double* __restrict__ cst, Val val, Tan tan) {\n";
    o << bodies(ks) << "}\n\n";
    o << "// Radau node: val[0..52] equalities; obv[0] power integrand, obv[1], obv[2] side slips;\n";
    o << "// dbp[i] = directional derivative of ex2 (beta_2^2 + beta_3^2) + ex3 power along kDbpDir[i];\n";
    o << "// ex0 = C[n][n] / (h t_f), ex1 = 1 / t_f\n";
    o << "template <int TS, int G, class In, class Th, class Val, class Tan, class Dbp, class Obv>\n"
         "AWE_HD void dual_node_radau(const In& in, const double ex0, const double ex1, const double ex2, "
         "const double ex3, Th th, const double* __restrict__ cst, Val val, Tan tan, Dbp dbp, Obv obv) {\n";
    o << bodies(kr) << "}\n\n}  // namespace awe_dgen\n";

    std::ofstream out(argv[2]);
    out << o.str();
    std::printf("{\"shooting\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"tangents\": %d, \"zero\": %d, "
                "\"max_live\": %d}, \"radau\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"tangents\": %d, "
                "\"zero\": %d, \"max_live\": %d}, \"dbp\": %zu, \"theta0_used\": %d}\n",
                ks.st.ops, ks.st.flops, ks.st.transcendental, ks.st.n_tan, ks.st.n_zero_tan, ks.st.max_live, kr.st.ops,
                kr.st.flops, kr.st.transcendental, kr.st.n_tan, kr.st.n_zero_tan, kr.st.max_live, ko_dbp_dirs.size(),
                n_th);
    for (const KindOut* k : {&ks, &kr})
        for (int g = 0; g < kGroups; ++g)
            std::printf("{\"kind\": %d, \"group\": %d, \"ops\": %d, \"tangents\": %d, \"max_live\": %d}\n",
                        k == &kr, g, k->group_stats[g].ops, k->group_stats[g].n_tan, k->group_stats[g].max_live);
    return 0;
}
