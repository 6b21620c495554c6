// Build-time generator of the tracking-MPC node-Jacobian code (awebox_amd/csrc/kite3_nodejac.gen.hpp).
//
//   kite3_jacgen <consts file> <output header>
//
// Traces kite3_node (kite3_model.hpp) on the symbolic scalar of gen/sym.hpp for the two node kinds
// of the MPC's collocation scheme (shooting node: 12 model equalities + 2 path inequalities; Radau
// node: 12 equalities), differentiates the tape along the 32 seed directions of the first-order pass
// (kite3_tables.hpp: at a Radau node direction i < 11 seeds x_i and xdot_i += C[n][n] / (h t_f),
// direction 11 + i seeds xdot_i alone, direction 30 carries d/d t_f through every xdot_i = -xdot_i / t_f,
// direction 31 is phi.gamma), and writes one straight-line function per kind that stores the node's
// row values and every entry of the J_g pattern build_tables derives (structural zeros included), plus
// the table mapping (row, direction) to the tangent slot.  This is the MPC counterpart of
// ap2_jacgen.cpp: what CasADi's SX jacobian + code generation produce for the reference's nlp_jac_g of
// the MPC NLP (pmpc.py:193-217), restricted to one node.
//
// The model constants and u_ref enter as run-time loads (cst[i], ex0); only the tether element count
// is fixed at generation time and written out, so that awempc_create can check it.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../kite3_tables.hpp"
#include "sym.hpp"

namespace {

using awe::Op;
using awe::Sym;
using namespace k3t;

struct RowSink {
    int rows[kRowsPerNode];
    RowSink() { for (int& r : rows) r = -1; }
    void eq_row(int r, const Sym& v) { rows[r] = v.id; }
    void ineq_row(int r, const Sym& v) { rows[K3_N_EQ + r] = v.id; }
};

struct SymIn {
    const Sym* w;
    Sym operator()(int i) const { return w[i]; }
};

struct KindOut {
    std::vector<std::string> body;   // one per direction strip
    awe::EmitStats st;
    std::vector<short> tan_idx;   // [kRowsPerNode][kLanes]
};

// direction strips: the node's tangents split into kStrips contiguous direction ranges of balanced
// tangent counts; a strip is its own function body (STRIP template argument) that recomputes the
// values it needs, so that kStrips wavefronts run one node side by side (strip 0 also stores the row
// values).  AWE_K3_STRIPS overrides the count for experiments.
constexpr int kStripsDefault = 1;

// structural pattern of (row, direction) at a node of `kind` (build_tables' rules)
bool in_pattern(int kind, uint32_t m, int dir) {
    constexpr uint32_t kXdotBits = ((1u << K3_NX) - 1u) << K3_NX;
    if (kind == 0) return (m >> dir) & 1u;
    if (dir < K3_NX) return ((m >> dir) & 1u) || ((m >> (K3_NX + dir)) & 1u);
    if (dir == kDirTf) return (m & kXdotBits) || ((m >> kDirTf) & 1u);
    return (m >> dir) & 1u;
}

KindOut generate(int kind, const std::vector<double>& cst, const Tables& T, int n_strips) {
    awe::Tape tape;
    awe::active_tape() = &tape;
    std::vector<Sym> w(kLanes), cs(cst.size());
    for (int i = 0; i < kLanes; ++i) w[i] = Sym::of(tape.leaf(Op::Input, i));
    for (size_t i = 0; i < cst.size(); ++i) cs[i] = Sym::of(tape.leaf(Op::Cs, (int)i, cst[i]));
    const Sym u_ref = Sym::of(tape.leaf(Op::Extra, 0));
    const int ex_cxx = tape.leaf(Op::Extra, 1), ex_inv_tf = tape.leaf(Op::Extra, 2);
    RowSink sink;
    awe::kite3_node<Sym>(SymIn{w.data()}, w[kDirGamma], u_ref, cs.data(), sink, kind == 0);
    const int n0 = (int)tape.n.size();
    const int one = tape.cnst(1.0);
    auto seed = [&](int i) -> awe::SparseGrad {
        if (kind == 1 && i >= K3_NX && i < 2 * K3_NX) {
            // xdot_s = sum_r C[r][n] X_r / (h t_f): d/d(dir s) = C[n][n] / (h t_f), d/d(dir 11 + s) = 1,
            // d/d t_f = -xdot_s / t_f
            const int s = i - K3_NX;
            const int dtf = tape.mul(tape.neg(w[i].id), ex_inv_tf);
            return {{s, ex_cxx}, {i, one}, {kDirTf, dtf}};
        }
        return {{i, one}};
    };
    std::vector<awe::SparseGrad> G = awe::forward_grads(tape, n0, seed);

    const int nrows = kind == 0 ? kRowsPerNode : K3_N_EQ;
    std::vector<awe::Store> stores;
    const int zero = tape.cnst(0.0);
    for (int r = 0; r < nrows; ++r) {
        const int v = sink.rows[r];
        if (v < 0) { std::fprintf(stderr, "row %d not produced\n", r); std::exit(1); }
        const uint32_t m = r < K3_N_EQ ? T.eq_mask[r] : T.ineq_mask[r - K3_N_EQ];
        stores.push_back({v, 0, r, -1});
        for (auto& e : G[v])
            if (!in_pattern(kind, m, e.first)) {
                std::fprintf(stderr, "kind %d row %d: derivative along direction %d outside the pattern\n", kind, r,
                             e.first);
                std::exit(1);
            }
        for (int dir = 0; dir < kLanes; ++dir) {
            if (!in_pattern(kind, m, dir)) continue;
            int node = zero;
            for (auto& e : G[v]) if (e.first == dir) node = e.second;
            stores.push_back({node, 1, r, dir});
        }
    }
    KindOut ko;
    std::vector<int> per_dir(kLanes, 0), strip_of(kLanes, 0);
    int total = 0;
    for (auto& s : stores) if (s.kind == 1) { per_dir[s.dir]++; total++; }
    for (int dir = 0, acc = 0; dir < kLanes; ++dir) {
        strip_of[dir] = std::min(n_strips - 1, (int)((long long)acc * n_strips / std::max(1, total)));
        acc += per_dir[dir];
    }
    ko.tan_idx.assign(kRowsPerNode * kLanes, -1);
    int slot_base = 0;
    for (int sidx = 0; sidx < n_strips; ++sidx) {
        std::vector<awe::Store> part;
        for (auto& s : stores)
            if ((s.kind != 1 && sidx == 0) || (s.kind == 1 && strip_of[s.dir] == sidx)) part.push_back(s);
        awe::EmitStats st;
        const int before = slot_base;
        ko.body.push_back(part.empty() ? std::string() : awe::emit(tape, part, st, true, 32, false, slot_base));
        slot_base = before + st.n_tan;
        ko.st.ops += st.ops; ko.st.flops += st.flops; ko.st.transcendental += st.transcendental;
        ko.st.loads += st.loads; ko.st.n_tan += st.n_tan; ko.st.n_zero_tan += st.n_zero_tan;
        ko.st.max_live = std::max(ko.st.max_live, st.max_live);
        for (auto& s : part)
            if (s.kind == 1) ko.tan_idx[s.row * kLanes + s.dir] = (short)s.slot;
    }
    awe::active_tape() = nullptr;
    return ko;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: kite3_jacgen <consts file> <output header>\n");
        return 2;
    }
    std::vector<double> cst;
    {
        std::ifstream f(argv[1]);
        double x;
        while (f >> x) cst.push_back(x);
    }
    if ((int)cst.size() != K3_NCONST) {
        std::fprintf(stderr, "expected %d constants, read %zu\n", K3_NCONST, cst.size());
        return 2;
    }
    Tables T;
    std::string err;
    if (build_tables(2, 4, cst.data(), (int)cst.size(), T, err)) {
        std::fprintf(stderr, "tables: %s\n", err.c_str());
        return 1;
    }
    const char* ns = std::getenv("AWE_K3_STRIPS");
    const int n_strips = ns ? std::max(1, std::atoi(ns)) : kStripsDefault;
    KindOut ks = generate(0, cst, T, n_strips), kr = generate(1, cst, T, n_strips);
    auto bodies = [&](const KindOut& k) {
        std::string b;
        for (int s = 0; s < n_strips; ++s)
            b += std::string(s ? "    else " : "    ") + "if constexpr (STRIP == " + std::to_string(s) + ") {\n" +
                 k.body[s] + "    }\n";
        return b;
    };

    std::ostringstream o;
    o << "// GENERATED by awebox_amd/csrc/gen/kite3_jacgen.cpp from kite3_model.hpp -- do not edit.\n"
         "// Straight-line value + sparse forward-mode Jacobian of one tracking-MPC collocation node along\n"
         "// the evaluator's 32 seed directions (see the generator's header comment).\n"
         "#pragma once\n\n#include \"scalar.hpp\"\n\n"
         "#if defined(__HIP_DEVICE_COMPILE__)\n#define AWE_GEN_FENCE() __builtin_amdgcn_sched_barrier(0)\n"
         "#else\n#define AWE_GEN_FENCE() ((void)0)\n#endif\n\nnamespace awe_k3gen {\n\n";
    o << "// integer structure of the model constants the code was generated for (awempc_create checks it)\n";
    o << "constexpr int kNElements = " << (int)cst[K3_C_N_ELEMENTS] << ";\n";
    o << "// direction strips: k3_node_*<TS, STRIP> stores the tangents of strip STRIP (strip 0 also the rows)\n";
    o << "constexpr int kNStrips = " << n_strips << ";\n";
    o << "// tangent slots per node kind (0 shooting, 1 Radau): one per J_g pattern entry of the node's rows\n";
    o << "constexpr int kNTan[2] = {" << ks.st.n_tan << ", " << kr.st.n_tan << "};\n";
    o << "// algorithmic operations per node kind: adds/muls/reciprocals, transcendental calls\n";
    o << "constexpr int kFlops[2] = {" << ks.st.flops << ", " << kr.st.flops << "};\n";
    o << "constexpr int kTranscendental[2] = {" << ks.st.transcendental << ", " << kr.st.transcendental << "};\n";
    o << "// tangent slot of (row, direction), -1 outside the pattern\n";
    o << "constexpr short kTanIdx[2][" << kRowsPerNode << "][" << kLanes << "] = {\n";
    for (const KindOut* k : {&ks, &kr}) {
        o << "  {\n";
        for (int r = 0; r < kRowsPerNode; ++r) {
            o << "    {";
            for (int d = 0; d < kLanes; ++d) o << (d ? "," : "") << k->tan_idx[r * kLanes + d];
            o << "},\n";
        }
        o << "  },\n";
    }
    o << "};\n\n";
    o << "// shooting node: val[0..13] = 12 equalities + 2 path inequalities; ex0 = u_ref\n";
    o << "// in(i): node variable i (31 = phi.gamma); tan[s]: an accessor that sends slot s to its J_g entries\n";
    o << "template <int TS, int STRIP, class In, class Val, class Tan>\nAWE_HD void k3_node_shoot(const In& in, "
         "const double ex0, const double* __restrict__ cst, Val val, Tan tan) {\n";
    o << bodies(ks) << "}\n\n";
    o << "// Radau node: val[0..11] equalities; ex0 = u_ref, ex1 = C[n][n] / (h t_f), ex2 = 1 / t_f\n";
    o << "template <int TS, int STRIP, class In, class Val, class Tan>\nAWE_HD void k3_node_radau(const In& in, "
         "const double ex0, const double ex1, const double ex2, const double* __restrict__ cst, Val val, Tan tan) {\n";
    o << bodies(kr) << "}\n\n}  // namespace awe_k3gen\n";

    std::ofstream out(argv[2]);
    out << o.str();
    std::printf("{\"shooting\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"tangents\": %d, \"zero\": %d, "
                "\"max_live\": %d}, \"radau\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"tangents\": %d, "
                "\"zero\": %d, \"max_live\": %d}}\n",
                ks.st.ops, ks.st.flops, ks.st.transcendental, ks.st.n_tan, ks.st.n_zero_tan, ks.st.max_live, kr.st.ops,
                kr.st.flops, kr.st.transcendental, kr.st.n_tan, kr.st.n_zero_tan, kr.st.max_live);
    return 0;
}
