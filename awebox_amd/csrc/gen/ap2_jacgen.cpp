// Build-time generator of the AP2 node-Jacobian code (awebox_amd/csrc/ap2_nodejac.gen.hpp).
//
//   ap2_jacgen <consts file> <output header>
//
// Traces ap2_node (ap2_model.hpp) on the symbolic scalar of gen/sym.hpp for the two node kinds
// of the collocation scheme (shooting node: 24 model equalities + 9 path inequalities; Radau
// node: 24 equalities + the power integrand and side slip the objective needs), differentiates
// the tape along the kernel's 61 seed directions (ap2_tables.hpp: at a Radau node direction i
// seeds x_i and xdot_i = C[j][j] / (h t_f), direction 23 + i seeds xdot_i, direction 58 carries
// d/d t_f through every xdot_i = -xdot_i / t_f), and writes one straight-line function per kind
// that stores the node's row values and every structurally non-zero directional derivative of
// the first-order pattern (ColorTabs::dmask), plus the table that maps (row, direction) to the
// tangent-buffer slot.  This is what CasADi's SX jacobian + code generation produce for the
// reference's nlp_jac_g (preparation.py:366-400), restricted to one node.
//
// The model constants enter as run-time loads (cst[i]); only the integer structure read from
// them (tether elements, stability-derivative table lengths) is fixed at generation time and
// written out, so that awe_create can check it.
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../ap2_tables.hpp"
#include "sym.hpp"

namespace {

using awe::Op;
using awe::Sym;

struct RowSink {
    int rows[awt::kRowBeta + 1];
    RowSink() { for (int& r : rows) r = -1; }
    void eq_row(int r, const Sym& v) { rows[r] = v.id; }
    void ineq_row(int r, const Sym& v) { rows[AWE_N_EQ + r] = v.id; }
    void power(const Sym& v) { rows[awt::kRowPower] = v.id; }
    void beta(const Sym& v) { rows[awt::kRowBeta] = v.id; }
};

struct SymIn {
    const Sym* w;
    Sym operator()(int i) const { return w[i]; }
};

struct KindOut {
    std::string body;
    awe::EmitStats st;
    std::vector<short> tan_idx;   // [35][64]
    int n_tan = 0;
};

std::vector<int> ko_dbp_dirs;   // directions of the Radau node's dbp entries, in order

KindOut generate(int kind, const std::vector<double>& cst, const awt::ColorTabs& ct, int n_strips) {
    awe::Tape tape;
    awe::active_tape() = &tape;
    std::vector<Sym> w(AWE_NW + 1), th(AWE_NTHETA0), cs(cst.size());
    for (int i = 0; i <= AWE_NW; ++i) w[i] = Sym::of(tape.leaf(Op::Input, i));
    for (int i = 0; i < AWE_NTHETA0; ++i) th[i] = Sym::of(tape.leaf(Op::Th, i));
    for (size_t i = 0; i < cst.size(); ++i) cs[i] = Sym::of(tape.leaf(Op::Cs, (int)i, cst[i]));
    const int ex_cxx = tape.leaf(Op::Extra, 0), ex_inv_tf = tape.leaf(Op::Extra, 1);
    RowSink sink;
    SymIn in{w.data()};
    awe::ap2_node<Sym>(in, w[awt::kDirGamma], th.data(), cs.data(), sink, kind == 0);
    // Radau node: the objective terms in the side slip and the power integrand (objective.py:390-421,
    // the (1 - psi) power cost), cb beta^2 + cpp p with cb = c_beta w_j / norm_beta (ex2) and
    // cpp = (1 - psi)(-c_P) w_j / N (ex3); its directional derivatives go to dbp[dir]
    int objbp = -1;
    if (kind == 1) {
        const Sym cb = Sym::of(tape.leaf(Op::Extra, 2)), cpp = Sym::of(tape.leaf(Op::Extra, 3));
        const Sym bt = Sym::of(sink.rows[awt::kRowBeta]), pw = Sym::of(sink.rows[awt::kRowPower]);
        objbp = (cb * (bt * bt) + cpp * pw).id;
    }
    const int n0 = (int)tape.n.size();

    const int one = tape.cnst(1.0);
    auto seed = [&](int i) -> awe::SparseGrad {
        if (kind == 1 && i >= AWE_NX && i < 2 * AWE_NX) {
            const int s = i - AWE_NX;
            // xdot_s = sum_r C[r][j] X_r / (h t_f): d/d(dir s) = C[j][j] / (h t_f), d/d(dir 23 + s) = 1,
            // d/d t_f = -xdot_s / t_f
            const int dtf = tape.mul(tape.neg(w[i].id), ex_inv_tf);
            return {{s, ex_cxx}, {i, one}, {awt::kDirTf, dtf}};
        }
        return {{i, one}};
    };
    std::vector<awe::SparseGrad> G = awe::forward_grads(tape, n0, seed);

    std::vector<int> rows;
    if (kind == 0) {
        for (int r = 0; r < awt::kRowPower; ++r) rows.push_back(r);
    } else {
        for (int r = 0; r < AWE_N_EQ; ++r) rows.push_back(r);
    }
    std::vector<awe::Store> stores;
    const int zero = tape.cnst(0.0);
    for (int r : rows) {
        const int v = sink.rows[r];
        if (v < 0) { std::fprintf(stderr, "row %d not produced\n", r); std::exit(1); }
        stores.push_back({v, 0, r, -1});
        const awe::SparseGrad& g = G[v];
        for (auto& e : g)
            if (!((ct.dmask[kind][e.first] >> r) & 1ull)) {
                std::fprintf(stderr, "kind %d row %d: derivative along direction %d outside the pattern\n", kind, r,
                             e.first);
                std::exit(1);
            }
        for (int dir = 0; dir < awt::kDirs; ++dir) {
            if (!((ct.dmask[kind][dir] >> r) & 1ull)) continue;
            int node = zero;
            for (auto& e : g) if (e.first == dir) node = e.second;
            stores.push_back({node, 1, r, dir});
        }
    }
    if (kind == 1) {   // objective: beta and power values (obv) and the tangents of cb beta^2 + cpp p (dbp)
        stores.push_back({sink.rows[awt::kRowBeta], 3, 0, -1});
        stores.push_back({sink.rows[awt::kRowPower], 3, 1, -1});
        // compact: dbp[i] is the derivative along direction kDbpDir[i]
        for (auto& e : G[objbp]) {
            if (e.first > awt::kDirGamma) continue;
            stores.push_back({e.second, 2, -1, (int)ko_dbp_dirs.size()});
            ko_dbp_dirs.push_back(e.first);
        }
    }
    KindOut ko;
    // a scheduling fence every kFenceEvery statements keeps the compiler's machine scheduler near
    // the pressure-scheduled order (without fences it hoists and interleaves until the register
    // allocator spills to scratch: 392 -> 127 scratch reloads in the instance-minor node kernel)
    constexpr int kFenceEvery = 32;
    const int fence = kFenceEvery;
    // direction strips: contiguous direction ranges with balanced tangent counts; strip 0 also
    // stores the row values.  Each strip is its own scope and recomputes the values it needs.
    std::vector<int> per_dir(awt::kDirs, 0);
    for (auto& s : stores) if (s.kind == 1) per_dir[s.dir]++;
    int total = 0;
    for (int c : per_dir) total += c;
    std::vector<int> strip_of(awt::kDirs, 0);
    {
        int acc = 0;
        for (int dir = 0; dir < awt::kDirs; ++dir) {
            strip_of[dir] = std::min(n_strips - 1, (int)((long long)acc * n_strips / std::max(1, total)));
            acc += per_dir[dir];
        }
    }
    ko.tan_idx.assign(35 * 64, -1);
    int slot_base = 0;
    for (int sidx = 0; sidx < n_strips; ++sidx) {
        std::vector<awe::Store> part;
        for (auto& s : stores)
            if ((s.kind != 1 && sidx == 0) || (s.kind == 1 && strip_of[s.dir] == sidx)) part.push_back(s);
        if (part.empty()) continue;
        awe::EmitStats st;
        const int before = slot_base;
        std::string body = awe::emit(tape, part, st, true, fence, sidx > 0, slot_base);
        slot_base = before + st.n_tan;
        ko.body += "    {   // strip " + std::to_string(sidx) + "\n" + body + "    }\n";
        ko.st.ops += st.ops; ko.st.flops += st.flops; ko.st.transcendental += st.transcendental;
        ko.st.loads += st.loads; ko.st.n_tan += st.n_tan; ko.st.n_zero_tan += st.n_zero_tan;
        ko.st.max_live = std::max(ko.st.max_live, st.max_live);
        for (auto& s : part)
            if (s.kind == 1) ko.tan_idx[s.row * 64 + s.dir] = (short)s.slot;
    }
    ko.n_tan = ko.st.n_tan;
    awe::active_tape() = nullptr;
    return ko;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: ap2_jacgen <consts file> <output header>\n");
        return 2;
    }
    std::vector<double> cst;
    {
        std::ifstream f(argv[1]);
        double x;
        while (f >> x) cst.push_back(x);
    }
    if ((int)cst.size() != AWE_NCONST) {
        std::fprintf(stderr, "expected %d constants, read %zu\n", AWE_NCONST, cst.size());
        return 2;
    }
    awt::Ap2Tables T;
    std::string err;
    if (awt::build_ap2_tables(2, 4, cst.data(), (int)cst.size(), T, err) != AWE_OK) {
        std::fprintf(stderr, "tables: %s\n", err.c_str());
        return 1;
    }
    const char* ns = std::getenv("AWE_GEN_STRIPS");
    const int n_strips = ns ? std::atoi(ns) : 1;
    KindOut ks = generate(0, cst, T.ct, n_strips), kr = generate(1, cst, T.ct, n_strips);

    std::ostringstream o;
    o << "// GENERATED by awebox_amd/csrc/gen/ap2_jacgen.cpp from ap2_model.hpp -- do not edit.\n"
         "// Straight-line value + sparse forward-mode Jacobian of one AP2 collocation node along the\n"
         "// evaluator's seed directions (see the generator's header comment).\n"
         "#pragma once\n\n#include \"scalar.hpp\"\n\n"
         "// scheduling fence: keeps the register allocator to the emitted (pressure-scheduled) order\n"
         "#if defined(__HIP_DEVICE_COMPILE__)\n#define AWE_GEN_FENCE() __builtin_amdgcn_sched_barrier(0)\n"
         "#else\n#define AWE_GEN_FENCE() ((void)0)\n#endif\n"
         "// opaque copy: a strip's values cannot be merged with another strip's (recomputed, not kept)\n"
         "#if defined(__HIP_DEVICE_COMPILE__)\n"
         "__device__ __forceinline__ double awe_gen_opaque(double x) { asm volatile(\"\" : \"+v\"(x)); return x; }\n"
         "#define AWE_GEN_OPAQUE(x) awe_gen_opaque(x)\n"
         "__device__ __forceinline__ double awe_gen_keep(double x) { asm(\"\" : \"+v\"(x)); return x; }\n"
         "#define AWE_GEN_KEEP(x) awe_gen_keep(x)\n"
         "#else\n#define AWE_GEN_OPAQUE(x) (x)\n#define AWE_GEN_KEEP(x) (x)\n#endif\n\nnamespace awe_gen {\n\n";
    o << "// integer structure of the model constants the code was generated for (awe_create checks it)\n";
    o << "constexpr int kNElements = " << (int)cst[AWE_C_N_ELEMENTS] << ";\n";
    o << "constexpr int kSdLen[54] = {";
    for (int i = 0; i < 54; ++i) o << (i ? ", " : "") << (int)cst[AWE_C_SD_LEN + i];
    o << "};\n";
    o << "// tangent-buffer entries per node kind (0 shooting, 1 Radau)\n";
    o << "constexpr int kNTan[2] = {" << ks.n_tan << ", " << kr.n_tan << "};\n";
    o << "// algorithmic operations per node kind: adds/muls/reciprocals, transcendental calls\n";
    o << "constexpr int kFlops[2] = {" << ks.st.flops << ", " << kr.st.flops << "};\n";
    o << "constexpr int kTranscendental[2] = {" << ks.st.transcendental << ", " << kr.st.transcendental << "};\n";
    o << "// dbp[i] of the Radau node is the derivative along seed direction kDbpDir[i]\n";
    o << "constexpr int kNDbp = " << ko_dbp_dirs.size() << ";\n";
    o << "constexpr int kDbpDir[" << std::max<size_t>(1, ko_dbp_dirs.size()) << "] = {";
    for (size_t i = 0; i < ko_dbp_dirs.size(); ++i) o << (i ? ", " : "") << ko_dbp_dirs[i];
    o << "};\n";
    // theta0 entries the node code reads (either kind): the instance-minor kernel stages only these
    std::vector<int> th_row(AWE_NTHETA0, -1);
    int n_th = 0;
    for (const std::string* b : {&ks.body, &kr.body})
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
    o << "// tangent-buffer slot of (row, direction), -1 where the pattern has no entry\n";
    o << "constexpr short kTanIdx[2][35][64] = {\n";
    for (const KindOut* k : {&ks, &kr}) {
        o << "  {\n";
        for (int r = 0; r < 35; ++r) {
            o << "    {";
            for (int d = 0; d < 64; ++d) o << (d ? "," : "") << k->tan_idx[r * 64 + d];
            o << "},\n";
        }
        o << "  },\n";
    }
    o << "};\n\n";
    o << "// shooting node: val[0..32] = 24 equalities + 9 path inequalities, tan[kNTan[0]]\n";
    o << "// tangent s of the node is stored at tan[s * TS] (TS = 64: lane-interleaved, one wavefront's nodes\n";
    o << "// side by side, so that a store instruction writes 64 consecutive doubles)\n";
    o << "// th, val, tan: pointers, or accessor objects with operator[] (the instance-minor kernel reads\n"
         "// th[i] at THT[i * ld + b] and sends tan[s] to the J_g entries of slot s)\n";
    o << "template <int TS, class In, class Th, class Val, class Tan>\nAWE_HD void ap2_node_shoot(const In& in, Th th, "
         "const double* __restrict__ cst, Val val, Tan tan) {\n";
    o << ks.body << "}\n\n";
    o << "// Radau node: val[0..23] equalities, tan[kNTan[1]]; obv[0] side slip, obv[1] power integrand;\n";
    o << "// dbp[i] = directional derivative of ex2 beta^2 + ex3 power along seed direction kDbpDir[i];\n";
    o << "// ex0 = C[j][j] / (h t_f), ex1 = 1 / t_f\n";
    o << "template <int TS, class In, class Th, class Val, class Tan, class Dbp, class Obv>\n"
         "AWE_HD void ap2_node_radau(const In& in, const double ex0, const double ex1, "
         "const double ex2, const double ex3, Th th, const double* __restrict__ cst, "
         "Val val, Tan tan, Dbp dbp, Obv obv) {\n";
    o << kr.body << "}\n\n}  // namespace awe_gen\n";

    std::ofstream out(argv[2]);
    out << o.str();
    std::printf("{\"shooting\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"tangents\": %d, \"zero\": %d, \"max_live\": %d}, "
                "\"radau\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"tangents\": %d, \"zero\": %d, \"max_live\": %d}}\n",
                ks.st.ops, ks.st.flops, ks.st.transcendental, ks.n_tan, ks.st.n_zero_tan, ks.st.max_live, kr.st.ops, kr.st.flops,
                kr.st.transcendental, kr.n_tan, kr.st.n_zero_tan, kr.st.max_live);
    return 0;
}
