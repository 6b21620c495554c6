// Build-time generator of the AP2 node-Hessian code (awebox_amd/csrc/ap2_nodehess.gen.hpp).
//
//   ap2_hessgen <consts file> <output header>
//
// The reference's exact-Hessian IPOPT runs CasADi's symbolic Hessian of the Lagrangian, generated
// from the expanded SX graph (opti/preparation.py:366-400, nlp_hess_l).  Here, per node kind, the
// node model (ap2_model.hpp) is traced on the symbolic scalar of gen/sym.hpp and the weighted row
// sum L = sum_r mu_r F_r (mu_r: run-time row weights -- the constraint multipliers, and at a Radau
// node the objective's power and side-slip weights) is differentiated twice by sparse symbolic
// forward mode along the evaluator's seed directions: the first pass gives dL/dp, the second pass
// the derivatives of those tangent expressions, d2L/dp dq.  The seeds are held constant in the
// second pass (their own derivatives -- the t_f curvature of xdot = C X / (h t_f) -- are the
// assembly's B and C terms, as in the hyper-dual kernel), so the output is exactly the
// direction-pair Hessian the hyper-dual colour-pair kernel accumulates (hd[pidx], pair numbering
// of ap2_tables.hpp build_hess_tables), one straight-line function per node kind.
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

// Extra leaves: 0 cxx = C[j][j] / (h t_f); 1 + i: the t_f seed of xdot_i, -xdot_i / t_f; 32 + r: mu_r
constexpr int kExCxx = 0, kExSx = 1, kExMu = 32;

struct KindOut {
    std::string body;
    awe::EmitStats st;
    int n_pairs = 0;
};

KindOut generate(int kind, const std::vector<double>& cst, const awt::Ap2HessTables& H) {
    awe::Tape tape;
    awe::active_tape() = &tape;
    std::vector<Sym> w(AWE_NW + 1), th(AWE_NTHETA0), cs(cst.size());
    for (int i = 0; i <= AWE_NW; ++i) w[i] = Sym::of(tape.leaf(Op::Input, i));
    for (int i = 0; i < AWE_NTHETA0; ++i) th[i] = Sym::of(tape.leaf(Op::Th, i));
    for (size_t i = 0; i < cst.size(); ++i) cs[i] = Sym::of(tape.leaf(Op::Cs, (int)i, cst[i]));
    RowSink sink;
    SymIn in{w.data()};
    awe::ap2_node<Sym>(in, w[awt::kDirGamma], th.data(), cs.data(), sink, kind == 0);
    // the node's weighted row sum
    Sym L(0.0);
    for (int r = 0; r < awt::kHRows; ++r) {
        const bool used = kind == 0 ? r < awt::kRowPower : (r < AWE_N_EQ || r == awt::kRowPower || r == awt::kRowBeta);
        if (!used) continue;
        if (sink.rows[r] < 0) { std::fprintf(stderr, "row %d not produced\n", r); std::exit(1); }
        L = L + Sym::of(tape.leaf(Op::Extra, kExMu + r)) * Sym::of(sink.rows[r]);
    }
    const int one = tape.cnst(1.0);
    const int ex_cxx = tape.leaf(Op::Extra, kExCxx);
    std::vector<int> ex_sx(AWE_NX);
    for (int i = 0; i < AWE_NX; ++i) ex_sx[i] = tape.leaf(Op::Extra, kExSx + i);
    auto seed = [&](int i) -> awe::SparseGrad {
        if (kind == 1 && i >= AWE_NX && i < 2 * AWE_NX) {
            const int s = i - AWE_NX;
            return {{s, ex_cxx}, {i, one}, {awt::kDirTf, ex_sx[s]}};
        }
        return {{i, one}};
    };
    const int n0 = (int)tape.n.size();
    std::vector<awe::SparseGrad> G1 = awe::forward_grads(tape, n0, seed);
    const awe::SparseGrad g1 = G1[L.id];
    const int n1 = (int)tape.n.size();
    std::vector<awe::SparseGrad> G2 = awe::forward_grads(tape, n1, seed);
    std::vector<awe::Store> stores;
    std::vector<int> first_dir;
    KindOut ko;
    for (const auto& pe : g1) {
        const int p = pe.first;
        for (const auto& qe : G2[pe.second]) {
            const int q = qe.first;
            if (q < p) continue;
            const int pidx = H.ht.pidx[kind][p][q];
            if (pidx < 0) {
                std::fprintf(stderr, "kind %d: pair (%d, %d) outside the Hessian pattern\n", kind, p, q);
                std::exit(1);
            }
            awe::Store s{qe.second, 3, pidx, -1};   // obv[row] = ... : hd[pidx]
            stores.push_back(s);
            first_dir.push_back(p);
            ko.n_pairs++;
        }
    }
    // direction strips: the pairs grouped by their first direction into n_strips balanced groups,
    // each emitted as its own scope that recomputes the values it needs (opaque leaf copies)
    const char* ns = std::getenv("AWE_HESS_STRIPS");
    const int n_strips = ns ? std::atoi(ns) : 1;
    std::vector<int> per_dir(awt::kDirs, 0);
    for (int p : first_dir) per_dir[p]++;
    std::vector<int> strip_of(awt::kDirs, 0);
    {
        int acc = 0;
        for (int d = 0; d < awt::kDirs; ++d) {
            strip_of[d] = std::min(n_strips - 1, (int)((long long)acc * n_strips / std::max(1, ko.n_pairs)));
            acc += per_dir[d];
        }
    }
    for (int sidx = 0; sidx < n_strips; ++sidx) {
        std::vector<awe::Store> part;
        for (size_t i = 0; i < stores.size(); ++i)
            if (strip_of[first_dir[i]] == sidx) part.push_back(stores[i]);
        if (part.empty()) continue;
        awe::EmitStats st;
        std::string body = awe::emit(tape, part, st, true, 32, sidx > 0, 0);
        ko.body += "    {   // strip " + std::to_string(sidx) + "\n" + body + "    }\n";
        ko.st.ops += st.ops; ko.st.flops += st.flops; ko.st.transcendental += st.transcendental;
        ko.st.max_live = std::max(ko.st.max_live, st.max_live);
        std::fprintf(stderr, "kind %d strip %d: %zu pairs, %d ops, max_live %d\n", kind, sidx, part.size(), st.ops, st.max_live);
    }
    awe::active_tape() = nullptr;
    return ko;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: ap2_hessgen <consts file> <output header>\n");
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
    awt::Ap2HessTables H;
    if (awt::build_hess_tables(T, H, err) != AWE_OK) {
        std::fprintf(stderr, "hessian tables: %s\n", err.c_str());
        return 1;
    }
    KindOut ks = generate(0, cst, H), kr = generate(1, cst, H);
    std::printf("{\"shooting\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"pairs\": %d, \"max_live\": %d}, "
                "\"radau\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"pairs\": %d, \"max_live\": %d}}\n",
                ks.st.ops, ks.st.flops, ks.st.transcendental, ks.n_pairs, ks.st.max_live, kr.st.ops, kr.st.flops,
                kr.st.transcendental, kr.n_pairs, kr.st.max_live);
    std::ofstream out(argv[2]);
    out << "// shooting\n" << ks.body << "\n// radau\n" << kr.body;
    return 0;
}
