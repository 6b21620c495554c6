// Build-time generator of the AP2 node-Hessian code (awebox_amd/csrc/ap2_nodehess.gen.hpp).
//
//   ap2_hessgen <consts file> <output header>
//
// The reference's exact-Hessian IPOPT evaluates CasADi's symbolic Hessian of the Lagrangian,
// generated from the expanded SX graph (opti/preparation.py:366-400, nlp_hess_l; exact Hessian is
// IPOPT's default, opts/default.py:323).  Here, per node kind, the node model (ap2_model.hpp) is
// traced on the symbolic scalar of gen/sym.hpp and the node Lagrangian
//     L = sum_r mu_r F_r  (+ at a Radau node: cb beta^2 + cpp p, the objective's side-slip and
//                            power terms, objective.py:279-298,390-421)
// is differentiated twice.  First order by a symbolic reverse (adjoint) sweep over the tape: one
// adjoint per tape node, so dL/dp costs a small multiple of the value work and no tangent vector
// per intermediate exists.  Second order by sparse symbolic forward mode over the adjoint tape
// along the evaluator's seed directions (forward-over-reverse), so only the pairs (p, q) of the
// node's second-order pattern are formed.  The seeds are held constant in the second pass (their
// own derivatives -- the t_f curvature of xdot = C X / (h t_f) -- enter the assembly as the B and C
// terms, as in the hyper-dual kernel), so the output is the direction-pair Hessian hd[pidx] (pair
// numbering of ap2_tables.hpp build_hess_tables) plus, at a Radau node, G[i] = dL/d xdot_i (the
// first-order part the B and C terms need).
//
// AWE_HESS_MODE=fof selects forward-over-forward instead (the earlier experiment, kept for the
// live-set comparison printed on stdout).
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

// Extra leaves: 0 cxx = C[j][j] / (h t_f); 1 + i: the t_f seed of xdot_i, -xdot_i / t_f;
// 24 cb = sigma c_beta w_j / norm_beta, 25 cpp = sigma (-c_P) w_j / N (the power cost without its
// (1 - psi) factor, which is traced: psi is node input AWE_NW + 1, direction kDirPsi); 32 + r: mu_r
constexpr int kExCxx = 0, kExSx = 1, kExCb = 24, kExCpp = 25, kExMu = 32;

struct KindOut {
    std::string body;
    awe::EmitStats st;
    int n_pairs = 0;
    std::vector<int> hd_row;     // pair index -> output row (-1: no model curvature)
    int n_hd = 0;
};

// symbolic reverse sweep: adjoints of every node in the cone of `out` (dL/dv for L = out)
std::vector<int> adjoints(awe::Tape& t, int out) {
    const int n0 = out + 1;
    std::vector<char> cone(n0, 0);
    cone[out] = 1;
    for (int v = out; v >= 0; --v) {
        if (!cone[v]) continue;
        if (t.n[v].a >= 0) cone[t.n[v].a] = 1;
        if (t.n[v].b >= 0) cone[t.n[v].b] = 1;
    }
    const int zero = t.cnst(0.0);
    std::vector<int> adj(n0, zero);
    adj[out] = t.cnst(1.0);
    auto acc = [&](int o, int term) { adj[o] = t.add(adj[o], term); };
    for (int v = out; v >= 0; --v) {
        if (!cone[v] || t.is_c(adj[v], 0.0)) continue;
        const awe::SNode s = t.n[v];
        const int av = adj[v];
        t.group = v;   // emitted with the value it differentiates (scheduling hint only)
        switch (s.op) {
            case Op::Add: acc(s.a, av); acc(s.b, av); break;
            case Op::Sub: acc(s.a, av); acc(s.b, t.neg(av)); break;
            case Op::Mul:
                if (s.a == s.b) { acc(s.a, t.mul(t.mul(t.cnst(2.0), s.a), av)); break; }
                acc(s.a, t.mul(av, s.b));
                acc(s.b, t.mul(s.a, av));
                break;
            case Op::Neg: acc(s.a, t.neg(av)); break;
            case Op::Rcp: acc(s.a, t.neg(t.mul(av, t.mul(v, v)))); break;
            case Op::Sqrt: acc(s.a, t.mul(av, t.mul(t.cnst(0.5), t.rcp(v)))); break;
            case Op::Exp: acc(s.a, t.mul(av, v)); break;
            case Op::Log: acc(s.a, t.mul(av, t.rcp(s.a))); break;
            case Op::Sin: acc(s.a, t.mul(av, t.un(Op::Cos, s.a))); break;
            case Op::Cos: acc(s.a, t.neg(t.mul(av, t.un(Op::Sin, s.a)))); break;
            default: break;
        }
    }
    t.group = -1;
    return adj;
}

KindOut generate(int kind, const std::vector<double>& cst, const awt::Ap2HessTables& H, bool fof,
                 std::vector<int>& g_dirs) {
    awe::Tape tape;
    tape.extra_call = true;
    awe::active_tape() = &tape;
    std::vector<Sym> w(AWE_NW + 1), th(AWE_NTHETA0), cs(cst.size());
    for (int i = 0; i <= AWE_NW; ++i) w[i] = Sym::of(tape.leaf(Op::Input, i));
    for (int i = 0; i < AWE_NTHETA0; ++i) th[i] = Sym::of(tape.leaf(Op::Th, i));
    for (size_t i = 0; i < cst.size(); ++i) cs[i] = Sym::of(tape.leaf(Op::Cs, (int)i, cst[i]));
    const int psi = tape.leaf(Op::Input, AWE_NW + 1);     // phi.psi (Radau node objective)
    RowSink sink;
    SymIn in{w.data()};
    awe::ap2_node<Sym>(in, w[awt::kDirGamma], th.data(), cs.data(), sink, kind == 0);
    // the node's Lagrangian
    Sym L(0.0);
    for (int r = 0; r < (kind == 0 ? awt::kRowPower : AWE_N_EQ); ++r) {
        if (sink.rows[r] < 0) { std::fprintf(stderr, "row %d not produced\n", r); std::exit(1); }
        L = L + Sym::of(tape.leaf(Op::Extra, kExMu + r)) * Sym::of(sink.rows[r]);
    }
    if (kind == 1) {
        const Sym bt = Sym::of(sink.rows[awt::kRowBeta]), pw = Sym::of(sink.rows[awt::kRowPower]);
        const Sym cb = Sym::of(tape.leaf(Op::Extra, kExCb)), cpp = Sym::of(tape.leaf(Op::Extra, kExCpp));
        L = L + cb * (bt * bt) + cpp * ((1.0 - Sym::of(psi)) * pw);
    }
    const int one = tape.cnst(1.0);
    const int ex_cxx = tape.leaf(Op::Extra, kExCxx);
    std::vector<int> ex_sx(AWE_NX);
    for (int i = 0; i < AWE_NX; ++i) ex_sx[i] = tape.leaf(Op::Extra, kExSx + i);
    auto seed = [&](int i) -> awe::SparseGrad {
        if (i == AWE_NW + 1) return {{awt::kDirPsi, one}};
        if (kind == 1 && i >= AWE_NX && i < 2 * AWE_NX) {
            const int s = i - AWE_NX;
            return {{s, ex_cxx}, {i, one}, {awt::kDirTf, ex_sx[s]}};
        }
        return {{i, one}};
    };
    // first order: g1[p] = dL / d(direction p)
    awe::SparseGrad g1;
    if (fof) {
        const int n0 = (int)tape.n.size();
        std::vector<awe::SparseGrad> G1 = awe::forward_grads(tape, n0, seed);
        g1 = G1[L.id];
    } else {
        std::vector<int> adj = adjoints(tape, L.id);
        std::vector<int> per_dir(awt::kDirs, -1);
        for (int v = 0; v <= L.id && v < (int)adj.size(); ++v) {
            if (tape.n[v].op != Op::Input || tape.is_c(adj[v], 0.0)) continue;
            for (auto& e : seed(tape.n[v].idx)) {
                const int term = tape.mul(e.second, adj[v]);
                per_dir[e.first] = per_dir[e.first] < 0 ? term : tape.add(per_dir[e.first], term);
            }
        }
        for (int p = 0; p < awt::kDirs; ++p)
            if (per_dir[p] >= 0 && !tape.is_c(per_dir[p], 0.0)) g1.emplace_back(p, per_dir[p]);
    }
    const int n1 = (int)tape.n.size();
    // second order in strips of forward directions q (each strip its own scope, which recomputes the
    // values and adjoints it needs): AWE_HESS_STRIPS, default 1
    const char* ns = std::getenv("AWE_HESS_STRIPS");
    const int n_strips = ns ? std::max(1, std::atoi(ns)) : 1;
    std::vector<awe::SparseGrad> G2 = awe::forward_grads(tape, n1, seed);
    std::vector<std::vector<awe::Store>> part(n_strips);
    std::vector<int> per_q(awt::kDirs, 0);
    KindOut ko;
    for (const auto& pe : g1)
        for (const auto& qe : G2[pe.second])
            if (qe.first >= pe.first) { per_q[qe.first]++; ko.n_pairs++; }
    std::vector<int> strip_of(awt::kDirs, 0);
    {
        int acc = 0;
        for (int q = 0; q < awt::kDirs; ++q) {
            strip_of[q] = std::min(n_strips - 1, (int)((long long)acc * n_strips / std::max(1, ko.n_pairs)));
            acc += per_q[q];
        }
    }
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
            part[strip_of[q]].push_back(awe::Store{qe.second, 3, pidx, -1});   // obv[pidx] = hd of the pair
        }
    }
    // compact output rows: obv[row] for the pairs the node model has curvature in, in pair order (the
    // objective-only pairs of the pattern have no row: the assembly kernel adds them analytically)
    {
        std::vector<int> row_of(H.ht.npairs[kind], -1);
        for (auto& pv : part)
            for (auto& st : pv) row_of[st.row] = 0;
        int nrow = 0;
        for (int i = 0; i < H.ht.npairs[kind]; ++i)
            if (row_of[i] == 0) row_of[i] = nrow++;
        for (auto& pv : part)
            for (auto& st : pv) st.row = row_of[st.row];
        ko.hd_row = row_of;
        ko.n_hd = nrow;
    }
    // Radau node: G[i] = dL / d xdot_i (direction AWE_NX + i), stored as dbp[i], in the first strip
    if (kind == 1) {
        for (const auto& pe : g1)
            if (pe.first >= AWE_NX && pe.first < 2 * AWE_NX) {
                part[0].push_back(awe::Store{pe.second, 2, -1, pe.first - AWE_NX});
                g_dirs.push_back(pe.first - AWE_NX);
            }
    }
    for (int sidx = 0; sidx < n_strips; ++sidx) {
        if (part[sidx].empty()) continue;
        awe::EmitStats st;
        std::string body = awe::emit(tape, part[sidx], st, true, 32, sidx > 0, 0);
        ko.body += "    {   // strip " + std::to_string(sidx) + "\n" + body + "    }\n";
        ko.st.ops += st.ops; ko.st.flops += st.flops; ko.st.transcendental += st.transcendental;
        ko.st.max_live = std::max(ko.st.max_live, st.max_live);
        if (n_strips > 1)
            std::fprintf(stderr, "kind %d strip %d: %zu stores, %d ops, max_live %d\n", kind, sidx, part[sidx].size(),
                         st.ops, st.max_live);
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
    const char* mode = std::getenv("AWE_HESS_MODE");
    const bool fof = mode && std::strcmp(mode, "fof") == 0;
    std::vector<int> gd0, gd1;
    KindOut ks = generate(0, cst, H, fof, gd0), kr = generate(1, cst, H, fof, gd1);
    std::printf("{\"mode\": \"%s\", \"shooting\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"pairs\": %d, \"max_live\": %d}, "
                "\"radau\": {\"ops\": %d, \"flops\": %d, \"transcendental\": %d, \"pairs\": %d, \"max_live\": %d, \"g\": %zu}}\n",
                fof ? "fof" : "for", ks.st.ops, ks.st.flops, ks.st.transcendental, ks.n_pairs, ks.st.max_live,
                kr.st.ops, kr.st.flops, kr.st.transcendental, kr.n_pairs, kr.st.max_live, gd1.size());
    if ((int)gd1.size() != AWE_NX) {
        std::fprintf(stderr, "expected a gradient entry for every xdot direction, got %zu\n", gd1.size());
        return 1;
    }
    std::ostringstream o;
    o << "// GENERATED by awebox_amd/csrc/gen/ap2_hessgen.cpp from ap2_model.hpp -- do not edit.\n"
         "// Straight-line direction-pair Hessian of one AP2 collocation node's Lagrangian (forward-over-\n"
         "// reverse; see the generator's header comment).\n"
         "#pragma once\n\n#include \"scalar.hpp\"\n\n"
         "#ifndef AWE_GEN_FENCE\n#if defined(__HIP_DEVICE_COMPILE__)\n#define AWE_GEN_FENCE() __builtin_amdgcn_sched_barrier(0)\n"
         "#else\n#define AWE_GEN_FENCE() ((void)0)\n#endif\n#endif\n"
         "#ifndef AWE_GEN_OPAQUE\n#if defined(__HIP_DEVICE_COMPILE__)\n"
         "__device__ __forceinline__ double awe_hgen_opaque(double x) { asm volatile(\"\" : \"+v\"(x)); return x; }\n"
         "#define AWE_GEN_OPAQUE(x) awe_hgen_opaque(x)\n#else\n#define AWE_GEN_OPAQUE(x) (x)\n#endif\n#endif\n\n"
         "namespace awe_hgen {\n\n";
    o << "// integer structure of the model constants the code was generated for (awe_create checks it)\n";
    o << "constexpr int kNElements = " << (int)cst[AWE_C_N_ELEMENTS] << ";\n";
    o << "constexpr int kSdLen[54] = {";
    for (int i = 0; i < 54; ++i) o << (i ? ", " : "") << (int)cst[AWE_C_SD_LEN + i];
    o << "};\n";
    o << "// direction pairs per node kind (0 shooting, 1 Radau): pair i is (kPairP, kPairQ), the numbering of\n"
         "// ap2_tables.hpp build_hess_tables for these constants\n";
    o << "constexpr int kNPairs[2] = {" << H.ht.npairs[0] << ", " << H.ht.npairs[1] << "};\n";
    int maxp = std::max(H.ht.npairs[0], H.ht.npairs[1]);
    for (const char* nm : {"kPairP", "kPairQ"}) {
        o << "constexpr short " << nm << "[2][" << maxp << "] = {";
        for (int kind = 0; kind < 2; ++kind) {
            o << (kind ? ", {" : "{");
            std::vector<short> v(maxp, -1);
            for (int p = 0; p < awt::kDirs; ++p)
                for (int q = p; q < awt::kDirs; ++q) {
                    const int i = H.ht.pidx[kind][p][q];
                    if (i >= 0) v[i] = (short)(nm[5] == 'P' ? p : q);
                }
            for (int i = 0; i < maxp; ++i) o << (i ? "," : "") << v[i];
            o << "}";
        }
        o << "};\n";
    }
    o << "// output rows: obv[kHdRow[kind][pidx]] holds pair pidx (-1: the node model has no curvature there)\n";
    o << "constexpr int kNHd[2] = {" << ks.n_hd << ", " << kr.n_hd << "};\n";
    o << "constexpr short kHdRow[2][" << maxp << "] = {";
    for (int kind = 0; kind < 2; ++kind) {
        const KindOut& k = kind ? kr : ks;
        o << (kind ? ", {" : "{");
        for (int i = 0; i < maxp; ++i) o << (i ? "," : "") << (i < (int)k.hd_row.size() ? k.hd_row[i] : -1);
        o << "}";
    }
    o << "};\n";
    o << "// algorithmic operations per node kind: adds/muls/reciprocals, transcendental calls\n";
    o << "constexpr int kFlops[2] = {" << ks.st.flops << ", " << kr.st.flops << "};\n";
    o << "constexpr int kTranscendental[2] = {" << ks.st.transcendental << ", " << kr.st.transcendental << "};\n";
    // theta0 entries the code reads (either kind): the kernels stage only these
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
    o << "};\n\n";
    o << "// in(i): node input i (0..58 the node variables, 59 phi.gamma, 60 phi.psi); th[i]: theta0;\n"
         "// ex(i): 0 C[j][j] / (h t_f), 1 + i -xdot_i / t_f, 24 sigma c_beta w_j / norm_beta,\n"
         "// 25 sigma (-c_P) w_j / N, 32 + r the multiplier of node row r; obv[kHdRow[kind][pidx]] = d2L / dp dq\n";
    o << "template <class In, class Th, class Ex, class Out>\nAWE_HD void ap2_hess_shoot(const In& in, Th th, "
         "const double* __restrict__ cst, const Ex& ex, Out obv) {\n";
    o << ks.body << "}\n\n";
    o << "// Radau node: also dbp[i] = dL / d xdot_i\n";
    o << "template <class In, class Th, class Ex, class Out, class Gout>\nAWE_HD void ap2_hess_radau(const In& in, Th th, "
         "const double* __restrict__ cst, const Ex& ex, Out obv, Gout dbp) {\n";
    o << kr.body << "}\n\n}  // namespace awe_hgen\n";
    std::ofstream out(argv[2]);
    out << o.str();
    return 0;
}
