// Host check of the generated node-Hessian code (ap2_nodehess.gen.hpp) against the templated
// model in hyper-dual arithmetic: for every direction pair (p, q) of the node's pattern one
// evaluation with e1 seeded along p and e2 along q (the seeding of awegpu.hip's LaneHIn, seeds held
// constant), of the node Lagrangian L = sum_r mu_r F_r (+ cb beta^2 + cpp (1 - psi) p at a Radau
// node); and dL / d xdot_i from the same evaluation's first-order part.
//
//   check_ap2_hess <consts> <theta0> <node values (59 + gamma + psi)> <cxx> <inv_tf> <sigma-free cb> <cpp>
//
// Prints one JSON line: the largest relative differences per node kind.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#include "../ap2_model.hpp"
#include "../ap2_nodehess.gen.hpp"
#include "../ap2_tables.hpp"

namespace {

std::vector<double> read(const char* path) {
    std::vector<double> v;
    std::ifstream f(path);
    double x;
    while (f >> x) v.push_back(x);
    return v;
}

struct PlainIn {
    const double* w;
    double operator()(int i) const { return w[i]; }
};

struct Ex {
    const double* w;
    double cxx, inv_tf, cb, cpp;
    const double* mu;
    double operator()(int i) const {
        if (i == 0) return cxx;
        if (i >= 1 && i <= AWE_NX) return -w[AWE_NX + i - 1] * inv_tf;
        if (i == 24) return cb;
        if (i == 25) return cpp;
        return mu[i - 32];
    }
};

// seed coefficient of node input i along direction dir
double seed(int kind, int i, int dir, const double* w, double cxx, double inv_tf) {
    double t = (i == dir) ? 1.0 : 0.0;
    if (kind == 1 && i >= AWE_NX && i < 2 * AWE_NX) {
        const int s = i - AWE_NX;
        if (dir == s) t += cxx;
        if (dir == awt::kDirTf) t += -w[i] * inv_tf;
    }
    return t;
}

struct HIn {
    const double* w;
    int kind, p, q;
    double cxx, inv_tf;
    awe::HDual operator()(int i) const {
        return awe::HDual(w[i], seed(kind, i, p, w, cxx, inv_tf), seed(kind, i, q, w, cxx, inv_tf), 0.0);
    }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 8) return 2;
    std::vector<double> cst = read(argv[1]), th = read(argv[2]), w = read(argv[3]);
    const double cxx = std::atof(argv[4]), inv_tf = std::atof(argv[5]), cb = std::atof(argv[6]),
                 cpp = std::atof(argv[7]);
    if ((int)cst.size() != AWE_NCONST || (int)th.size() != AWE_NTHETA0 || (int)w.size() != AWE_NW + 2) return 3;
    std::vector<double> mu(36);
    for (int r = 0; r < 36; ++r) mu[r] = std::sin(1.7 * r + 0.3);   // multipliers
    std::printf("{");
    for (int kind = 0; kind < 2; ++kind) {
        const int np = awe_hgen::kNPairs[kind];
        std::vector<double> hd(awe_hgen::kNHd[kind], std::nan("")), gd(AWE_NX, std::nan(""));
        PlainIn pin{w.data()};
        Ex ex{w.data(), cxx, inv_tf, cb, cpp, mu.data()};
        if (kind == 0) awe_hgen::ap2_hess_shoot(pin, th.data(), cst.data(), ex, hd.data());
        else awe_hgen::ap2_hess_radau(pin, th.data(), cst.data(), ex, hd.data(), gd.data());
        double dh = 0.0, dg = 0.0, hmax = 0.0;
        int nonzero = 0;
        for (int i = 0; i < np; ++i) {
            const int p = awe_hgen::kPairP[kind][i], q = awe_hgen::kPairQ[kind][i];
            HIn in{w.data(), kind, p, q, cxx, inv_tf};
            awe::NodeResult<awe::HDual> res;
            const awe::HDual gamma(w[awt::kDirGamma], p == awt::kDirGamma ? 1.0 : 0.0, q == awt::kDirGamma ? 1.0 : 0.0, 0.0);
            awe::ap2_node<awe::HDual>(in, gamma, th.data(), cst.data(), res, kind == 0);
            awe::HDual L(0.0);
            for (int r = 0; r < (kind == 0 ? AWE_N_EQ + AWE_N_INEQ : AWE_N_EQ); ++r)
                L = L + mu[r] * (r < AWE_N_EQ ? res.eq[r] : res.ineq[r - AWE_N_EQ]);
            if (kind == 1) {
                const awe::HDual psi(w[AWE_NW + 1], p == awt::kDirPsi ? 1.0 : 0.0, q == awt::kDirPsi ? 1.0 : 0.0, 0.0);
                L = L + cb * (res.bt * res.bt) + cpp * ((1.0 - psi) * res.pw);
            }
            const int row = awe_hgen::kHdRow[kind][i];
            const double got = row >= 0 ? hd[row] : 0.0;
            if (std::isnan(got)) { dh = INFINITY; continue; }
            dh = std::fmax(dh, std::fabs(got - L.ab) / std::fmax(1.0, std::fabs(L.ab)));
            hmax = std::fmax(hmax, std::fabs(L.ab));
            if (L.ab != 0.0) ++nonzero;
            // dL / d xdot_s from the first-order part of pair (23 + s, q)
            if (kind == 1 && p >= AWE_NX && p < 2 * AWE_NX) {
                const double g = gd[p - AWE_NX];
                dg = std::fmax(dg, std::fabs(g - L.a) / std::fmax(1.0, std::fabs(L.a)));
            }
        }
        std::printf("%s\"%s\": {\"hess_rel\": %.3e, \"grad_rel\": %.3e, \"hess_max\": %.3e, \"pairs\": %d, \"rows\": %d, \"nonzero\": %d}",
                    kind ? ", " : "", kind ? "radau" : "shooting", dh, dg, hmax, np, awe_hgen::kNHd[kind], nonzero);
    }
    std::printf("}\n");
    return 0;
}
