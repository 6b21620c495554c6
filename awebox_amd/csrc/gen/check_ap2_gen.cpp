// Host check of the generated node-Jacobian code (ap2_nodejac.gen.hpp) against the templated
// model on dual numbers (one forward pass per seed direction, the seeding of awegpu.hip's LaneIn).
//
//   check_ap2_gen <consts> <theta0> <node values (59 + gamma)> <cxx> <inv_tf>
//
// Prints one JSON line: the largest relative value and tangent differences per node kind.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <vector>

#include "../ap2_model.hpp"
#include "../ap2_nodejac.gen.hpp"
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

struct SeedIn {
    const double* w;
    int kind, dir;
    double cxx, inv_tf;
    awe::Dual operator()(int i) const {
        double t = (i == dir) ? 1.0 : 0.0;
        if (kind == 1 && i >= AWE_NX && i < 2 * AWE_NX) {
            const int s = i - AWE_NX;
            if (dir == s) t += cxx;
            if (dir == awt::kDirTf) t += -w[i] * inv_tf;
        }
        return awe::Dual(w[i], t);
    }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) return 2;
    std::vector<double> cst = read(argv[1]), th = read(argv[2]), w = read(argv[3]);
    const double cxx = std::atof(argv[4]), inv_tf = std::atof(argv[5]);
    if ((int)cst.size() != AWE_NCONST || (int)th.size() != AWE_NTHETA0 || (int)w.size() != AWE_NW + 1) return 3;
    std::printf("{");
    for (int kind = 0; kind < 2; ++kind) {
        std::vector<double> val(36, 0.0), tan(awe_gen::kNTan[kind], 0.0), dbp(64, 0.0), obv(2, 0.0);
        const double cb = 0.37, cpp = -1.9;   // objective weights of the beta^2 and power terms
        PlainIn pin{w.data()};
        if (kind == 0) awe_gen::ap2_node_shoot<1>(pin, th.data(), cst.data(), val.data(), tan.data());
        else awe_gen::ap2_node_radau<1>(pin, cxx, inv_tf, cb, cpp, th.data(), cst.data(), val.data(), tan.data(),
                                     dbp.data(), obv.data());
        double dv = 0.0, dt = 0.0, tmax = 0.0;
        int covered = 0;
        for (int dir = 0; dir <= awt::kDirGamma; ++dir) {
            SeedIn in{w.data(), kind, dir, cxx, inv_tf};
            awe::NodeResult<awe::Dual> res;
            awe::Dual gamma(w[awt::kDirGamma], dir == awt::kDirGamma ? 1.0 : 0.0);
            awe::ap2_node<awe::Dual>(in, gamma, th.data(), cst.data(), res, kind == 0);
            if (kind == 1) {   // objective terms cb beta^2 + cpp p
                if (dir == 0) {
                    dv = std::fmax(dv, std::fabs(obv[0] - res.bt.v) / std::fmax(1.0, std::fabs(res.bt.v)));
                    dv = std::fmax(dv, std::fabs(obv[1] - res.pw.v) / std::fmax(1.0, std::fabs(res.pw.v)));
                }
                const double ref = 2.0 * cb * res.bt.v * res.bt.d + cpp * res.pw.d;
                double got = 0.0;   // dbp is compact: entry i is direction kDbpDir[i]
                for (int i = 0; i < awe_gen::kNDbp; ++i)
                    if (awe_gen::kDbpDir[i] == dir) got = dbp[i];
                dt = std::fmax(dt, std::fabs(got - ref) / std::fmax(1.0, std::fabs(ref)));
            }
            for (int r = 0; r < AWE_N_EQ + AWE_N_INEQ; ++r) {
                if (kind == 1 && r >= AWE_N_EQ) continue;
                const awe::Dual ref = r < AWE_N_EQ ? res.eq[r] : res.ineq[r - AWE_N_EQ];
                if (dir == 0) dv = std::fmax(dv, std::fabs(val[r] - ref.v) / std::fmax(1.0, std::fabs(ref.v)));
                const int idx = awe_gen::kTanIdx[kind][r][dir];
                const double got = idx >= 0 ? tan[idx] : 0.0;
                if (idx >= 0) ++covered;
                tmax = std::fmax(tmax, std::fabs(ref.d));
                dt = std::fmax(dt, std::fabs(got - ref.d) / std::fmax(1.0, std::fabs(ref.d)));
            }
        }
        std::printf("%s\"%s\": {\"value_rel\": %.3e, \"tangent_rel\": %.3e, \"tangent_max\": %.3e, \"entries\": %d, "
                    "\"n_tan\": %d}", kind ? ", " : "", kind ? "radau" : "shooting", dv, dt, tmax, covered,
                    awe_gen::kNTan[kind]);
    }
    std::printf("}\n");
    return 0;
}
