// Host check of the generated MPC node-Jacobian code (kite3_nodejac.gen.hpp) against the templated
// 3-DOF model on dual numbers (one forward pass per seed direction, the seeding of awempc.hip's LaneIn).
//
//   check_kite3_gen <consts (55)> <node values (31 + gamma)> <u_ref> <cxx> <inv_tf>
//
// Prints one JSON line: the largest relative value and tangent differences per node kind.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <type_traits>
#include <vector>

#include "../kite3_nodejac.gen.hpp"
#include "../kite3_tables.hpp"

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
        if (kind == 1 && i >= K3_NX && i < 2 * K3_NX) {
            if (dir == i - K3_NX) t += cxx;
            if (dir == k3t::kDirTf) t += -w[i] * inv_tf;
        }
        return awe::Dual(w[i], t);
    }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) return 2;
    std::vector<double> cst = read(argv[1]), w = read(argv[2]);
    const double u_ref = std::atof(argv[3]), cxx = std::atof(argv[4]), inv_tf = std::atof(argv[5]);
    if ((int)cst.size() != K3_NCONST || (int)w.size() != k3t::kLanes) return 3;
    std::printf("{");
    for (int kind = 0; kind < 2; ++kind) {
        std::vector<double> val(k3t::kRowsPerNode, 0.0), tan(awe_k3gen::kNTan[kind], 0.0);
        PlainIn pin{w.data()};
        auto strip = [&](auto st) {   // every direction strip of the generated code
            constexpr int S = decltype(st)::value;
            if constexpr (S < awe_k3gen::kNStrips) {
                if (kind == 0) awe_k3gen::k3_node_shoot<1, S>(pin, u_ref, cst.data(), val.data(), tan.data());
                else awe_k3gen::k3_node_radau<1, S>(pin, u_ref, cxx, inv_tf, cst.data(), val.data(), tan.data());
            }
        };
        strip(std::integral_constant<int, 0>{});
        strip(std::integral_constant<int, 1>{});
        strip(std::integral_constant<int, 2>{});
        strip(std::integral_constant<int, 3>{});
        static_assert(awe_k3gen::kNStrips <= 4, "checker covers up to 4 strips");
        double dv = 0.0, dt = 0.0, tmax = 0.0;
        int covered = 0;
        const int nrows = kind == 0 ? k3t::kRowsPerNode : K3_N_EQ;
        for (int dir = 0; dir < k3t::kLanes; ++dir) {
            SeedIn in{w.data(), kind, dir, cxx, inv_tf};
            awe::Kite3Result<awe::Dual> res;
            awe::Dual gamma(w[k3t::kDirGamma], dir == k3t::kDirGamma ? 1.0 : 0.0);
            awe::kite3_node<awe::Dual>(in, gamma, u_ref, cst.data(), res, kind == 0);
            for (int r = 0; r < nrows; ++r) {
                const awe::Dual ref = r < K3_N_EQ ? res.eq[r] : res.ineq[r - K3_N_EQ];
                if (dir == 0) dv = std::fmax(dv, std::fabs(val[r] - ref.v) / std::fmax(1.0, std::fabs(ref.v)));
                const int idx = awe_k3gen::kTanIdx[kind][r][dir];
                const double got = idx >= 0 ? tan[idx] : 0.0;
                if (idx >= 0) ++covered;
                tmax = std::fmax(tmax, std::fabs(ref.d));
                dt = std::fmax(dt, std::fabs(got - ref.d) / std::fmax(1.0, std::fabs(ref.d)));
            }
        }
        std::printf("%s\"%s\": {\"value_rel\": %.3e, \"tangent_rel\": %.3e, \"tangent_max\": %.3e, \"entries\": %d, "
                    "\"n_tan\": %d}", kind ? ", " : "", kind ? "radau" : "shooting", dv, dt, tmax, covered,
                    awe_k3gen::kNTan[kind]);
    }
    std::printf("}\n");
    return 0;
}
