// Host check of the generated dual-kite node-Jacobian code (dual_nodejac.gen.hpp: four wavefront
// roles per node kind) against the templated two-kite model on dual numbers -- one forward pass per
// seed direction with the seeding of awedual.hip's colour kernel (DLaneIn) -- for the row values,
// every tangent slot, the power and side-slip values and the directional derivatives of the Radau
// node's objective terms ex2 (beta_2^2 + beta_3^2) + ex3 p.
//
//   check_dual_gen <consts> <theta0 (200)> <node values (126 + gamma)> <cxx> <inv_tf> <ex2> <ex3>
//
// Prints one JSON line: the largest relative differences per node kind.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <type_traits>
#include <vector>

#include "../dual_nodejac.gen.hpp"
#include "../dual_tables.hpp"

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
        if (kind == 1 && i >= ADL_NX && i < 2 * ADL_NX) {
            if (dir == i - ADL_NX) t += cxx;
            if (dir == awe::dl::kTf) t += -w[i] * inv_tf;
        }
        return awe::Dual(w[i], t);
    }
};

struct RowSink {
    awe::Dual rows[dlt::kNRows];
    void eq_row(int r, const awe::Dual& v) { rows[r] = v; }
    void ineq_row(int r, const awe::Dual& v) { rows[ADL_N_EQ + r] = v; }
    void power(const awe::Dual& v) { rows[dlt::kRowPower] = v; }
    void beta(int k, const awe::Dual& v) { rows[dlt::kRowBeta0 + k] = v; }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc < 8) return 2;
    std::vector<double> cst = read(argv[1]), th = read(argv[2]), w = read(argv[3]);
    const double cxx = std::atof(argv[4]), inv_tf = std::atof(argv[5]), ex2 = std::atof(argv[6]),
                 ex3 = std::atof(argv[7]);
    if ((int)cst.size() != ADL_NCONST || (int)th.size() != AWE_NTHETA0 || (int)w.size() != dlt::kDirs) return 3;
    std::printf("{");
    for (int kind = 0; kind < 2; ++kind) {
        std::vector<double> val(dlt::kRowPower, 0.0), tan(awe_dgen::kNTan[kind], 0.0);
        std::vector<double> obv(3, 0.0), dbp(awe_dgen::kNDbp, 0.0);
        PlainIn pin{w.data()};
        auto role = [&](auto rl) {
            constexpr int G = decltype(rl)::value;
            if (kind == 0) awe_dgen::dual_node_shoot<1, G>(pin, th.data(), cst.data(), val.data(), tan.data());
            else
                awe_dgen::dual_node_radau<1, G>(pin, cxx, inv_tf, ex2, ex3, th.data(), cst.data(), val.data(),
                                                tan.data(), dbp.data(), obv.data());
        };
        role(std::integral_constant<int, 0>{});
        role(std::integral_constant<int, 1>{});
        role(std::integral_constant<int, 2>{});
        role(std::integral_constant<int, 3>{});
        static_assert(awe_dgen::kRoles == 4, "checker runs four roles");
        double dv = 0.0, dt = 0.0, tmax = 0.0, dobv = 0.0, ddbp = 0.0;
        int covered = 0;
        const int nrows = kind == 0 ? dlt::kRowPower : ADL_N_EQ;
        for (int dir = 0; dir < dlt::kDirs; ++dir) {
            SeedIn in{w.data(), kind, dir, kind ? cxx : 0.0, inv_tf};
            RowSink res;
            awe::Dual gamma(w[awe::dl::kGamma], dir == awe::dl::kGamma ? 1.0 : 0.0);
            awe::dual_node<awe::Dual>(in, gamma, th.data(), cst.data(), res, kind == 0);
            for (int r = 0; r < nrows; ++r) {
                const awe::Dual ref = res.rows[r];
                if (dir == 0) dv = std::fmax(dv, std::fabs(val[r] - ref.v) / std::fmax(1.0, std::fabs(ref.v)));
                const int idx = awe_dgen::kTanIdx[kind][r][dir];
                const double got = idx >= 0 ? tan[idx] : 0.0;
                if (idx >= 0) ++covered;
                tmax = std::fmax(tmax, std::fabs(ref.d));
                dt = std::fmax(dt, std::fabs(got - ref.d) / std::fmax(1.0, std::fabs(ref.d)));
            }
            if (kind == 1) {
                const awe::Dual p = res.rows[dlt::kRowPower], b0 = res.rows[dlt::kRowBeta0],
                                b1 = res.rows[dlt::kRowBeta0 + 1];
                if (dir == 0) {
                    const double ref[3] = {p.v, b0.v, b1.v};
                    for (int e = 0; e < 3; ++e)
                        dobv = std::fmax(dobv, std::fabs(obv[e] - ref[e]) / std::fmax(1.0, std::fabs(ref[e])));
                }
                if (dir == awe::dl::kGamma) continue;
                const double want = 2.0 * ex2 * (b0.v * b0.d + b1.v * b1.d) + ex3 * p.d;
                double got = 0.0;
                for (int q = 0; q < awe_dgen::kNDbp; ++q)
                    if (awe_dgen::kDbpDir[q] == dir) got += dbp[q];
                ddbp = std::fmax(ddbp, std::fabs(got - want) / std::fmax(1.0, std::fabs(want)));
            }
        }
        std::printf("%s\"%s\": {\"value_rel\": %.3e, \"tangent_rel\": %.3e, \"tangent_max\": %.3e, \"entries\": %d, "
                    "\"n_tan\": %d, \"obv_rel\": %.3e, \"dbp_rel\": %.3e}",
                    kind ? ", " : "", kind ? "radau" : "shooting", dv, dt, tmax, covered, awe_dgen::kNTan[kind], dobv,
                    ddbp);
    }
    std::printf("}\n");
    return 0;
}
