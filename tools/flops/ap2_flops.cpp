// Algorithmic floating-point operation count of one AP2 NLP evaluation {f, g, grad f, J_g}
// ("count them once with an op-counting scalar type on the CPU
// restatement").  A measurement tool, not product code.
//
// The node model (awebox_amd/csrc/ap2_model.hpp) is instantiated on Cnt: a value plus the set of
// colours (the compressed Jacobian directions of the node kind, ap2_tables.hpp) its tangent
// structurally depends on.  Every operation counts
//   value flops    once per node: + - * / as 1, sqrt exp log sin cos as 1 transcendental;
//   tangent flops  per colour of the result's tangent, the forward-mode rule's operations:
//                  a+-b: 1 if both depend on the colour (else a copy), a*b: 3 (1 if one
//                  depends), a/b: 3 (1 if only a, 2 if only b), const*a, a/const: 1, f(a): 1.
// This is the work of compressed forward-mode differentiation with the kernel's colouring when
// nothing is recomputed: the kernel evaluates the value part in each of a node's 32 lanes and
// the tangent of every lane's colour whether or not it is structurally zero, so its issued FP64
// operations exceed this count.  The assembly around the node model (xdot polynomial, objective
// directional derivatives, continuity rows, gradient columns, the Jacobian gather scaling and the
// finalize reduction) is counted operation by operation from the kernel's loops.
//
//   g++ -O2 -std=c++17 -I awebox_amd/csrc -I include tools/flops/ap2_flops.cpp -o /tmp/ap2_flops
//   /tmp/ap2_flops <n_k> <d> <consts file: one double per line>
#include <bitset>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "ap2_tables.hpp"

namespace cnt {

struct Counters {
    double value = 0, trans = 0, tangent = 0;
};
static Counters C;

inline int pc(uint32_t m) { return __builtin_popcount(m); }

struct Cnt {
    double v;
    uint32_t m;   // colours the tangent depends on
    Cnt() : v(0.0), m(0) {}
    Cnt(double a) : v(a), m(0) {}
    Cnt(double a, uint32_t mm) : v(a), m(mm) {}
};

inline Cnt add_like(double v, const Cnt& a, const Cnt& b) {
    C.value += 1;
    C.tangent += pc(a.m & b.m);       // both: one add per colour; one side: a copy
    return Cnt(v, a.m | b.m);
}
inline Cnt operator+(const Cnt& a, const Cnt& b) { return add_like(a.v + b.v, a, b); }
inline Cnt operator-(const Cnt& a, const Cnt& b) { return add_like(a.v - b.v, a, b); }
inline Cnt operator-(const Cnt& a) { return Cnt(-a.v, a.m); }
inline Cnt operator*(const Cnt& a, const Cnt& b) {
    C.value += 1;
    C.tangent += 3 * pc(a.m & b.m) + pc(a.m ^ b.m);
    return Cnt(a.v * b.v, a.m | b.m);
}
inline Cnt operator/(const Cnt& a, const Cnt& b) {
    C.value += 1;
    C.tangent += 3 * pc(a.m & b.m) + pc(a.m & ~b.m) + 2 * pc(b.m & ~a.m);
    return Cnt(a.v / b.v, a.m | b.m);
}
inline Cnt operator+(const Cnt& a, double b) { C.value += 1; return Cnt(a.v + b, a.m); }
inline Cnt operator+(double a, const Cnt& b) { C.value += 1; return Cnt(a + b.v, b.m); }
inline Cnt operator-(const Cnt& a, double b) { C.value += 1; return Cnt(a.v - b, a.m); }
inline Cnt operator-(double a, const Cnt& b) { C.value += 1; return Cnt(a - b.v, b.m); }
inline Cnt operator*(const Cnt& a, double b) { C.value += 1; C.tangent += pc(a.m); return Cnt(a.v * b, a.m); }
inline Cnt operator*(double a, const Cnt& b) { return b * a; }
inline Cnt operator/(const Cnt& a, double b) { C.value += 1; C.tangent += pc(a.m); return Cnt(a.v / b, a.m); }
inline Cnt operator/(double a, const Cnt& b) {
    C.value += 1;
    C.tangent += 2 * pc(b.m);
    return Cnt(a / b.v, b.m);
}
inline Cnt& operator+=(Cnt& a, const Cnt& b) { a = a + b; return a; }
inline Cnt& operator-=(Cnt& a, const Cnt& b) { a = a - b; return a; }
inline Cnt& operator*=(Cnt& a, const Cnt& b) { a = a * b; return a; }
inline Cnt unary(double v, const Cnt& a, int extra_value) {
    C.trans += 1;
    C.value += extra_value;           // the derivative coefficient (e.g. 0.5 / s), once
    C.tangent += pc(a.m);
    return Cnt(v, a.m);
}
inline Cnt sqrt(const Cnt& a) { return unary(std::sqrt(a.v), a, a.m ? 2 : 0); }
inline Cnt exp(const Cnt& a) { return unary(std::exp(a.v), a, 0); }
inline Cnt log(const Cnt& a) { return unary(std::log(a.v), a, a.m ? 1 : 0); }
inline Cnt sin(const Cnt& a) { C.trans += a.m ? 1 : 0; return unary(std::sin(a.v), a, 0); }
inline Cnt cos(const Cnt& a) { C.trans += a.m ? 1 : 0; return unary(std::cos(a.v), a, 0); }
inline double value(const Cnt& a) { return a.v; }

}  // namespace cnt

namespace awe {
using cnt::Cnt;
using cnt::sqrt;
using cnt::exp;
using cnt::log;
using cnt::sin;
using cnt::cos;
using cnt::value;
}  // namespace awe

using namespace awt;
using cnt::Cnt;

struct CntIn {
    const double* w;
    const ColorTabs* ct;
    int kind;
    Cnt operator()(int i) const {
        uint32_t m = 0;
        for (int c = 0; c < kHalf; ++c) {
            bool dep = (ct->seedA[kind][c] >> i) & 1ull;
            if (i >= AWE_NX && i < 2 * AWE_NX) {
                const int j = i - AWE_NX;
                dep = dep || ((ct->seedA[kind][c] >> j) & 1ull) || ((ct->seedXD[kind][c] >> j) & 1u) ||
                      c == ct->tf_color[kind];
            }
            if (dep) m |= 1u << c;
        }
        return Cnt(w[i], m);
    }
};

struct CntSink {
    void eq_row(int, const Cnt&) {}
    void ineq_row(int, const Cnt&) {}
    void power(const Cnt&) {}
    void beta(const Cnt&) {}
};

int main(int argc, char** argv) {
    if (argc < 4) { std::fprintf(stderr, "usage: ap2_flops n_k d consts_file\n"); return 2; }
    const int n_k = std::atoi(argv[1]), d = std::atoi(argv[2]);
    std::vector<double> consts;
    {
        std::ifstream in(argv[3]);
        double x;
        while (in >> x) consts.push_back(x);
    }
    Ap2Tables T;
    std::string err;
    if (build_ap2_tables(n_k, d, consts.data(), (int)consts.size(), T, err)) {
        std::fprintf(stderr, "tables: %s\n", err.c_str());
        return 1;
    }
    const ColorTabs& ct = T.ct;
    const int NN = d + 1;
    // a generic node point: the values do not change the operation count (the model has no
    // data-dependent branches), only the structure does
    std::vector<double> th(AWE_NTHETA0, 0.5), w(64, 0.3);
    th[AWE_TH_G] = 9.81; th[AWE_TH_GAMMA_AIR] = 6.5e-3; th[AWE_TH_R] = 287.053; th[AWE_TH_T_REF] = 288.15;
    th[AWE_TH_RHO_REF] = 1.225; th[AWE_TH_Z_REF] = 100.0; th[AWE_TH_U_REF] = 10.0; th[AWE_TH_EXP_REF] = 0.15;
    double node_value[2], node_trans[2], node_tangent[2];
    for (int kind = 0; kind < 2; ++kind) {
        cnt::C = cnt::Counters{};
        CntIn in{w.data(), &ct, kind};
        CntSink sink;
        uint32_t gm = 0;
        for (int c = 0; c < kHalf; ++c)
            if ((ct.seedA[kind][c] >> kDirGamma) & 1ull) gm |= 1u << c;
        awe::ap2_node<Cnt>(in, Cnt(0.3, gm), th.data(), T.cst.data(), sink, kind == 0);
        node_value[kind] = cnt::C.value;
        node_trans[kind] = cnt::C.trans;
        node_tangent[kind] = cnt::C.tangent;
    }
    // assembly per interval, from ap2_interval_kernel's loops (awegpu.hip)
    double asm_xdot = (double)d * AWE_NX * (2.0 * NN + 1.0);          // sum_r C X_r, times 1/(h t_f)
    double asm_obj = 0.0;                                              // per Radau node
    {
        const double per_x = 13.0, per_xd = 7.0, per_u = 8.0, per_z = 9.0, per_diam = 8.0;
        double o = AWE_NX * per_x + AWE_NX * per_xd + AWE_NU * per_u + per_z + per_diam;
        o += 3.0 * 3.0 + 3.0 * 2.0 + 8.0;          // wave sums of three partial sums, tf / psi columns, f node
        for (int dir = 0; dir < kDirs; ++dir) {
            if (ct.obj_beta[dir] >= 0) o += 4.0;
            if (ct.obj_power[dir] >= 0) o += 4.0;
        }
        asm_obj = d * o;
    }
    int nD = 0;
    for (int r = 0; r < NN; ++r) nD += T.dcoll.D[r] != 0.0;
    double asm_cont = AWE_NX * (2.0 * nD + 1.0);
    double asm_grad = AWE_NX * 3.0 * d + AWE_NU * d + d * AWE_NX * (1.0 + 3.0 * (d - 1)) + 3.0 * d;
    double asm_interval = asm_xdot + asm_obj + asm_cont + asm_grad;
    double jac = (double)T.nnz;                                        // one scaling multiply per entry
    double finalize = 4.0 * n_k + 64.0;
    double model = n_k * (node_value[0] + node_tangent[0] + node_trans[0] +
                          d * (node_value[1] + node_tangent[1] + node_trans[1]));
    double total = model + n_k * asm_interval + jac + finalize;
    std::printf("{\"n_k\": %d, \"d\": %d, \"nnz\": %d, "
                "\"node\": {\"shooting\": {\"value\": %.0f, \"transcendental\": %.0f, \"tangent\": %.0f}, "
                "\"radau\": {\"value\": %.0f, \"transcendental\": %.0f, \"tangent\": %.0f}}, "
                "\"assembly_per_interval\": {\"xdot\": %.0f, \"objective\": %.0f, \"continuity\": %.0f, \"gradient\": %.0f}, "
                "\"model_flops\": %.0f, \"assembly_flops\": %.0f, \"jacobian_scaling_flops\": %.0f, "
                "\"finalize_flops\": %.0f, \"flops_per_eval\": %.0f}\n",
                n_k, d, T.nnz, node_value[0], node_trans[0], node_tangent[0], node_value[1], node_trans[1],
                node_tangent[1], asm_xdot, asm_obj, asm_cont, asm_grad, model, n_k * asm_interval, jac, finalize,
                total);
    return 0;
}
