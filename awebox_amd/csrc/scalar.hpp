// Scalar types the AP2 node model is instantiated with.
//
//   double  -- value only (f/g evaluation)
//   Dual    -- forward-mode derivative along ONE direction; on the GPU every lane of a
//              wavefront carries a different direction, so one wavefront produces a full
//              node Jacobian block
//   HDual   -- hyper-dual number: mixed second derivative along two directions (Hessian)
//   Dep     -- structural dependency bitmask over <= 64 node inputs; used once on the host to
//              derive the fixed CCS sparsity of the constraint Jacobian (what CasADi's
//              symbolic sparsity propagation provides in the reference, preparation.py:366-400)
#pragma once

#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define AWE_HD __host__ __device__ __forceinline__
#else
#define AWE_HD inline
#endif

namespace awe {

// ------------------------------------------------------------------------------------------
struct Dual {
    double v, d;
    AWE_HD Dual() : v(0.0), d(0.0) {}
    AWE_HD Dual(double a) : v(a), d(0.0) {}
    AWE_HD Dual(double a, double b) : v(a), d(b) {}
};

AWE_HD Dual operator+(Dual a, Dual b) { return Dual(a.v + b.v, a.d + b.d); }
AWE_HD Dual operator-(Dual a, Dual b) { return Dual(a.v - b.v, a.d - b.d); }
AWE_HD Dual operator-(Dual a) { return Dual(-a.v, -a.d); }
AWE_HD Dual operator*(Dual a, Dual b) { return Dual(a.v * b.v, a.d * b.v + a.v * b.d); }
// 1/x: hardware v_rcp_f64 (~2^-23 relative) refined by two Newton steps to ~1 ulp.  The dual
// quotient rules below use one reciprocal each instead of two IEEE division sequences.
AWE_HD double rcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    return __builtin_fma(r, e, r);
#else
    return 1.0 / x;
#endif
}

AWE_HD Dual operator/(Dual a, Dual b) {
    double r = rcp(b.v);
    double q = a.v * r;
    return Dual(q, (a.d - q * b.d) * r);
}
AWE_HD Dual operator+(Dual a, double b) { return Dual(a.v + b, a.d); }
AWE_HD Dual operator+(double a, Dual b) { return Dual(a + b.v, b.d); }
AWE_HD Dual operator-(Dual a, double b) { return Dual(a.v - b, a.d); }
AWE_HD Dual operator-(double a, Dual b) { return Dual(a - b.v, -b.d); }
AWE_HD Dual operator*(Dual a, double b) { return Dual(a.v * b, a.d * b); }
AWE_HD Dual operator*(double a, Dual b) { return Dual(a * b.v, a * b.d); }
AWE_HD Dual operator/(Dual a, double b) {
    // b is a model constant: a literal folds to its reciprocal, a run-time constant costs one
    // reciprocal instead of two divisions
    double r = __builtin_constant_p(b) ? 1.0 / b : rcp(b);
    return Dual(a.v * r, a.d * r);
}
AWE_HD Dual operator/(double a, Dual b) {
    double r = rcp(b.v);
    double q = a * r;
    return Dual(q, -q * b.d * r);
}
AWE_HD Dual& operator+=(Dual& a, Dual b) { a = a + b; return a; }
AWE_HD Dual& operator-=(Dual& a, Dual b) { a = a - b; return a; }
AWE_HD Dual& operator*=(Dual& a, Dual b) { a = a * b; return a; }

AWE_HD Dual sqrt(Dual a) {
    double s = ::sqrt(a.v);
    return Dual(s, a.d * 0.5 * rcp(s));
}
AWE_HD Dual exp(Dual a) {
    double e = ::exp(a.v);
    return Dual(e, e * a.d);
}
AWE_HD Dual log(Dual a) { return Dual(::log(a.v), a.d * rcp(a.v)); }
AWE_HD Dual sin(Dual a) { return Dual(::sin(a.v), ::cos(a.v) * a.d); }
AWE_HD Dual cos(Dual a) { return Dual(::cos(a.v), -::sin(a.v) * a.d); }
AWE_HD double value(Dual a) { return a.v; }
AWE_HD double tangent(Dual a) { return a.d; }

// ------------------------------------------------------------------------------------------
// Hyper-dual number v + a e1 + b e2 + ab e1 e2 (e1^2 = e2^2 = 0): forward-over-forward second
// derivatives.  With e1, e2 seeded along two directions, ab is the mixed second derivative.
struct HDual {
    double v, a, b, ab;
    AWE_HD HDual() : v(0.0), a(0.0), b(0.0), ab(0.0) {}
    AWE_HD HDual(double x) : v(x), a(0.0), b(0.0), ab(0.0) {}
    AWE_HD HDual(double x, double xa, double xb, double xab) : v(x), a(xa), b(xb), ab(xab) {}
};
AWE_HD HDual operator+(HDual x, HDual y) { return HDual(x.v + y.v, x.a + y.a, x.b + y.b, x.ab + y.ab); }
AWE_HD HDual operator-(HDual x, HDual y) { return HDual(x.v - y.v, x.a - y.a, x.b - y.b, x.ab - y.ab); }
AWE_HD HDual operator-(HDual x) { return HDual(-x.v, -x.a, -x.b, -x.ab); }
AWE_HD HDual operator*(HDual x, HDual y) {
    return HDual(x.v * y.v, x.a * y.v + x.v * y.a, x.b * y.v + x.v * y.b,
                 x.ab * y.v + x.a * y.b + x.b * y.a + x.v * y.ab);
}
// f(x) for a scalar function with value f0 and derivatives f1, f2 at x.v (chain rule)
AWE_HD HDual hd_apply(HDual x, double f0, double f1, double f2) {
    return HDual(f0, f1 * x.a, f1 * x.b, f1 * x.ab + f2 * x.a * x.b);
}
AWE_HD HDual operator/(HDual x, HDual y) {
    const double r = rcp(y.v);
    return x * hd_apply(y, r, -r * r, 2.0 * r * r * r);
}
AWE_HD HDual operator+(HDual x, double y) { return HDual(x.v + y, x.a, x.b, x.ab); }
AWE_HD HDual operator+(double x, HDual y) { return HDual(x + y.v, y.a, y.b, y.ab); }
AWE_HD HDual operator-(HDual x, double y) { return HDual(x.v - y, x.a, x.b, x.ab); }
AWE_HD HDual operator-(double x, HDual y) { return HDual(x - y.v, -y.a, -y.b, -y.ab); }
AWE_HD HDual operator*(HDual x, double y) { return HDual(x.v * y, x.a * y, x.b * y, x.ab * y); }
AWE_HD HDual operator*(double x, HDual y) { return HDual(x * y.v, x * y.a, x * y.b, x * y.ab); }
AWE_HD HDual operator/(HDual x, double y) {
    const double r = __builtin_constant_p(y) ? 1.0 / y : rcp(y);
    return x * r;
}
AWE_HD HDual operator/(double x, HDual y) {
    const double r = rcp(y.v);
    return x * hd_apply(y, r, -r * r, 2.0 * r * r * r);
}
AWE_HD HDual sqrt(HDual x) {
    const double s = ::sqrt(x.v), r = rcp(s);
    return hd_apply(x, s, 0.5 * r, -0.25 * r * r * r);
}
AWE_HD HDual exp(HDual x) {
    const double e = ::exp(x.v);
    return hd_apply(x, e, e, e);
}
AWE_HD HDual log(HDual x) {
    const double r = rcp(x.v);
    return hd_apply(x, ::log(x.v), r, -r * r);
}

// ------------------------------------------------------------------------------------------
struct Dep {
    uint64_t m;
    AWE_HD Dep() : m(0) {}
    AWE_HD Dep(double) : m(0) {}
    AWE_HD static Dep bit(int i) { Dep d; d.m = (uint64_t)1 << i; return d; }
};
AWE_HD Dep mk_dep(uint64_t m) { Dep d; d.m = m; return d; }
AWE_HD Dep operator+(Dep a, Dep b) { return mk_dep(a.m | b.m); }
AWE_HD Dep operator-(Dep a, Dep b) { return mk_dep(a.m | b.m); }
AWE_HD Dep operator-(Dep a) { return a; }
AWE_HD Dep operator*(Dep a, Dep b) { return mk_dep(a.m | b.m); }
AWE_HD Dep operator/(Dep a, Dep b) { return mk_dep(a.m | b.m); }
AWE_HD Dep operator+(Dep a, double) { return a; }
AWE_HD Dep operator+(double, Dep b) { return b; }
AWE_HD Dep operator-(Dep a, double) { return a; }
AWE_HD Dep operator-(double, Dep b) { return b; }
AWE_HD Dep operator*(Dep a, double) { return a; }
AWE_HD Dep operator*(double, Dep b) { return b; }
AWE_HD Dep operator/(Dep a, double) { return a; }
AWE_HD Dep operator/(double, Dep b) { return b; }
AWE_HD Dep& operator+=(Dep& a, Dep b) { a.m |= b.m; return a; }
AWE_HD Dep& operator-=(Dep& a, Dep b) { a.m |= b.m; return a; }
AWE_HD Dep& operator*=(Dep& a, Dep b) { a.m |= b.m; return a; }
AWE_HD Dep sqrt(Dep a) { return a; }
AWE_HD Dep exp(Dep a) { return a; }
AWE_HD Dep log(Dep a) { return a; }
AWE_HD Dep sin(Dep a) { return a; }
AWE_HD Dep cos(Dep a) { return a; }

// Dep over <= 128 inputs (the multi-kite node has 126 variables + phi.gamma); host only.
struct Dep2 {
    uint64_t lo, hi;
    AWE_HD Dep2() : lo(0), hi(0) {}
    AWE_HD Dep2(double) : lo(0), hi(0) {}
    AWE_HD static Dep2 bit(int i) {
        Dep2 d;
        if (i < 64) d.lo = (uint64_t)1 << i; else d.hi = (uint64_t)1 << (i - 64);
        return d;
    }
    AWE_HD bool has(int i) const { return i < 64 ? ((lo >> i) & 1u) : ((hi >> (i - 64)) & 1u); }
};
AWE_HD Dep2 mk_dep2(uint64_t lo, uint64_t hi) { Dep2 d; d.lo = lo; d.hi = hi; return d; }
AWE_HD Dep2 operator+(Dep2 a, Dep2 b) { return mk_dep2(a.lo | b.lo, a.hi | b.hi); }
AWE_HD Dep2 operator-(Dep2 a, Dep2 b) { return mk_dep2(a.lo | b.lo, a.hi | b.hi); }
AWE_HD Dep2 operator-(Dep2 a) { return a; }
AWE_HD Dep2 operator*(Dep2 a, Dep2 b) { return mk_dep2(a.lo | b.lo, a.hi | b.hi); }
AWE_HD Dep2 operator/(Dep2 a, Dep2 b) { return mk_dep2(a.lo | b.lo, a.hi | b.hi); }
AWE_HD Dep2 operator+(Dep2 a, double) { return a; }
AWE_HD Dep2 operator+(double, Dep2 b) { return b; }
AWE_HD Dep2 operator-(Dep2 a, double) { return a; }
AWE_HD Dep2 operator-(double, Dep2 b) { return b; }
AWE_HD Dep2 operator*(Dep2 a, double) { return a; }
AWE_HD Dep2 operator*(double, Dep2 b) { return b; }
AWE_HD Dep2 operator/(Dep2 a, double) { return a; }
AWE_HD Dep2 operator/(double, Dep2 b) { return b; }
AWE_HD Dep2 sqrt(Dep2 a) { return a; }
AWE_HD Dep2 exp(Dep2 a) { return a; }
AWE_HD Dep2 log(Dep2 a) { return a; }

// integer structure read from a model constant (element counts, table lengths); the tracing
// scalar of the code generator (gen/sym.hpp) overloads it with the value recorded at trace time
AWE_HD int structural(double a) { return (int)a; }

AWE_HD double value(double a) { return a; }
AWE_HD double sqrt(double a) { return ::sqrt(a); }
AWE_HD double exp(double a) { return ::exp(a); }
AWE_HD double log(double a) { return ::log(a); }
AWE_HD double sin(double a) { return ::sin(a); }
AWE_HD double cos(double a) { return ::cos(a); }

}  // namespace awe
