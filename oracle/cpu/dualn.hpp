// Vector forward-mode dual number for the CPU port: one value and N tangents, so one model
// evaluation yields all N (compressed) directions.  The loops vectorise (AVX2/AVX-512).
#pragma once

#include <cmath>

namespace cpu {

template <int N>
struct DualN {
    double v;
    double d[N];
    DualN() : v(0.0) { for (int i = 0; i < N; ++i) d[i] = 0.0; }
    DualN(double a) : v(a) { for (int i = 0; i < N; ++i) d[i] = 0.0; }
};

#define DN template <int N> inline DualN<N>
DN operator+(const DualN<N>& a, const DualN<N>& b) {
    DualN<N> r; r.v = a.v + b.v;
    for (int i = 0; i < N; ++i) r.d[i] = a.d[i] + b.d[i];
    return r;
}
DN operator-(const DualN<N>& a, const DualN<N>& b) {
    DualN<N> r; r.v = a.v - b.v;
    for (int i = 0; i < N; ++i) r.d[i] = a.d[i] - b.d[i];
    return r;
}
DN operator-(const DualN<N>& a) {
    DualN<N> r; r.v = -a.v;
    for (int i = 0; i < N; ++i) r.d[i] = -a.d[i];
    return r;
}
DN operator*(const DualN<N>& a, const DualN<N>& b) {
    DualN<N> r; r.v = a.v * b.v;
    for (int i = 0; i < N; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
    return r;
}
DN operator/(const DualN<N>& a, const DualN<N>& b) {
    const double rb = 1.0 / b.v, q = a.v * rb;
    DualN<N> r; r.v = q;
    for (int i = 0; i < N; ++i) r.d[i] = (a.d[i] - q * b.d[i]) * rb;
    return r;
}
DN operator+(const DualN<N>& a, double b) { DualN<N> r = a; r.v += b; return r; }
DN operator+(double a, const DualN<N>& b) { DualN<N> r = b; r.v += a; return r; }
DN operator-(const DualN<N>& a, double b) { DualN<N> r = a; r.v -= b; return r; }
DN operator-(double a, const DualN<N>& b) {
    DualN<N> r; r.v = a - b.v;
    for (int i = 0; i < N; ++i) r.d[i] = -b.d[i];
    return r;
}
DN operator*(const DualN<N>& a, double b) {
    DualN<N> r; r.v = a.v * b;
    for (int i = 0; i < N; ++i) r.d[i] = a.d[i] * b;
    return r;
}
DN operator*(double a, const DualN<N>& b) { return b * a; }
DN operator/(const DualN<N>& a, double b) { return a * (1.0 / b); }
DN operator/(double a, const DualN<N>& b) {
    const double rb = 1.0 / b.v, q = a * rb;
    DualN<N> r; r.v = q;
    for (int i = 0; i < N; ++i) r.d[i] = -q * b.d[i] * rb;
    return r;
}
DN sqrt(const DualN<N>& a) {
    const double s = std::sqrt(a.v), h = 0.5 / s;
    DualN<N> r; r.v = s;
    for (int i = 0; i < N; ++i) r.d[i] = a.d[i] * h;
    return r;
}
DN exp(const DualN<N>& a) {
    const double e = std::exp(a.v);
    DualN<N> r; r.v = e;
    for (int i = 0; i < N; ++i) r.d[i] = e * a.d[i];
    return r;
}
DN log(const DualN<N>& a) {
    const double ra = 1.0 / a.v;
    DualN<N> r; r.v = std::log(a.v);
    for (int i = 0; i < N; ++i) r.d[i] = a.d[i] * ra;
    return r;
}
#undef DN

}  // namespace cpu
