// cfx_dual.h — forward-mode derivative numbers used by the gfx950 kernels.
//
// Dual<D>: value + D first-order directions (Jacobian columns carried through the RK recursion).
// Jet<D>:  value + D first-order directions + the D(D+1)/2 second-order terms (packed lower
//          triangle, (i,j) with j <= i at i*(i+1)/2 + j) for Lagrangian-Hessian blocks.
// Everything is compile-time sized so the compiler keeps it in VGPRs and unrolls every loop; D = 0
// degenerates to a plain double.  Values are computed with the same operation as the double path
// (q = a / b, never a * (1/b)) so g is identical whether or not derivatives are requested.
#pragma once

#include <hip/hip_runtime.h>

namespace cfx {

#define CFX_HD __device__ __forceinline__

template <int D>
struct Dual {
    double v;
    double d[D > 0 ? D : 1];
};

template <int D>
CFX_HD Dual<D> dconst(double v) {
    Dual<D> r;
    r.v = v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = 0.0;
    return r;
}

template <int D>
CFX_HD Dual<D> operator+(const Dual<D>& a, const Dual<D>& b) {
    Dual<D> r;
    r.v = a.v + b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = a.d[i] + b.d[i];
    return r;
}
template <int D>
CFX_HD Dual<D> operator-(const Dual<D>& a, const Dual<D>& b) {
    Dual<D> r;
    r.v = a.v - b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = a.d[i] - b.d[i];
    return r;
}
template <int D>
CFX_HD Dual<D> operator+(const Dual<D>& a, double b) {
    Dual<D> r = a;
    r.v = a.v + b;
    return r;
}
template <int D>
CFX_HD Dual<D> operator+(double b, const Dual<D>& a) {
    return a + b;
}
template <int D>
CFX_HD Dual<D> operator-(const Dual<D>& a, double b) {
    Dual<D> r = a;
    r.v = a.v - b;
    return r;
}
template <int D>
CFX_HD Dual<D> operator-(double a, const Dual<D>& b) {
    Dual<D> r;
    r.v = a - b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = -b.d[i];
    return r;
}
template <int D>
CFX_HD Dual<D> operator*(double s, const Dual<D>& a) {
    Dual<D> r;
    r.v = s * a.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = s * a.d[i];
    return r;
}
template <int D>
CFX_HD Dual<D> operator*(const Dual<D>& a, double s) {
    return s * a;
}
template <int D>
CFX_HD Dual<D> operator*(const Dual<D>& a, const Dual<D>& b) {
    Dual<D> r;
    r.v = a.v * b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = a.v * b.d[i] + b.v * a.d[i];
    return r;
}
// Reciprocal for the derivative parts of a quotient (the value part keeps the IEEE division): v_rcp_f64 and the
// cubic correction y (1 + e + e^2), e = 1 - x y, half the instructions of a correctly rounded 1 / x and within an ulp of
// it (cfx_kernels.h frcp).  Finite non-zero inputs.
CFX_HD double drcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rcp(x);
    const double e = fma(-x, y, 1.0);
    return fma(y, fma(e, e, e), y);
#else
    return 1.0 / x;
#endif
}
template <int D>
CFX_HD Dual<D> operator/(const Dual<D>& a, const Dual<D>& b) {
    Dual<D> r;
    r.v = a.v / b.v;
    if (D > 0) {
        const double inv = drcp(b.v);
#pragma unroll
        for (int i = 0; i < D; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) * inv;
    }
    return r;
}
template <int D>
CFX_HD Dual<D> operator/(const Dual<D>& a, double b) {
    Dual<D> r;
    r.v = a.v / b;
    if (D > 0) {
        const double inv = 1.0 / b;
#pragma unroll
        for (int i = 0; i < D; ++i) r.d[i] = a.d[i] * inv;
    }
    return r;
}
template <int D>
CFX_HD Dual<D> operator/(double a, const Dual<D>& b) {
    Dual<D> r;
    r.v = a / b.v;
    if (D > 0) {
        const double inv = drcp(b.v);
#pragma unroll
        for (int i = 0; i < D; ++i) r.d[i] = -r.v * b.d[i] * inv;
    }
    return r;
}

// ---- second-order jets -------------------------------------------------------------------------------

template <int D>
struct Jet {
    static constexpr int H = D * (D + 1) / 2;
    double v;
    double g[D > 0 ? D : 1];
    double h[H > 0 ? H : 1];
};

template <int D>
CFX_HD Jet<D> jconst(double v) {
    Jet<D> r;
    r.v = v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.g[i] = 0.0;
#pragma unroll
    for (int i = 0; i < Jet<D>::H; ++i) r.h[i] = 0.0;
    return r;
}

template <int D>
CFX_HD Jet<D> operator+(const Jet<D>& a, const Jet<D>& b) {
    Jet<D> r;
    r.v = a.v + b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.g[i] = a.g[i] + b.g[i];
#pragma unroll
    for (int i = 0; i < Jet<D>::H; ++i) r.h[i] = a.h[i] + b.h[i];
    return r;
}
template <int D>
CFX_HD Jet<D> operator-(const Jet<D>& a, const Jet<D>& b) {
    Jet<D> r;
    r.v = a.v - b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.g[i] = a.g[i] - b.g[i];
#pragma unroll
    for (int i = 0; i < Jet<D>::H; ++i) r.h[i] = a.h[i] - b.h[i];
    return r;
}
template <int D>
CFX_HD Jet<D> operator+(const Jet<D>& a, double b) {
    Jet<D> r = a;
    r.v = a.v + b;
    return r;
}
template <int D>
CFX_HD Jet<D> operator+(double b, const Jet<D>& a) {
    return a + b;
}
template <int D>
CFX_HD Jet<D> operator-(const Jet<D>& a, double b) {
    Jet<D> r = a;
    r.v = a.v - b;
    return r;
}
template <int D>
CFX_HD Jet<D> operator-(double a, const Jet<D>& b) {
    Jet<D> r;
    r.v = a - b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.g[i] = -b.g[i];
#pragma unroll
    for (int i = 0; i < Jet<D>::H; ++i) r.h[i] = -b.h[i];
    return r;
}
template <int D>
CFX_HD Jet<D> operator*(double s, const Jet<D>& a) {
    Jet<D> r;
    r.v = s * a.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.g[i] = s * a.g[i];
#pragma unroll
    for (int i = 0; i < Jet<D>::H; ++i) r.h[i] = s * a.h[i];
    return r;
}
template <int D>
CFX_HD Jet<D> operator*(const Jet<D>& a, double s) {
    return s * a;
}
template <int D>
CFX_HD Jet<D> operator*(const Jet<D>& a, const Jet<D>& b) {
    Jet<D> r;
    r.v = a.v * b.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.g[i] = a.v * b.g[i] + b.v * a.g[i];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            const int p = i * (i + 1) / 2 + j;
            r.h[p] = a.v * b.h[p] + b.v * a.h[p] + a.g[i] * b.g[j] + a.g[j] * b.g[i];
        }
    return r;
}
// phi(a) for a scalar function with value f0, first derivative f1 and second derivative f2 at a.v
template <int D>
CFX_HD Jet<D> jchain(const Jet<D>& a, double f0, double f1, double f2) {
    Jet<D> r;
    r.v = f0;
#pragma unroll
    for (int i = 0; i < D; ++i) r.g[i] = f1 * a.g[i];
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            const int p = i * (i + 1) / 2 + j;
            r.h[p] = f1 * a.h[p] + f2 * a.g[i] * a.g[j];
        }
    return r;
}
template <int D>
CFX_HD Jet<D> operator/(const Jet<D>& a, const Jet<D>& b) {
    const double inv = 1.0 / b.v;
    Jet<D> r = a * jchain(b, inv, -inv * inv, 2.0 * inv * inv * inv);
    r.v = a.v / b.v;
    return r;
}
template <int D>
CFX_HD Jet<D> operator/(const Jet<D>& a, double b) {
    Jet<D> r = a * (1.0 / b);
    r.v = a.v / b;
    return r;
}
template <int D>
CFX_HD Jet<D> operator/(double a, const Jet<D>& b) {
    const double inv = 1.0 / b.v;
    Jet<D> r = jchain(b, a * inv, -a * inv * inv, 2.0 * a * inv * inv * inv);
    r.v = a / b.v;
    return r;
}

// ---- scalar helpers so the model code is written once for double, Dual and Jet ----------------------

CFX_HD double value(double x) { return x; }
template <int D>
CFX_HD double value(const Dual<D>& x) {
    return x.v;
}
template <int D>
CFX_HD double value(const Jet<D>& x) {
    return x.v;
}

// exp / tanh of a scalar input carrying derivatives
CFX_HD double sexp(double x) { return exp(x); }
template <int D>
CFX_HD Dual<D> sexp(const Dual<D>& a) {
    Dual<D> r;
    r.v = exp(a.v);
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = r.v * a.d[i];
    return r;
}
template <int D>
CFX_HD Jet<D> sexp(const Jet<D>& a) {
    const double e = exp(a.v);
    return jchain(a, e, e, e);
}
CFX_HD double stanh(double x) { return tanh(x); }
template <int D>
CFX_HD Dual<D> stanh(const Dual<D>& a) {
    Dual<D> r;
    r.v = tanh(a.v);
    const double d1 = 1.0 - r.v * r.v;
#pragma unroll
    for (int i = 0; i < D; ++i) r.d[i] = d1 * a.d[i];
    return r;
}
template <int D>
CFX_HD Jet<D> stanh(const Jet<D>& a) {
    const double t = tanh(a.v);
    const double d1 = 1.0 - t * t;
    return jchain(a, t, d1, -2.0 * t * d1);
}

}  // namespace cfx
