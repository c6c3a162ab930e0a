// Correctly rounded float64 x**e (x >= 0) for get_action_probs' `visits ** (1 / T)` at temperatures
// outside NumPy's fast_scalar_power paths (mcts.py:672-674; the fast paths stay in k_act).
//
// Why not the device library's pow: it is within 1 ulp but not correctly rounded (it differs from the
// correctly rounded value in 14-25% of the entries k_act sees, profiles/r02w_pow.txt, and in 20% of
// test_device_pow_cr_equals_host_pow_cr's inputs, profiles/r02x_pytest_gpu.log).
// NumPy's own result is host-dependent: with AVX512 it runs a SIMD power (differs from libm in ~4% of
// entries), otherwise glibc pow (0.52-ulp bound: differs from the correctly rounded value in ~0.08%).
// The correctly rounded value is the one target every implementation approximates, so k_act computes
// it: log and exp in double-double (hi + lo, ~2^-100 relative), rounded once at the end. A result is
// misrounded only when the exact power lies within ~2^-90 relative of a rounding midpoint.
//
// log x = k ln2 + 2 atanh(s), s = (m - 1) / (m + 1), m in [sqrt(1/2), sqrt(2)) (|s| <= 0.1716);
// exp t = 2^n (1 + expm1(r)), r = t - n ln2 scaled by 2^-8, expm1 by its Taylor series, then eight
// doublings expm1(2r) = 2 expm1(r) + expm1(r)^2 (keeps the relative accuracy of expm1).
// Host and device share the code (tools/alt exports both, tests compare them bitwise and the host
// form against 60-digit decimal arithmetic). Build with -ffp-contract=off (the error-free
// transformations below rely on separately rounded products and sums).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace rvz_pow {

struct dd {
    double hi, lo;
};

__host__ __device__ inline dd two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline dd quick_sum(double a, double b) {  // |a| >= |b|
    const double s = a + b;
    return {s, b - (s - a)};
}
__host__ __device__ inline dd two_prod(double a, double b) {
    const double p = a * b;
    return {p, fma(a, b, -p)};
}
__host__ __device__ inline dd neg(dd a) { return {-a.hi, -a.lo}; }
__host__ __device__ inline dd add(dd a, dd b) {
    dd s = two_sum(a.hi, b.hi);
    const dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = quick_sum(s.hi, s.lo);
    s.lo += t.lo;
    return quick_sum(s.hi, s.lo);
}
__host__ __device__ inline dd mul(dd a, dd b) {
    dd p = two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return quick_sum(p.hi, p.lo);
}
__host__ __device__ inline dd mul_d(dd a, double b) {
    dd p = two_prod(a.hi, b);
    p.lo += a.lo * b;
    return quick_sum(p.hi, p.lo);
}
__host__ __device__ inline dd div_d(dd a, double b) {
    const double q1 = a.hi / b;
    const dd p = two_prod(q1, b);
    const double r = ((a.hi - p.hi) - p.lo) + a.lo;
    return quick_sum(q1, r / b);
}
__host__ __device__ inline dd div(dd a, dd b) {
    const double q1 = a.hi / b.hi;
    dd r = add(a, neg(mul_d(b, q1)));
    const double q2 = r.hi / b.hi;
    r = add(r, neg(mul_d(b, q2)));
    const double q3 = r.hi / b.hi;
    return add(quick_sum(q1, q2), dd{q3, 0.0});
}

constexpr double LN2_HI = 0x1.62e42fefa39efp-1, LN2_LO = 0x1.abc9e3b39803fp-56;
constexpr double INV_LN2 = 0x1.71547652b82fep+0;

// ln x for finite x > 0
__host__ __device__ inline dd log_dd(double x) {
    int k;
    double m = frexp(x, &k);  // x = m 2^k, m in [0.5, 1)
    if (m < 0x1.6a09e667f3bcdp-1) {
        m *= 2.0;
        --k;
    }
    const dd s = div(dd{m - 1.0, 0.0}, two_sum(m, 1.0));  // m - 1 is exact
    const dd z = mul(s, s);                                // <= 0.02944
    // atanh(s) / s = sum_j z^j / (2j + 1): j = 8..19 in double (< 2^-44 of the sum), 7..0 in dd
    double tail = 1.0 / 39.0;
    for (int j = 18; j >= 8; --j) tail = 1.0 / (2 * j + 1) + z.hi * tail;
    dd acc = {tail, 0.0};
    for (int j = 7; j >= 0; --j) acc = add(div_d(dd{1.0, 0.0}, 2.0 * j + 1.0), mul(z, acc));
    const dd lm = mul_d(mul(s, acc), 2.0);
    return add(mul_d(dd{LN2_HI, LN2_LO}, (double)k), lm);
}

// e^t rounded to double; t finite
__host__ __device__ inline double exp_dd(dd t) {
    if (t.hi < -746.0) return 0.0;
    if (t.hi > 710.0) return INFINITY;
    const double n = rint(t.hi * INV_LN2);
    dd r = add(t, neg(mul_d(dd{LN2_HI, LN2_LO}, n)));  // |r| <= ~0.347
    r.hi = ldexp(r.hi, -8);
    r.lo = ldexp(r.lo, -8);
    dd a = {1.0, 0.0};  // expm1(r) = r (1 + r/2 (1 + r/3 (1 + ...)))
    for (int k = 11; k >= 2; --k) a = add(dd{1.0, 0.0}, mul(div_d(r, (double)k), a));
    a = mul(r, a);
    for (int i = 0; i < 8; ++i) a = add(mul_d(a, 2.0), mul(a, a));
    const dd y = add(dd{1.0, 0.0}, a);
    const int ni = (int)n;
    if (ni >= -1021) return ldexp(y.hi, ni);
    // subnormal range: round (hi + lo) 2^n once, on the 2^-1074 grid (ldexp of hi alone would round
    // twice); n >= -1077 here, so both scalings are exact
    const double sh = ldexp(y.hi, ni + 1074), sl = ldexp(y.lo, ni + 1074);
    double q = rint(sh);
    const double fr = sh - q;  // exact, in [-0.5, 0.5]; |fr| < 0.5 cannot cross with sl
    if (fr == 0.5 && sl > 0.0) q += 1.0;
    if (fr == -0.5 && sl < 0.0) q -= 1.0;
    return ldexp(q, -1074);
}

// x ** e, x >= 0 (NumPy semantics for the cases k_act can meet; NaN for x < 0)
__host__ __device__ inline double pow_cr(double x, double e) {
    if (e == 0.0 || x == 1.0) return 1.0;
    if (x == 0.0) return e > 0.0 ? 0.0 : INFINITY;
    if (!(x > 0.0) || isnan(e)) return NAN;
    if (isinf(x)) return e > 0.0 ? INFINITY : 0.0;
    if (isinf(e)) return (x < 1.0) == (e > 0.0) ? 0.0 : INFINITY;
    const dd l = log_dd(x);
    return exp_dd(mul_d(l, e));
}

}  // namespace rvz_pow
