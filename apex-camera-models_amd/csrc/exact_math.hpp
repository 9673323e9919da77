// exact_math.hpp -- correctly rounded atan2 for the reference-exact ("exact
// math") projections of Kannala-Brandt and FOV.
//
// The reference calls f64::atan2 (glibc's atan2 on x86_64-linux-gnu, the libm
// Rust std links).  The default kernels use a degree-20 polynomial within
// ~2 ulp of it (camera_models.hpp atan2_ge0), held to 1e-10 like the rest of
// the KB / FOV path.  Callers whose outputs are quantised by round() / floor()
// (undistort_image, undistort.rs:61,70,100) or that ask for reference-exact
// values (acm_project with ACM_EXACT_MATH) use atan2_cr below instead: atan2
// evaluated in double-double arithmetic (~2^-100 relative) and rounded once,
// i.e. the correctly rounded result except with probability ~2^-45 per
// argument.  glibc 2.35's atan2 is itself correctly rounded on all but about
// 0.2% of arguments (its slow multi-precision paths were removed; max error
// < 1 ulp): there it and atan2_cr differ by one ulp, and atan2_cr is the
// correctly rounded one (tests/test_exact_math.py, tests/test_gpu_exact.py
// check both claims against 300-bit mpmath).
//
// Method: q = min(y,x) / max(y,x) in [0, 1] as a double-double (quotient +
// exact FMA remainder); c = k/64 nearest to q; atan(q) = atan(c) + atan(t),
// t = (q - c) / (1 + q c), |t| <= 1/128, atan(t) = t * sum_{n<8} (-1)^n
// t^{2n} / (2n+1) (truncation < 2^-112); pi/2 - atan(q) when y > x.  The
// constants are double-double values from tools/gen_exact_tables.py (mpmath,
// 300 bits).  Every function is __host__ __device__, so the same code is
// unit-tested on the host (ACM_HD defined empty for a plain C++ build).
#pragma once

#include <math.h>

#ifndef ACM_HD
#define ACM_HD __host__ __device__
#endif

namespace acm {
namespace xm {

struct dd { double hi, lo; };

// Error-free transformations (Knuth two-sum, FMA two-product); the file is
// compiled with -ffp-contract=off, so nothing below is re-associated or fused.
ACM_HD inline dd two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
ACM_HD inline dd quick_two_sum(double a, double b) {  // |a| >= |b|
    const double s = a + b;
    return {s, b - (s - a)};
}
ACM_HD inline dd two_prod(double a, double b) {
    const double p = a * b;
    return {p, fma(a, b, -p)};
}
ACM_HD inline dd dd_add(dd a, dd b) {
    dd s = two_sum(a.hi, b.hi);
    const dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return quick_two_sum(s.hi, s.lo);
}
ACM_HD inline dd dd_neg(dd a) { return {-a.hi, -a.lo}; }
ACM_HD inline dd dd_mul(dd a, dd b) {
    dd p = two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return quick_two_sum(p.hi, p.lo);
}
ACM_HD inline dd dd_mul_d(dd a, double b) {
    dd p = two_prod(a.hi, b);
    p.lo += a.lo * b;
    return quick_two_sum(p.hi, p.lo);
}
ACM_HD inline dd dd_div(dd a, dd b) {  // long division, three quotient digits
    const double q1 = a.hi / b.hi;
    dd r = dd_add(a, dd_neg(dd_mul_d(b, q1)));
    const double q2 = r.hi / b.hi;
    r = dd_add(r, dd_neg(dd_mul_d(b, q2)));
    const double q3 = r.hi / b.hi;
    return dd_add(quick_two_sum(q1, q2), dd{q3, 0.0});
}

// atan(k / 64), k = 0..64 (tools/gen_exact_tables.py)
constexpr double kAtanK64[65][2] = {
    {0x0.0p+0, 0x0.0p+0}, {0x1.fff555bbb729bp-7, -0x1.220c39d4dff50p-61},
    {0x1.ffd55bba97625p-6, -0x1.5ec431444912cp-60}, {0x1.7fb818430da2ap-5, -0x1.86ef8f794f105p-63},
    {0x1.ff55bb72cfdeap-5, -0x1.c934d86d23f1dp-60}, {0x1.3f59f0e7c559dp-4, 0x1.ac4ce285df847p-58},
    {0x1.7ee182602f10fp-4, -0x1.cfb654c0c3d98p-58}, {0x1.be39ebe6f07c3p-4, 0x1.f7b8f29a05987p-58},
    {0x1.fd5ba9aac2f6ep-4, -0x1.cd37686760c17p-59}, {0x1.1e1fafb043727p-3, -0x1.b485914dacf8cp-59},
    {0x1.3d6eee8c6626cp-3, 0x1.61a3b0ce9281bp-57}, {0x1.5c9811e3ec26ap-3, -0x1.054ab2c010f3dp-58},
    {0x1.7b97b4bce5b02p-3, 0x1.347b0b4f881cap-58}, {0x1.9a6a8e96c8626p-3, 0x1.cf601e7b4348ep-59},
    {0x1.b90d7529260a2p-3, 0x1.17b10d2e0e5abp-61}, {0x1.d77d5df205736p-3, 0x1.c648d1534597ep-57},
    {0x1.f5b75f92c80ddp-3, 0x1.8ab6e3cf7afbdp-57}, {0x1.09dc597d86362p-2, 0x1.62e47390cb865p-56},
    {0x1.18bf5a30bf178p-2, 0x1.30ca4748b1bf9p-57}, {0x1.278372057ef46p-2, -0x1.077cdd36dfc81p-56},
    {0x1.362773707ebccp-2, -0x1.963a544b672d8p-57}, {0x1.44aa436c2af0ap-2, -0x1.5d5e43c55b3bap-56},
    {0x1.530ad9951cd4ap-2, -0x1.2566480884082p-57}, {0x1.614840309cfe2p-2, -0x1.a725715711f00p-56},
    {0x1.6f61941e4def1p-2, -0x1.c63aae6f6e918p-56}, {0x1.7d5604b63b3f7p-2, 0x1.69c885c2b249ap-56},
    {0x1.8b24d394a1b25p-2, 0x1.b6d0ba3748fa8p-56}, {0x1.98cd5454d6b18p-2, 0x1.9e6c988fd0a77p-56},
    {0x1.a64eec3cc23fdp-2, -0x1.24dec1b50b7ffp-56}, {0x1.b3a911da65c6cp-2, 0x1.ae187b1ca5040p-56},
    {0x1.c0db4c94ec9f0p-2, -0x1.cc1ce70934c34p-56}, {0x1.cde53432c1351p-2, -0x1.a2cfa4418f1adp-56},
    {0x1.dac670561bb4fp-2, 0x1.a2b7f222f65e2p-56}, {0x1.e77eb7f175a34p-2, 0x1.0e53dc1bf3435p-56},
    {0x1.f40dd0b541418p-2, -0x1.a3992dc382a23p-57}, {0x1.0039c73c1a40cp-1, -0x1.b32c949c9d593p-55},
    {0x1.0657e94db30d0p-1, -0x1.d5b495f6349e6p-56}, {0x1.0c6145b5b43dap-1, 0x1.974fa13b5404fp-58},
    {0x1.1255d9bfbd2a9p-1, -0x1.2bdaee1c0ee35p-58}, {0x1.1835a88be7c13p-1, 0x1.c621cec00c301p-55},
    {0x1.1e00babdefeb4p-1, -0x1.928df287a668fp-58}, {0x1.23b71e2cc9e6ap-1, 0x1.c421c9f38224ep-57},
    {0x1.2958e59308e31p-1, -0x1.09e73b0c6c087p-56}, {0x1.2ee628406cbcap-1, 0x1.c5d5e9ff0cf8dp-55},
    {0x1.345f01cce37bbp-1, 0x1.1021137c71102p-55}, {0x1.39c391cd4171ap-1, -0x1.2304331d8bf46p-55},
    {0x1.3f13fb89e96f4p-1, 0x1.ecf8b492644f0p-56}, {0x1.445065b795b56p-1, -0x1.f76d0163f79c8p-56},
    {0x1.4978fa3269ee1p-1, 0x1.2419a87f2a458p-56}, {0x1.4e8de5bb6ec04p-1, 0x1.4a33dbeb3796cp-55},
    {0x1.538f57b89061fp-1, -0x1.1bb74abda520cp-55}, {0x1.587d81f732fbbp-1, -0x1.5e5c9d8c5a950p-56},
    {0x1.5d58987169b18p-1, 0x1.0028e4bc5e7cap-57}, {0x1.6220d115d7b8ep-1, -0x1.2b785350ee8c1p-57},
    {0x1.66d663923e087p-1, -0x1.6ea6febe8bbbap-56}, {0x1.6b798920b3d99p-1, -0x1.a80386188c50ep-55},
    {0x1.700a7c5784634p-1, -0x1.8c34d25aadef6p-56}, {0x1.748978fba8e0fp-1, 0x1.7b2a6165884a1p-59},
    {0x1.78f6bbd5d315ep-1, 0x1.406a089803740p-55}, {0x1.7d528289fa093p-1, 0x1.560821e2f3aa9p-55},
    {0x1.819d0b7158a4dp-1, -0x1.bf76229d3b917p-56}, {0x1.85d69576cc2c5p-1, 0x1.6b66e7fc8b8c3p-57},
    {0x1.89ff5ff57f1f8p-1, -0x1.55b9a5e177a1bp-55}, {0x1.8e17aa99cc05ep-1, -0x1.ec182ab042f61p-56},
    {0x1.921fb54442d18p-1, 0x1.1a62633145c07p-55},
};
// (-1)^n / (2n + 1), n = 0..7
constexpr double kAtanSeries[8][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.5555555555555p-2, -0x1.5555555555555p-56},
    {0x1.999999999999ap-3, -0x1.999999999999ap-57},
    {-0x1.2492492492492p-3, -0x1.2492492492492p-57},
    {0x1.c71c71c71c71cp-4, 0x1.c71c71c71c71cp-58},
    {-0x1.745d1745d1746p-4, 0x1.745d1745d1746p-59},
    {0x1.3b13b13b13b14p-4, -0x1.3b13b13b13b14p-58},
    {-0x1.1111111111111p-4, -0x1.1111111111111p-60},
};
constexpr double kPiHalfHi = 0x1.921fb54442d18p+0, kPiHalfLo = 0x1.1a62633145c07p-54;

// atan(q) for a double-double q in [0, 1]
ACM_HD inline dd atan_dd01(dd q) {
    const int k = (int)(q.hi * 64.0 + 0.5);
    const double c = (double)k * 0.015625;  // exact
    // q - c: q.hi - c is exact (Sterbenz, or c = 0)
    const dd num = dd_add(dd{q.hi - c, 0.0}, dd{q.lo, 0.0});
    const dd den = dd_add(dd{1.0, 0.0}, dd_mul_d(q, c));
    const dd t = dd_div(num, den);
    const dd u = dd_mul(t, t);
    dd p = {kAtanSeries[7][0], kAtanSeries[7][1]};
    for (int n = 6; n >= 0; --n) p = dd_add(dd_mul(p, u), dd{kAtanSeries[n][0], kAtanSeries[n][1]});
    return dd_add(dd{kAtanK64[k][0], kAtanK64[k][1]}, dd_mul(p, t));
}

// atan2(y, x) for y >= 0, x > 0, both finite (every valid KB / FOV
// projection: y is a radius, x = z >= EPS): correctly rounded except with
// probability ~2^-45.  Any other argument returns NaN; callers route those
// to the library atan2 (they only arise on points whose status is an error).
ACM_HD inline double atan2_cr(double y, double x) {
    if (!(y >= 0.0 && x > 0.0 && y <= 1.79769313486231570815e308 && x <= 1.79769313486231570815e308))
        return NAN;
    if (y == 0.0) return 0.0;  // atan2(+0, x > 0) = +0
    const bool swap = y > x;
    double a = swap ? x : y, b = swap ? y : x;  // 0 < a <= b
    // atan2 is scale invariant: bring b into [2^-400, 2^1000] (exact power-of-
    // two scaling; an a that underflows is negligible against b anyway)
    if (b < 0x1p-400) { a *= 0x1p600; b *= 0x1p600; }
    if (b > 0x1p1000) { a *= 0x1p-600; b *= 0x1p-600; }
    const double qh = a / b;
    dd q;
    if (qh >= 0x1p-450) {
        // a >= 2^-850: the remainder a - qh*b is exact, then the second digit
        q = quick_two_sum(qh, fma(-qh, b, a) / b);
    } else {
        q = {qh, 0.0};  // atan(q) = q (1 - q^2/3 ...) rounds to RN(q) here
    }
    const dd at = atan_dd01(q);
    if (!swap) return at.hi;
    return dd_add(dd{kPiHalfHi, kPiHalfLo}, dd_neg(at)).hi;
}

}  // namespace xm
}  // namespace acm
