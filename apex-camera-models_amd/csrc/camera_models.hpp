// camera_models.hpp -- per-point device math of the seven camera models.
//
// Each model is a struct of __device__ functions templated on the scalar T
// (double for the parity path, float for the f32 tolerance sweep).  The
// arithmetic follows the reference Rust code expression by expression (Rust
// evaluates `a + b + c` as (a + b) + c and never contracts to FMA; this file
// is compiled with -ffp-contract=off so hipcc does not either), which is what
// makes the validity masks bit-exact: every threshold test sees the same
// doubles as the reference.
//
// Where the double path is NOT the reference's correctly rounded operation
// sequence (every other division and square root is the IEEE sequence hipcc
// emits by default, no -ffast-math):
//   * KB project: atan2 is the polynomial atan2_ge0 (<= ~2 ulp from glibc),
//     and r = sqrt(x^2+y^2), 1/r and the atan2 quotient come from
//     v_rsq_f64 / v_rcp_f64 + two Newton steps (~1 ulp; rsq_nr, rcp_nr) for
//     r^2, z in [2^-1000, 2^1000] (the IEEE forms outside; ACM_IEEE_MATH
//     builds the IEEE forms everywhere).  The axis test r < EPS stays exact:
//     it is r^2 < 2^-104 (kAxisR2).
//   * KB unproject: sin / cos of the Newton angle are polynomials on [0, 2]
//     (sincos_0_2, OCML beyond), and after the Newton loop 1/ru and 1/|p|
//     come from rcp_nr / rsq_nr (the IEEE forms outside [2^-1000, 2^1000]).
//   * KB and RadTan unproject: the Newton loops are the certified fast ones
//     (KannalaBrandt::newton_fast / front_fast, RadTan::newton_fast): FMA
//     and reciprocal iterates (ru from rsq for KB, 1/|p| from rsq for
//     RadTan) that make every break / continue / failure decision of the
//     reference's loop, certified per step against an error bound; any
//     pixel that cannot be certified runs the reference's loop from the
//     start.  Statuses are the reference's; rays within a few ulp.
//     ACM_REFERENCE_NEWTON (per call) runs the reference's loops for every pixel
//     (RadTan's rays are then the reference's bit for bit).
//   * FOV project: atan2 is atan2_ge0; FOV unproject: sincos_0_2 and
//     rsq / rcp + Newton for 1 / rd, 1 / cos and 1 / |p| (its one decision,
//     rd > sqrt(EPS), taken exactly on r2).
//   * project<.., FAST = true> (the fused normal equations only): one
//     reciprocal and products instead of the per-point divisions.
// None of these feeds a status decision, so statuses are bit-exact
// everywhere; values are held to 1e-10 relative (tests/test_gpu_parity.py,
// observed ~1e-15).  project<.., EXACT = true> (acm_project with
// ACM_EXACT_MATH, and undistort_image, whose bytes round() / floor() the
// source coordinates) takes the IEEE sqrt / divisions and the correctly
// rounded double-double atan2 of exact_math.hpp: KB and FOV projections and
// Jacobians then equal the reference bit for bit wherever glibc's atan2 is
// correctly rounded (all but ~0.2% of arguments; there they differ by one
// ulp and ours is the correctly rounded one).  tests/test_gpu_exact.py pins
// the EXACT path to the oracle and the fast path to the EXACT one.
// Several divisions by one divisor go through div_shared, bit-identical to
// dividing each.
//
// Status decisions are computed branch-free where possible so a wave does
// not diverge on the rare failing point; the caller selects outputs.
//
// project<WJ, FAST>: FAST = true (used only by the fused normal-equations
// kernel, whose sums are held to 1e-10 anyway and are summed in a different
// order than the reference) replaces the divisions by a per-point denominator
// with one reciprocal and multiplies: u, v, J within ~1 ulp of the exact
// path.  Status decisions never depend on those divisions, so the validity
// mask (and n_valid) stays bit-exact.  Every other caller uses FAST = false,
// the reference's operation order.
//
// Reference citations: /root/reference/src/camera/<model>.rs:line.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "exact_math.hpp"

namespace acm {

enum : uint8_t {
    ST_OK = 0,
    ST_PROJECTION_OUT_SIDE_IMAGE = 1,
    ST_POINT_IS_OUT_SIDE_IMAGE = 2,
    ST_POINT_AT_CAMERA_CENTER = 3,
    ST_NUMERICAL_ERROR = 4,
};

constexpr double kEps = 2.220446049250313e-16;      // f64::EPSILON
constexpr double kEpsSqrt = 1.4901161193847656e-08;  // f64::EPSILON.sqrt()
constexpr double kPi = 3.141592653589793;
// Smallest double s with sqrt(s) >= 1e-6 under correctly rounded sqrt, so
// `sqrt(s) < 1e-6` == `s < kNewtonTol2` for every s >= 0 (and both are false
// for NaN).  Lets the RadTan Newton loop drop two sqrt per step with the
// reference's decisions unchanged bit for bit (tests/test_capi.py pins it).
constexpr double kNewtonTol2 = 0x1.19799812dea10p-40;
// The same for KB's axis test `r < EPS` with r = sqrt(r2) (kannala_brandt.rs
// :375): 2^-104 = EPS^2 is the smallest double whose correctly rounded sqrt
// is >= EPS, so `sqrt(r2) < EPS` == `r2 < 2^-104` for every r2 >= 0 and NaN
// -- no sqrt (the compiler had been computing one for every point).
constexpr double kAxisR2 = 0x1p-104;

// atan(b) for 0 <= b <= 1: b * P(b^2), P the degree-20 Chebyshev
// interpolant of atan(sqrt(s))/sqrt(s) on s in [0, 1] (60-digit mpmath fit,
// tools/fit_atan.py), evaluated as two interleaved Horner chains in s^2 so
// the dependent FMA depth is 11, not 21.  Max relative error 4.5e-16 against
// glibc atan over 2e8 arguments (tools/fit_atan.py --check).
__constant__ double kAtanE[11] = {  // even-index coefficients c0, c2, ..., c20
        0x1.0000000000000p+0, 0x1.9999999993702p-3, 0x1.c71c716e724e1p-4,
        0x1.3b135af6a0e88p-4, 0x1.e1b7b5bcacd55p-5, 0x1.82a3c93dd0230p-5,
        0x1.2b18b9c197546p-5, 0x1.643110da5054fp-6, 0x1.cd48e33ffd1aep-8,
        0x1.a53135c884a6dp-11, 0x1.a7d4ff1d17f2cp-17};
__constant__ double kAtanO[10] = {  // odd-index coefficients c1, c3, ..., c19
        -0x1.5555555555500p-2, -0x1.2492492327bf2p-3, -0x1.745d1099f743ep-4,
        -0x1.110df7e57b3d8p-4, -0x1.ae4da39abd8c9p-5, -0x1.59180bd7d7b67p-5,
        -0x1.e69dd6d612131p-6, -0x1.c012fe85b6413p-7, -0x1.6fa050a5cad37p-9,
        -0x1.328ae5000addbp-13};
// (coefficients in constant memory: uniform s_loads into SGPRs, used as FMA
// operands -- as literals they were materialised in 42 VGPRs, which held the
// grid kernel at 3 waves/SIMD)
//
// coef_at_use (r05): the table's address passes through an empty asm with
// an SGPR operand at every evaluation, so the s_loads of its coefficients
// are issued there and cannot be hoisted to the kernel entry or merged with
// another evaluation's.  Hoisted, the 21 atan and 22 sin / cos coefficients
// stayed live in SGPRs across the whole kernel beside the camera's
// constants, overflowed the 102 SGPRs and were spilled to VGPR lanes: every
// evaluation then re-read them with ~20-45 v_readlane (VALU) instructions
// (k_round_trip<KB>: 256 v_readlane + 80 v_writelane in the code, ~100 VALU
// instructions of its ~400 per point).  Same coefficients, same operation
// order: the results are bit-identical.
// fma_sc: fma(a, b, c) with the coefficient c read straight from its SGPRs
// (v_fma_f64 takes one scalar operand).  Left to itself the compiler picked
// the two-operand v_fmac_f64 and first copied every coefficient into a VGPR
// pair (two v_mov_b32 per Horner step).  The same single rounding as fma().
typedef __attribute__((address_space(4))) const double coef_t;
// (Unoptimised device builds -- the host-sanitizer tests compile the device
// side at -O0 -- cannot place these operands in SGPRs: plain forms there.)
__device__ __forceinline__ coef_t* coef_at_use(const double* table) {
    coef_t* p = (coef_t*)table;
#ifdef __OPTIMIZE__
    asm volatile("" : "+s"(p));
#endif
    return p;
}
__device__ __forceinline__ double fma_sc(double a, double b, double c) {
#ifdef __OPTIMIZE__
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
#else
    return fma(a, b, c);
#endif
}

__device__ __forceinline__ double atan01(double b) {
    coef_t* E = coef_at_use(kAtanE);
    coef_t* O = coef_at_use(kAtanO);
    const double s = b * b, s2 = s * s;
    double pe = E[10], po = O[9];
#pragma unroll
    for (int k = 9; k >= 0; --k) pe = fma_sc(pe, s2, E[k]);
#pragma unroll
    for (int k = 8; k >= 0; --k) po = fma_sc(po, s2, O[k]);
    return b * fma(po, s, pe);
}

// atan2(y, x) for y >= +0 (every use here: y is a radius) in double: one
// IEEE division min(y,|x|)/max(y,|x|) in [0, 1] and the polynomial above
// (pi/2 - atan(|x|/y) when y > |x|, mirrored through pi for x < 0); the
// special values (zeros, infinities, NaN) as C's atan2 defines them.
// Within 4.5e-16 relative of glibc's atan2 like OCML's own (tests hold
// KB / FOV to 1e-10), with fewer instructions -- and no OCML atan2 in the
// kernel at all: its 19 coefficients, live only on the rare path, were
// hoisted into 38 VGPRs across every grid-stride loop that inlined it.
__device__ __forceinline__ double atan2_ge0(double y, double x) {
    constexpr double kPiD = 3.141592653589793, kPiO2 = 1.5707963267948966;
    if (x > 0.0 && x < INFINITY && y < INFINITY) {
        const bool swap = y > x;
        const double q = swap ? x / y : y / x;
        const double at = atan01(q);
        return swap ? kPiO2 - at : at;
    }
    if (x != x || y != y) return x + y;
    if (y == INFINITY)
        return x == INFINITY ? 0.7853981633974483 : (x == -INFINITY ? 2.356194490192345 : kPiO2);
    if (x == INFINITY) return 0.0;   // y finite
    if (x == -INFINITY) return kPiD;
    if (x == 0.0) return y > 0.0 ? kPiO2 : (signbit(x) ? kPiD : 0.0);
    const double ax = -x;  // x < 0 finite, y finite
    const bool swap = y > ax;
    const double q = swap ? ax / y : y / ax;
    const double at = atan01(q);
    return swap ? kPiO2 + at : kPiD - at;
}
__device__ __forceinline__ float atan2_ge0(float y, float x) { return atan2(y, x); }

// The reference-exact atan2 (EXACT projections): the double-double,
// correctly rounded atan2_cr of exact_math.hpp where it is defined (y >= 0,
// x > 0, finite: every point whose status is Ok), OCML's atan2 elsewhere.
__device__ __forceinline__ double atan2_exact(double y, double x) {
    const double t = xm::atan2_cr(y, x);
    return t == t ? t : atan2(y, x);
}
__device__ __forceinline__ float atan2_exact(float y, float x) { return atan2(y, x); }

// 1/sqrt(a) and 1/a from the hardware estimates (v_rsq_f64 / v_rcp_f64)
// with two Newton-Raphson steps each: within ~1 ulp for a in
// [2^-1000, 2^1000] (callers check the range and take the IEEE forms
// outside it).  Used only where the model already differs from the
// reference in the last bits (KB's atan2 is a polynomial) and no status
// decision depends on the value.
__device__ __forceinline__ double rsq_nr(double a) {
    double y = __builtin_amdgcn_rsq(a);
    const double h = 0.5 * a;
    double e = fma(-h * y, y, 0.5);
    y = fma(y, e, y);
    e = fma(-h * y, y, 0.5);
    return fma(y, e, y);
}
__device__ __forceinline__ double rcp_nr(double a) {
    double y = __builtin_amdgcn_rcp(a);
    double e = fma(-a, y, 1.0);
    y = fma(y, e, y);
    e = fma(-a, y, 1.0);
    return fma(y, e, y);
}
__device__ __forceinline__ bool nr_range(double a) {
    return a >= 0x1p-1000 && a <= 0x1p1000;
}

// (r06) sqrt(a) correctly rounded, bit for bit the compiler's f64 sqrt: its
// expansion is v_rsq_f64 and the two Goldschmidt / Newton corrections below,
// wrapped in a rescaling of inputs under 2^-767 and a fixup for 0 and inf
// (10 of its ~20 VALU instructions).  Here the same ten-instruction core runs
// for a in [2^-767, DBL_MAX] and the full sqrt() for the rest (0, the
// rescaled range, inf, NaN, negative), laid out as a cold branch that a wave
// skips when none of its lanes needs it (computed unconditionally and
// selected, as the compiler does without the expectation, both paths cost
// more than the one sqrt).  Same operations in the same order on the range
// where the compiler's version does not rescale, so the same bits.
template <class T>
__device__ __forceinline__ T sqrt_rn(T a) {
    if constexpr (sizeof(T) == 8) {
        if (__builtin_expect(a >= 0x1p-767 && a <= 0x1.fffffffffffffp1023, 1)) {
            const double y = __builtin_amdgcn_rsq(a);
            double g = a * y;
            double h = y * 0.5;
            const double r = fma(-h, g, 0.5);
            g = fma(g, r, g);
            h = fma(h, r, h);
            double d = fma(-g, g, a);
            g = fma(d, h, g);
            d = fma(-g, g, a);
            return fma(d, h, g);
        }
        return sqrt(a);
    } else {
        return sqrt(a);
    }
}

// sin and cos of theta in [0, 2] (KB's unprojection angle, at most ~pi/2):
// theta * S(theta^2) and C(theta^2), S and C the degree-10 Chebyshev
// interpolants of sin(sqrt(s))/sqrt(s) and cos(sqrt(s)) on s in [0, 4]
// (60-digit mpmath fit, tools/fit_atan.py --sincos): max relative error of
// sin 3.6e-16, max absolute error of cos 3.3e-16.  Outside [0, 2] (or NaN)
// OCML's sincos.  Coefficients in constant memory (SGPR operands).
__constant__ double kSinS[11] = {
    0x1.0000000000000p+0, -0x1.5555555555555p-3, 0x1.1111111111111p-7,
    -0x1.a01a01a01a014p-13, 0x1.71de3a556c3f4p-19, -0x1.ae64567f35f76p-26,
    0x1.6124612f7c108p-33, -0x1.ae7f394959b00p-41, 0x1.952ae9a768f94p-49,
    -0x1.2eff6f253dc73p-57, 0x1.61fa5d5d95885p-66};
__constant__ double kCosC[11] = {
    0x1.0000000000000p+0, -0x1.0000000000000p-1, 0x1.5555555555555p-5,
    -0x1.6c16c16c16c04p-10, 0x1.a01a01a0196cap-16, -0x1.27e4fb775e7b3p-22,
    0x1.1eed8eefba3c1p-29, -0x1.939743254b313p-37, 0x1.ae7d04cacc91dp-45,
    -0x1.67bd0466d94d5p-53, 0x1.ceab379e35c76p-62};
__device__ __forceinline__ void sincos_0_2(double t, double* sn, double* cs) {
    if (t >= 0.0 && t <= 2.0) {
        const double s = t * t;
        coef_t* S = coef_at_use(kSinS);
        coef_t* C = coef_at_use(kCosC);
        double ps = S[10], pc = C[10];
#pragma unroll
        for (int k = 9; k >= 0; --k) {
            ps = fma_sc(ps, s, S[k]);
            pc = fma_sc(pc, s, C[k]);
        }
        *sn = t * ps;
        *cs = pc;
        return;
    }
    sincos(t, sn, cs);
}
__device__ __forceinline__ void sincos_0_2(float t, float* sn, float* cs) { sincosf(t, sn, cs); }
// The same polynomials without the OCML fallback, for a caller that knows
// t is in [0, 2] (KannalaBrandt::ray_certified: theta in [0, pi/2)).
__device__ __forceinline__ void sincos_poly_0_2(double t, double* sn, double* cs) {
    const double s = t * t;
    coef_t* S = coef_at_use(kSinS);
    coef_t* C = coef_at_use(kCosC);
    double ps = S[10], pc = C[10];
#pragma unroll
    for (int k = 9; k >= 0; --k) {
        ps = fma_sc(ps, s, S[k]);
        pc = fma_sc(pc, s, C[k]);
    }
    *sn = t * ps;
    *cs = pc;
}

// ------------------------------------------- division by a shared divisor
// RN(a / b) from y = RN(1 / b) (one IEEE division) and two FMAs: q = RN(a*y)
// is within one ulp of a/b, so r = a - b*q is exact, and RN(q + r*y) =
// RN(a/b) (Markstein's correction; Muller et al., Handbook of Floating-Point
// Arithmetic, Thm 4.11 -- a/b of two binary64 numbers is never a midpoint,
// so there is no tie to get wrong).  Valid while nothing over/underflows:
// every operand must lie in [2^-500, 2^500] in magnitude (zero, NaN, inf and
// extreme values take the plain IEEE division instead).  Bit-identical to
// dividing each numerator -- checked on 1.8e9 random and adversarial pairs
// (all-ones significands, quotients near 1, short significands) against
// x86 IEEE division -- so the models keep the reference's exact results
// while K divisions by one divisor cost one division plus 3K FMA-class ops.
template <class T>
__device__ __forceinline__ bool div_safe(T x) {
    const T ax = fabs(x);
    return ax >= T(0x1p-500) && ax <= T(0x1p500);
}

template <class T>
__device__ __forceinline__ T div_rn(T a, T y, T b) {
    const T q = a * y;
    const T r = fma(-b, q, a);
    return fma(r, y, q);
}

// q[k] = a[k] / b (correctly rounded); returns 1 / b (correctly rounded)
template <class T, int K>
__device__ __forceinline__ T div_shared(const T (&a)[K], T b, T (&q)[K]) {
    const T y = T(1) / b;
    if constexpr (sizeof(T) == 8) {
        bool ok = div_safe(b);
#pragma unroll
        for (int k = 0; k < K; ++k) ok = ok && div_safe(a[k]);
        if (ok) {
#pragma unroll
            for (int k = 0; k < K; ++k) q[k] = div_rn(a[k], y, b);
            return y;
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) q[k] = a[k] / b;
    return y;
}

// a / b given y = RN(1 / b) from an earlier div_shared by the same b: the
// same correctly rounded quotient, or the IEEE division outside the range
template <class T>
__device__ __forceinline__ T div_by_y(T a, T b, T y) {
    if constexpr (sizeof(T) == 8) {
        if (div_safe(a) && div_safe(b)) return div_rn(a, y, b);
    }
    return a / b;
}

// (r06) the projections' two divisions by one divisor
// (x / z, y / z; x / denom, y / denom) as one IEEE reciprocal and two
// Markstein corrections: RN(x / b), RN(y / b) bit for bit (div_shared).
// One v_rcp_f64 and division sequence fewer per point, but the operands'
// range tests cost about what that saves: RadTan's round trip measured
// even (0.628 vs 0.632 ms at 50M, profiles/r06e_ab.log); the +J forms
// share the reciprocal with their two further divisions (div_by_y).
template <class T>
__device__ __forceinline__ T div2(T x, T y, T b, T& qx, T& qy) {
    const T a[2] = {x, y};
    T q[2];
    const T r = div_shared(a, b, q);
    qx = q[0];
    qy = q[1];
    return r;
}

template <class T>
__device__ __forceinline__ bool norm_below_1e6(T sq) {
    if constexpr (sizeof(T) == 8) return sq < T(kNewtonTol2);
    else return sqrt(sq) < T(1e-6);
}

// Coefficients of each of KB's certified-ray polynomials (degree 16 in r2)
constexpr int kRayPolyN = 17;
// One Horner step's coefficients of both ray polynomials, (C_i, S_i), as the
// sample_points kernels stage them in LDS (acm.hip poly_to_lds).
struct alignas(16) RayPolyPair {
    double c, s;
};
typedef __attribute__((address_space(3))) const RayPolyPair lds_ray_poly;

// Uniform camera parameters, converted once per thread from the kernel
// argument (they stay in SGPRs: every lane reads the same values).
template <class T>
struct Cam {
    T p[9];
    T w, h;        // resolution as f64, like `width as f64` in the reference
    uint32_t wi, hi;
    // Per-camera constants of the unprojections (acm.hip make_cam / prep):
    // ifx, ify = RN(1 / fx), RN(1 / fy) from the host for div_by_f (0 = divide
    // instead), and uk = uniform subexpressions the reference evaluates per
    // point (IEEE results, identical wherever they are computed).
    T ifx, ify;
    T uk[4];
    // KB sample_points (kc[1] > 0 only there): cells whose ru lies in the
    // host-certified kept interval [kc[0], kc[1]] (acm.hip kb_seg_cert) take
    // KannalaBrandt::ray_certified; kc[2] = its Newton steps (1 or 2) from
    // the initial-guess polynomial kc[3..11], or 3: the ray polynomials rp
    // (cos theta*, sin theta* / ru in r2; acm.hip kb_fit_ray).
    T kc[12];
    T rp[2 * kRayPolyN];
    // The same polynomials staged in LDS by the sample_points kernels (r04):
    // ray_certified<true> reads them from there, per evaluation, instead of
    // holding 34 doubles in SGPRs across the kernel -- together with the
    // general path's constants they exceeded the 102 SGPRs and spilled to
    // VGPR lanes (~100 v_readlane per 64-cell segment on the hot path).
    lds_ray_poly* rpl;
};

// (u - cx) / fx with fx uniform: RN(a / b) from the host's RN(1 / b) and the
// Markstein correction of div_rn, bit-identical to the IEEE division (see
// div_shared) while |a| and |b| lie in [2^-500, 2^500]; anything else (and
// every float) divides.  Saves an IEEE division sequence per coordinate.
template <class T>
__device__ __forceinline__ T div_by_f(T a, T b, T ib) {
    if constexpr (sizeof(T) == 8) {
        if (ib != T(0) && div_safe(a)) return div_rn(a, ib, b);
    }
    return a / b;
}

// ---------------------------------------------------------------- Pinhole
template <class T>
struct Pinhole {
    static constexpr int P = 4;
    // pinhole.rs:165-182
    template <bool WJ, bool FAST = false, bool EXACT = false>
    __device__ static __forceinline__ uint8_t project(const Cam<T>& c, T x, T y, T z, T& u,
                                                      T& v, T* ju, T* jv) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T iz = FAST ? T(1) / z : T(0);
        T fxx, fyy, rz = T(0);  // fx * x / z is (fx * x) / z (:170-171)
        if (FAST) {
            fxx = fx * (x * iz);
            fyy = fy * (y * iz);
        } else {
            rz = div2(fx * x, fy * y, z, fxx, fyy);
        }
        u = fxx + cx;  // :170
        v = fyy + cy;  // :171
        uint8_t st = ST_OK;
        if (u < T(0) || u >= c.w || v < T(0) || v >= c.h) st = ST_PROJECTION_OUT_SIDE_IMAGE;
        if (z < T(kEpsSqrt)) st = ST_POINT_AT_CAMERA_CENTER;  // :167, checked first
        if (WJ) {
            T xz, yz;
            if (FAST) {
                xz = x * iz;
                yz = y * iz;
            } else {  // x / z, y / z from the same reciprocal
                xz = div_by_y(x, z, rz);
                yz = div_by_y(y, z, rz);
            }
            ju[0] = xz; ju[1] = T(0); ju[2] = T(1); ju[3] = T(0);
            jv[0] = T(0); jv[1] = yz; jv[2] = T(0); jv[3] = T(1);
        }
        return st;
    }
    // pinhole.rs:228-246
    __device__ static __forceinline__ uint8_t unproject(const Cam<T>& c, T u, T v, T& X, T& Y,
                                                        T& Z) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const bool out = u < T(0) || u >= c.w || v < T(0) || v >= c.h;
        T mx = div_by_f(u - cx, fx, c.ifx);  // (u - cx) / fx
        T my = div_by_f(v - cy, fy, c.ify);
        T r2 = mx * mx + my * my;
        T norm = sqrt_rn(T(1) + r2);
        T ninv = T(1) / norm;
        X = mx * ninv;
        Y = my * ninv;
        Z = ninv;
        return out ? ST_POINT_IS_OUT_SIDE_IMAGE : ST_OK;
    }
};

// ----------------------------------------------------------------- RadTan
template <class T>
struct RadTan {
    static constexpr int P = 9;  // fx fy cx cy k1 k2 p1 p2 k3
    // rad_tan.rs:302-348
    template <bool WJ, bool FAST = false, bool EXACT = false>
    __device__ static __forceinline__ uint8_t project(const Cam<T>& c, T x, T y, T z, T& u,
                                                      T& v, T* ju, T* jv) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T k1 = c.p[4], k2 = c.p[5], p1 = c.p[6], p2 = c.p[7], k3 = c.p[8];
        const T iz = FAST ? T(1) / z : T(0);
        T xp, yp;
        if (FAST) {
            xp = x * iz;
            yp = y * iz;
        } else {
            div2(x, y, z, xp, yp);  // x / z, y / z (:315-316)
        }
        T r2 = xp * xp + yp * yp;
        T r4 = r2 * r2;
        T r6 = r4 * r2;
        T radial = T(1) + k1 * r2 + k2 * r4 + k3 * r6;
        T xd = xp * radial + T(2) * p1 * xp * yp + p2 * (r2 + T(2) * xp * xp);
        T yd = yp * radial + p1 * (r2 + T(2) * yp * yp) + T(2) * p2 * xp * yp;
        u = fx * xd + cx;
        v = fy * yd + cy;
        uint8_t st = ST_OK;
        if (u < T(0) || u >= c.w || v < T(0) || v >= c.h) st = ST_PROJECTION_OUT_SIDE_IMAGE;
        if (z < T(kEpsSqrt)) st = ST_POINT_AT_CAMERA_CENTER;  // :304
        if (WJ) {
            T xpyp2 = T(2) * xp * yp;
            ju[0] = xd; ju[1] = T(0); ju[2] = T(1); ju[3] = T(0);
            ju[4] = fx * xp * r2;
            ju[5] = fx * xp * r4;
            ju[6] = fx * xpyp2;
            ju[7] = fx * (r2 + T(2) * xp * xp);
            ju[8] = fx * xp * r6;
            jv[0] = T(0); jv[1] = yd; jv[2] = T(0); jv[3] = T(1);
            jv[4] = fy * yp * r2;
            jv[5] = fy * yp * r4;
            jv[6] = fy * (r2 + T(2) * yp * yp);
            jv[7] = fy * xpyp2;
            jv[8] = fy * yp * r6;
        }
        return st;
    }
    // rad_tan.rs:401-524: Newton on the 2x2 distortion Jacobian, <=100 steps,
    // split into init / step / finish (the round-2 lane-refill experiment ran
    // the same per-point iterates from them; CHANGELOG round 2); unproject() chains
    // them.
    struct Newton {
        T tx, ty, px, py;
        unsigned it;
        uint8_t st;
    };
    // :401-433; false when the pixel is outside the image (the ray is NaN).
    // INSIDE: the caller knows the bounds test is false -- a pixel RadTan's
    // own project() returned Ok (it applies the same test, :339-345) or a
    // NaN pixel (every comparison false) -- so it is not evaluated.
    template <bool INSIDE = false>
    __device__ static __forceinline__ bool newton_init(const Cam<T>& c, T u, T v, Newton& s) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        if (!INSIDE && (u < T(0) || u >= c.w || v < T(0) || v >= c.h)) {
            s.st = ST_POINT_IS_OUT_SIDE_IMAGE;
            return false;
        }
        s.tx = div_by_f(u - cx, fx, c.ifx);  // (u - cx) / fx
        s.ty = div_by_f(v - cy, fy, c.ify);
        s.px = s.tx;
        s.py = s.ty;
        s.it = 0;
        s.st = ST_OK;
        return true;
    }
    // one pass of the loop at :436-518; true when the loop has ended
    __device__ static __forceinline__ bool newton_step(const Cam<T>& c, Newton& s) {
        const T k1 = c.p[4], k2 = c.p[5], p1 = c.p[6], p2 = c.p[7], k3 = c.p[8];
        T x = s.px, y = s.py;
        T r2 = x * x + y * y;
        T r4 = r2 * r2;
        T r6 = r4 * r2;
        T rad = T(1) + k1 * r2 + k2 * r4 + k3 * r6;
        T xe = x * rad + T(2) * p1 * x * y + p2 * (r2 + T(2) * x * x);
        T ye = y * rad + p1 * (r2 + T(2) * y * y) + T(2) * p2 * x * y;
        T ex = xe - s.tx, ey = ye - s.ty;
        // A NaN error can never pass the two EPS tests nor make det == 0,
        // so the reference would spin to MAX_ITERATIONS and return
        // NumericalError (:514-520): stop now with the same outcome.  This
        // keeps NaN/inf pixels (0.1% of the bench cloud) from holding
        // their whole wave for 100 iterations.
        if (ex != ex || ey != ey) { s.st = ST_NUMERICAL_ERROR; return true; }
        if (norm_below_1e6(ex * ex + ey * ey)) return true;  // :459, sqrt(.) < EPS
        T drdx = T(2) * x, drdy = T(2) * y;
        T ddx = (k1 + T(2) * k2 * r2 + T(3) * k3 * r4) * drdx;
        T ddy = (k1 + T(2) * k2 * r2 + T(3) * k3 * r4) * drdy;
        T j00 = rad + x * ddx + T(2) * p1 * y + p2 * (drdx + T(4) * x);
        T j01 = x * ddy + T(2) * p1 * x + p2 * (drdy);
        T j10 = y * ddx + p1 * (drdx) + T(2) * p2 * y;
        T j11 = rad + y * ddy + p1 * (drdy + T(4) * y) + T(2) * p2 * x;
        // nalgebra Matrix2::try_inverse: det = m11*m22 - m21*m12
        T det = j00 * j11 - j10 * j01;
        if (det == T(0)) { s.st = ST_NUMERICAL_ERROR; return true; }
        const T nq[4] = {j11, -j01, -j10, j00};
        T inv[4];
        div_shared(nq, det, inv);  // = j11 / det, -j01 / det, -j10 / det, j00 / det
        T i00 = inv[0], i01 = inv[1];
        T i10 = inv[2], i11 = inv[3];
        T dx = i00 * ex + i01 * ey;
        T dy = i10 * ex + i11 * ey;
        s.px = s.px - dx;
        s.py = s.py - dy;
        if (norm_below_1e6(dx * dx + dy * dy)) return true;  // :503, sqrt(.) < EPS
        if (s.it == 99u) { s.st = ST_NUMERICAL_ERROR; return true; }  // :514
        ++s.it;
        return false;
    }
    // Certified fast Newton (double only), the RadTan analogue of
    // KannalaBrandt::newton_fast.  The reference's step (:436-518) is ~110
    // VALU instructions: unfused products and sums, j10 computed apart from
    // j01 (they are equal), and four IEEE divisions by det.  Here the same
    // step takes FMAs, j10 = j01 and 1 / det from v_rcp_f64 + one Newton
    // step (~55 instructions).  Accepted only while |x|, |y| <= 2,
    // |det| >= 1/16 and |j00| + |j11| + 2 |j01| <= 64 (so ||J^-1|| <= 1024)
    // and both convergence tests (:459 on the error, :503 on the step) fall
    // outside a 2^-10 relative band around the squared threshold; with the
    // per-camera bound on the distortion terms (unproject_consts) the
    // residual differs from the reference's by < 2e-14 and the step by
    // < 2e-11, against a band of ~5e-10 on the norm.  Returns true only when
    // the reference's loop breaks at the same step as converged (at most 12
    // steps of its 100); anything uncertain, and every NaN, returns false and
    // the caller runs newton_step from the start.
    __device__ static __forceinline__ bool newton_fast(const Cam<T>& c, T tx, T ty, T& px,
                                                       T& py) {
        const T k1 = c.p[4], k2 = c.p[5], p1 = c.p[6], p2 = c.p[7];
        T k3 = c.p[8];
        const T k2d = k2 + k2, k3t = T(3) * k3, p1d = p1 + p1, p2d = p2 + p2;
        const T p1s = T(6) * p1, p2s = T(6) * p2;
        constexpr T lo = T(kNewtonTol2) * (T(1) - T(0x1p-10));
        constexpr T hi = T(kNewtonTol2) * (T(1) + T(0x1p-10));
        T x = tx, y = ty;
        int state = 0;  // 0 iterating, 1 certified converged, 2 uncertain
        // uk[1] = S > 0 (r05, acm.hip radtan_newton_disk): on the disk
        // x^2 + y^2 <= S the host has bounded |det| >= 1/16 and the row sums
        // <= 64 for every point, so the step needs only the test s <= S.  k3
        // is copied to a VGPR once: fma(k3, s, k2) with both in SGPRs cost a
        // v_mov per step (one scalar operand per VALU instruction).
        const T S = c.uk[1];
        if (S > T(0)) {
            asm volatile("" : "+v"(k3));
#pragma unroll 1
            for (int i = 0; i < 12 && state == 0; ++i) {
                const T x2 = x * x, y2 = y * y, xy = x * y;
                const T s = x2 + y2;
                int st;
                if (!(s <= S)) {
                    st = 2;  // outside the disk, or NaN
                } else {
                    // (r05) the target folded into the FMA chains, s + 2 x^2
                    // from x^2, and J's sums chained as FMAs: 6 fewer VALU
                    // instructions per step than the r04 form, the same
                    // quantities to within a few ulps of their terms (far
                    // inside the certification bands)
                    const T rad = fma(fma(fma(k3, s, k2), s, k1), s, T(1));
                    const T ex = fma(x, rad, fma(p1d, xy, fma(p2, fma(T(2), x2, s), -tx)));
                    const T ey = fma(y, rad, fma(p1, fma(T(2), y2, s), fma(p2d, xy, -ty)));
                    const T en2 = fma(ex, ex, ey * ey);
                    if (en2 < lo) {
                        st = 1;  // :459 breaks before the step
                    } else if (!(en2 > hi)) {
                        st = 2;  // in the band, or NaN
                    } else {
                        const T cm = fma(fma(k3t, s, k2d), s, k1);
                        const T w = cm + cm;
                        const T j00 = fma(x2, w, fma(p1d, y, fma(p2s, x, rad)));
                        const T j11 = fma(y2, w, fma(p1s, y, fma(p2d, x, rad)));
                        const T j01 = fma(xy, w, fma(p1d, x, p2d * y));
                        const T det = fma(j00, j11, -(j01 * j01));
                        const T r0 = __builtin_amdgcn_rcp(det);
                        const T id = fma(r0, fma(-det, r0, T(1)), r0);
                        const T dx = fma(j11, ex, -(j01 * ey)) * id;
                        const T dy = fma(j00, ey, -(j01 * ex)) * id;
                        x -= dx;
                        y -= dy;
                        const T dn2 = fma(dx, dx, dy * dy);
                        st = dn2 < lo ? 1 : (dn2 > hi ? 0 : 2);  // :503
                    }
                }
                state = st;
            }
            px = x;
            py = y;
            return state == 1;
        }
#pragma unroll 1
        for (int i = 0; i < 12 && state == 0; ++i) {
            const T x2 = x * x, y2 = y * y, xy = x * y;
            const T s = x2 + y2;
            const T rad = fma(fma(fma(k3, s, k2), s, k1), s, T(1));
            const T ex = fma(x, rad, fma(p1d, xy, fma(p2, fma(T(2), x2, s), -tx)));
            const T ey = fma(y, rad, fma(p1, fma(T(2), y2, s), fma(p2d, xy, -ty)));
            const T en2 = fma(ex, ex, ey * ey);
            int st;
            if (!(fabs(x) <= T(2) && fabs(y) <= T(2))) {
                st = 2;
            } else if (en2 < lo) {
                st = 1;  // :459 breaks before the step
            } else if (!(en2 > hi)) {
                st = 2;  // in the band, or NaN
            } else {
                const T cm = fma(fma(k3t, s, k2d), s, k1);  // k1 + 2 k2 r2 + 3 k3 r4
                const T w = cm + cm;
                const T j00 = fma(x2, w, fma(p1d, y, fma(p2s, x, rad)));
                const T j11 = fma(y2, w, fma(p1s, y, fma(p2d, x, rad)));
                const T j01 = fma(xy, w, fma(p1d, x, p2d * y));
                const T det = fma(j00, j11, -(j01 * j01));
                const T sj = fabs(j00) + fabs(j11) + T(2) * fabs(j01);
                if (!(fabs(det) >= T(0.0625) && sj <= T(64))) {
                    st = 2;
                } else {
                    const T r0 = __builtin_amdgcn_rcp(det);
                    const T id = fma(r0, fma(-det, r0, T(1)), r0);
                    const T dx = fma(j11, ex, -(j01 * ey)) * id;
                    const T dy = fma(j00, ey, -(j01 * ex)) * id;
                    x -= dx;
                    y -= dy;
                    const T dn2 = fma(dx, dx, dy * dy);
                    st = dn2 < lo ? 1 : (dn2 > hi ? 0 : 2);  // :503
                }
            }
            state = st;
        }
        px = x;
        py = y;
        return state == 1;
    }
    // :520-524: (x, y, 1).normalize()
    __device__ static __forceinline__ uint8_t newton_finish(const Newton& s, T& X, T& Y, T& Z) {
        T n = sqrt_rn(s.px * s.px + s.py * s.py + T(1) * T(1));
        const T nq[2] = {s.px, s.py};
        T q[2];
        Z = div_shared(nq, n, q);  // X = px / n, Y = py / n, Z = 1 / n
        X = q[0];
        Y = q[1];
        return s.st;
    }
    template <bool INSIDE = false>
    __device__ static __forceinline__ uint8_t unproject(const Cam<T>& c, T u, T v, T& X, T& Y,
                                                        T& Z) {
        Newton s;
        if (!newton_init<INSIDE>(c, u, v, s)) {
            X = Y = Z = T(NAN);
            return s.st;
        }
        // A NaN pixel passes the bounds test (every comparison is false) and
        // the reference then iterates on NaN errors until MAX_ITERATIONS:
        // NumericalError (:514-520), as newton_step's NaN exit returns.
        // Taken here, before the fast loop, so a failed projection's NaN
        // pixel (an unfiltered round trip has ~13% of them) does not send
        // its whole wave through the reference loop's first step.
        if (!(s.tx == s.tx && s.ty == s.ty)) {
            X = Y = Z = T(NAN);
            return ST_NUMERICAL_ERROR;
        }
#ifndef ACM_IEEE_MATH
        if constexpr (sizeof(T) == 8) {
            T px, py;  // uk[0] NaN: unbounded terms, or ACM_REFERENCE_NEWTON
            if (c.uk[0] == c.uk[0] && newton_fast(c, s.tx, s.ty, px, py)) {
                // (x, y, 1).normalize() with 1 / |p| from rsq + Newton (~1 ulp)
                const T in = rsq_nr(fma(px, px, fma(py, py, T(1))));
                X = px * in;
                Y = py * in;
                Z = in;
                return ST_OK;
            }
        }
#endif
        while (!newton_step(c, s)) {
        }
        return newton_finish(s, X, Y, Z);
    }

};

// --------------------------------------------------------- Kannala-Brandt
template <class T>
struct KannalaBrandt {
    static constexpr int P = 8;  // fx fy cx cy k1 k2 k3 k4
    // kannala_brandt.rs:340-394
    template <bool WJ, bool FAST = false, bool EXACT = false>
    __device__ static __forceinline__ uint8_t project(const Cam<T>& c, T x, T y, T z, T& u,
                                                      T& v, T* ju, T* jv) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T k1 = c.p[4], k2 = c.p[5], k3 = c.p[6], k4 = c.p[7];
        uint8_t st = z < T(0) ? ST_POINT_IS_OUT_SIDE_IMAGE
                              : (z < T(kEps) ? ST_POINT_AT_CAMERA_CENTER : ST_OK);
        const T r2 = x * x + y * y;  // :363-364
        T r, theta, ir = T(0);
        bool axis;
#ifndef ACM_IEEE_MATH
        if constexpr (sizeof(T) == 8 && !EXACT) {
            // r, 1/r and the atan2 quotient from rsq / rcp + Newton (~1 ulp;
            // the model is already held to 1e-10, not bit-exactness).  The
            // axis test r < EPS (:375) stays exact (kAxisR2).
            if (nr_range(r2) && nr_range(z) && z < T(INFINITY)) {
                ir = rsq_nr(r2);
                r = r2 * ir;
                const bool swap = r > z;  // atan2(r, z), z > 0 finite
                const T q = swap ? z * ir : r * rcp_nr(z);
                const T at = atan01(q);
                theta = swap ? T(1.5707963267948966) - at : at;
            } else {
                r = sqrt_rn(r2);
                theta = atan2_ge0(r, z);  // :365 (r >= 0)
                ir = T(1) / r;
            }
            axis = r2 < T(kAxisR2);  // == sqrt(r2) < EPS (:375), exactly
        } else
#endif
        {
            r = sqrt_rn(r2);
            theta = EXACT ? atan2_exact(r, z) : atan2_ge0(r, z);  // :365 (r >= 0)
            axis = r < T(kEps);  // :375
            if (FAST) ir = T(1) / r;
        }
        T theta2 = theta * theta;
        T theta3 = theta2 * theta;
        T theta5 = theta3 * theta2;
        T theta7 = theta5 * theta2;
        T theta9 = theta7 * theta2;
        T theta_d = theta + k1 * theta3 + k2 * theta5 + k3 * theta7 + k4 * theta9;
#ifndef ACM_IEEE_MATH
        constexpr bool kMul = FAST || (sizeof(T) == 8 && !EXACT);
#else
        constexpr bool kMul = FAST;
#endif
        T x_r = axis ? T(0) : (kMul ? x * ir : x / r);
        T y_r = axis ? T(0) : (kMul ? y * ir : y / r);
        u = fx * theta_d * x_r + cx;  // :390
        v = fy * theta_d * y_r + cy;
        if (WJ) {
            T fxr = fx * x_r, fyr = fy * y_r;
            ju[0] = theta_d * x_r; ju[1] = T(0); ju[2] = T(1); ju[3] = T(0);
            ju[4] = fxr * theta3; ju[5] = fxr * theta5; ju[6] = fxr * theta7; ju[7] = fxr * theta9;
            jv[0] = T(0); jv[1] = theta_d * y_r; jv[2] = T(0); jv[3] = T(1);
            jv[4] = fyr * theta3; jv[5] = fyr * theta5; jv[6] = fyr * theta7; jv[7] = fyr * theta9;
        }
        return st;
    }
    // The fused normal equations' view of project<true, true> (FAST): the
    // same u, v and status, and instead of the 2 x 8 Jacobian the scalars it
    // is built from -- a = theta_d x_r (du/dfx), b = theta_d y_r (dv/dfy),
    // fx x_r, fy y_r, theta^2, theta^3 -- since du/dk_i = fx x_r
    // theta^(2i+1) and dv/dk_i = fy y_r theta^(2i+1) (kannala_brandt.rs:
    // 367-390): k_normal_eq then accumulates the distortion block from
    // powers of theta on the fly instead of holding 16 Jacobian entries.
    __device__ static __forceinline__ uint8_t project_ne(const Cam<T>& c, T x, T y, T z, T& u,
                                                         T& v, T& a, T& b, T& fxr, T& fyr,
                                                         T& th2, T& th3) {
        // the FAST form of project() above, operation for operation
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T k1 = c.p[4], k2 = c.p[5], k3 = c.p[6], k4 = c.p[7];
        const uint8_t st = z < T(0) ? ST_POINT_IS_OUT_SIDE_IMAGE
                                    : (z < T(kEps) ? ST_POINT_AT_CAMERA_CENTER : ST_OK);
        const T r2 = x * x + y * y;
        T r, theta, ir;
        bool axis;
#ifndef ACM_IEEE_MATH
        if (nr_range(r2) && nr_range(z) && z < T(INFINITY)) {
            ir = rsq_nr(r2);
            r = r2 * ir;
            const bool swap = r > z;
            const T q = swap ? z * ir : r * rcp_nr(z);
            const T at = atan01(q);
            theta = swap ? T(1.5707963267948966) - at : at;
        } else {
            r = sqrt_rn(r2);
            theta = atan2_ge0(r, z);
            ir = T(1) / r;
        }
        axis = r2 < T(kAxisR2);
#else
        r = sqrt_rn(r2);
        theta = atan2_ge0(r, z);
        axis = r < T(kEps);
        ir = T(1) / r;
#endif
        th2 = theta * theta;
        th3 = th2 * theta;
        const T theta5 = th3 * th2, theta7 = theta5 * th2, theta9 = theta7 * th2;
        const T theta_d = theta + k1 * th3 + k2 * theta5 + k3 * theta7 + k4 * theta9;
        const T x_r = axis ? T(0) : x * ir;
        const T y_r = axis ? T(0) : y * ir;
        u = fx * theta_d * x_r + cx;
        v = fy * theta_d * y_r + cy;
        a = theta_d * x_r;
        b = theta_d * y_r;
        fxr = fx * x_r;
        fyr = fy * y_r;
        return st;
    }
    // Certified fast Newton (double only).  The reference's loop
    // (kannala_brandt.rs:474-511) costs ~38 VALU instructions per step: the
    // unfused products and sums it spells out plus an IEEE division.  Here
    // each step is the same Newton step in Horner form with FMAs and
    // delta = f * rcp(f') (~16 instructions), so the iterates differ from
    // the reference's by rounding only.  The decisions are certified, not
    // assumed: a step is accepted only when |f'| >= 1/16, |theta| <= 2 and
    // |delta| lies outside [PREC (1 - 2^-12), PREC (1 + 2^-12)].  With the
    // polynomial's terms bounded (sum |k_i| 4^i <= 63, checked per camera
    // in unproject_consts; NaN coefficients otherwise) f differs from the
    // reference's f by < 3e-13 and the iterates by < 4e-12, so the two
    // deltas differ by < 1e-11, far inside the 2.4e-10 band: every accepted
    // step makes the reference's break / continue decision, and the fast
    // loop returns true only when it reached the reference's `break` within
    // 6 steps (the reference gives up after 10).  Anything else -- a delta
    // in the band, a small or non-finite f', a wandering theta, more than 6
    // steps, NaN -- returns false and the caller runs the reference loop from
    // the start, so the status is the reference's in every case and theta
    // within a few ulp of its theta.
    __device__ static __forceinline__ bool newton_fast(const Cam<T>& c, T ru, T& theta) {
        const T k1 = c.p[4], k2 = c.p[5], k3 = c.p[6], k4 = c.p[7];
        constexpr T lo = T(1e-6) * (T(1) - T(0x1p-12)), hi = T(1e-6) * (T(1) + T(0x1p-12));
        // One lane state instead of early returns, and a rolled loop: an
        // unrolled loop with per-lane exits kept one exec mask per exit live
        // and spilled SGPRs in the sample_points tile loop.
        T t = ru;
        int state = 0;  // 0 iterating, 1 certified converged, 2 uncertain
#pragma unroll 1
        for (int i = 0; i < 6 && state == 0; ++i) {
            // f = t P(s) - ru and f' = P(s) + 2 s P'(s), s = t^2, P(s) =
            // 1 + k1 s + k2 s^2 + k3 s^3 + k4 s^4: P and P' by one Horner
            // pass with synthetic division, so only k1..k4 are needed (the
            // SGPR budget of the sample_points tile loop is tight)
            const T s = t * t;
            const T b3 = fma(k4, s, k3);
            const T c2 = fma(k4, s, b3);
            const T b2 = fma(b3, s, k2);
            const T c1 = fma(c2, s, b2);
            const T b1 = fma(b2, s, k1);
            const T c0 = fma(c1, s, b1);
            const T p = fma(b1, s, T(1));
            const T fp = fma(s + s, c0, p);
            const T f = fma(t, p, -ru);
            // 1 / f' from v_rcp_f64 and one Newton step: relative error
            // ~2^-44 at worst, i.e. < 1e-19 on a delta near the threshold
            const T y0 = __builtin_amdgcn_rcp(fp);
            const T y = fma(y0, fma(-fp, y0, T(1)), y0);
            const T d = f * y;
            t -= d;
            const T ad = fabs(d);
            // |f'| <= 1 + 9 * 63 here (|t| <= 2, bounded terms): only the
            // lower bound (and NaN) needs a test
            const bool sane = fabs(fp) >= T(0.0625) && fabs(t) <= T(2);
            state = !sane ? 2 : (ad < lo ? 1 : (ad > hi ? 0 : 2));  // band or NaN: 2
        }
        theta = t;
        return state == 1;
    }
    // The front of the unprojection on the certified path: ru from rsq + two
    // Newton steps (within ~1 ulp of the reference's IEEE sqrt, which is
    // within the Newton loop's error budget above) with the reference's two
    // decisions on it certified the same way -- ru > 1e-6 (:472) and the
    // pi/2 clamp (:467) are taken only when ru is 2^-30 (relative) away from
    // either threshold -- then newton_fast.  Returns false when anything is
    // uncertain; the caller then runs the reference's own sequence.  On
    // success ir ~= 1 / ru (the rsq itself, or 2 / pi after the clamp).
    __device__ static __forceinline__ bool front_fast(const Cam<T>& c, T r2, T& ru, T& theta,
                                                      T& ir) {
        // uk[0] NaN: the camera's terms are unbounded, or ACM_REFERENCE_NEWTON
        if (!nr_range(r2) || !(c.uk[0] == c.uk[0])) return false;
        const T y = rsq_nr(r2);
        const T rf = r2 * y;
        constexpr T kHalfPi = T(kPi / 2.0);
        constexpr T kLoPrec = T(1e-6) * (T(1) + T(0x1p-30));
        constexpr T kClampLo = kHalfPi * (T(1) - T(0x1p-30)), kClampHi = kHalfPi * (T(1) + T(0x1p-30));
        if (!(rf > kLoPrec)) return false;
        const bool clamp = rf > kClampHi;
        if (!clamp && !(rf < kClampLo)) return false;
        ru = clamp ? kHalfPi : rf;
        ir = clamp ? T(2.0 / kPi) : y;
        return newton_fast(c, ru, theta);
    }
    // The ray of a cell the host has certified Ok and kept (sample_points):
    // the status and the keep decision are known, and the ray is held to
    // 1e-10, so theta need not follow the reference's iterates -- only be
    // accurate.  The reference stops at |delta| < 1e-6, i.e. within ~M 1e-12
    // of the root theta* (kb_seg_cert's bound); here theta_0 = ru g(ru^2),
    // the host's fit of theta*(ru) (its error e0 measured on the host), then
    // kc[2] Newton steps -- one when M e0^2 is already at rounding level,
    // else two (M^3 e0^4 <= 1e-13).  1 / ru from rsq.  The certified interval
    // ends below the clamp (ru = |m| < pi/2), so (sin(theta) m / ru,
    // cos(theta)) is a unit vector up to rounding (sin^2 + cos^2 = 1): no
    // normalisation -- within a few ulp of the reference's normalised ray.
    //
    // kc[2] = 3 (the default wherever the host fit holds, r03): the ray is
    // read off two polynomials in r2 = ru^2 the host fits per camera on the
    // certified interval, C(r2) = cos(theta*(ru)) and S(r2) = sin(theta*(ru))
    // / ru (both analytic in r2; long-double roots at Chebyshev nodes, the
    // error bounded and required <= 1e-13, kb_fit_ray): X =
    // mx S, Y = my S, Z = C -- 34 FMAs instead of the square root, the
    // initial guess, the Newton step and sin / cos (~55 FP64 operations).
    // POLY selects the form at compile time (the launcher picks the kernel
    // by kc[2]): a kernel holding both forms' coefficients spilled SGPRs.
    template <bool POLY>
    __device__ static __forceinline__ void ray_certified(const Cam<T>& c, T mx, T my, T r2, T& X,
                                                         T& Y, T& Z) {
        if constexpr (POLY) {
            // (C_i, S_i) pairs from LDS, one ds_read_b128 broadcast each; the
            // empty asm makes the table address opaque per evaluation, so
            // the reads stay here instead of being hoisted out of the
            // kernel's loops into 68 registers
            lds_ray_poly* q = c.rpl;
            asm volatile("" : "+v"(q));
            T cp = q[kRayPolyN - 1].c, sp = q[kRayPolyN - 1].s;
#pragma unroll
            for (int i = kRayPolyN - 2; i >= 0; --i) {
                cp = fma(cp, r2, q[i].c);
                sp = fma(sp, r2, q[i].s);
            }
            X = mx * sp;
            Y = my * sp;
            Z = cp;
            return;
        }
        const T k1 = c.p[4], k2 = c.p[5], k3 = c.p[6], k4 = c.p[7];
        const T ir = rsq_nr(r2);
        const T ru = r2 * ir;
        const T s0 = ru * ru;
        T g = c.kc[11];
#pragma unroll
        for (int i = 10; i >= 3; --i) g = fma(g, s0, c.kc[i]);
        T t = ru * g;
        const int steps = c.kc[2] > T(1.5) ? 2 : 1;
#pragma unroll 1
        for (int it = 0; it < steps; ++it) {
            const T s = t * t;
            const T b3 = fma(k4, s, k3);
            const T c2 = fma(k4, s, b3);
            const T b2 = fma(b3, s, k2);
            const T c1 = fma(c2, s, b2);
            const T b1 = fma(b2, s, k1);
            const T c0 = fma(c1, s, b1);
            const T pp = fma(b1, s, T(1));
            const T fp = fma(s + s, c0, pp);
            const T f = fma(t, pp, -ru);
            const T y0 = __builtin_amdgcn_rcp(fp);
            t -= f * fma(y0, fma(-fp, y0, T(1)), y0);
        }
        T sn, cs;
#ifdef ACM_AB_RAY_SINCOS_FALLBACK  // A/B build (Makefile lib/libacm_ab.so)
        sincos_0_2(t, &sn, &cs);
#else
        sincos_poly_0_2(t, &sn, &cs);  // theta in [0, pi/2): no OCML fallback
#endif
        const T q = sn * ir;  // sin(theta) / ru
        X = mx * q;
        Y = my * q;
        Z = cs;
    }

    // kannala_brandt.rs:445-562: Newton on theta_d(theta) = ru, <=10 steps.
    __device__ static __forceinline__ uint8_t unproject(const Cam<T>& c, T u, T v, T& X, T& Y,
                                                        T& Z) {
        bool keep;
        return unproject_k<false>(c, u, v, X, Y, Z, keep);
    }
    // The largest double below pi/2.  For a double theta with |theta| <= 2,
    // cos(theta) > 0 exactly when |theta| <= kHalfPiDown (cos(kHalfPiDown) =
    // +6.1e-17, cos of the next double up = -1.6e-16: any faithful libm,
    // glibc's included, gets both signs right).
    static constexpr double kHalfPiDown = 0x1.921fb54442d18p0;
    // unproject_k<true> also returns the sample_points keep decision
    // (point_sampling.rs:91-94: Ok and z > 0) decided exactly, not read off
    // the ray: z = cos(theta) / |p| > 0 iff cos(theta) > 0 (and |p| finite),
    // taken by the comparison above on the reference's own theta -- not on
    // the polynomial cos, whose 3.3e-16 absolute error exceeds cos(theta)
    // at kHalfPiDown.  The certified fast Newton's theta is within 4e-12 of
    // the reference's; when it lies within 1e-11 of the threshold the pixel
    // runs the reference loop, so the comparison always sees either a theta
    // on the same side as the reference's or the reference's theta itself.
    template <bool KEEP, bool POLY = false>
    __device__ static __forceinline__ uint8_t unproject_k(const Cam<T>& c, T u, T v, T& X, T& Y,
                                                          T& Z, bool& keep) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T k1 = c.p[4], k2 = c.p[5], k3 = c.p[6], k4 = c.p[7];
        keep = false;
        if (c.wi > 0 && c.hi > 0 && (u < T(0) || u >= c.w || v < T(0) || v >= c.h)) {
            X = Y = Z = T(NAN);
            return ST_POINT_IS_OUT_SIDE_IMAGE;  // :447-455
        }
        T mx = div_by_f(u - cx, fx, c.ifx);  // (u - cx) / fx
        T my = div_by_f(v - cy, fy, c.ify);
        const T r2 = mx * mx + my * my;
        const T PREC = T(1e-6);
        T ru, theta, ir_fast = T(0);
        bool converged = true;
        bool certified = false;
#ifndef ACM_IEEE_MATH
        if constexpr (sizeof(T) == 8 && KEEP) {
            // sample_points: a cell inside the host-certified kept interval
            // is Ok and kept whatever its Newton run does (kb_seg_cert), so
            // only its ray is needed, to 1e-10: ray_certified
            if (r2 >= c.kc[0] * c.kc[0] * T(1 + 0x1p-30) &&
                r2 <= c.kc[1] * c.kc[1] * T(1 - 0x1p-30)) {
                ray_certified<POLY>(c, mx, my, r2, X, Y, Z);
                keep = true;
                return ST_OK;
            }
        }
        if constexpr (sizeof(T) == 8) {
            // A NaN pixel: ru = min(NaN, pi/2) = pi/2 (f64::min returns the
            // other operand, :467), the loop runs on that constant, and the
            // ray is NaN (mx / ru); the status of that run is a camera
            // constant, precomputed on the host by the same reference loop
            // (uk[1], unproject_consts).  Skips the reference loop per pixel.
            if (r2 != r2) {
                X = Y = Z = T(NAN);
                return (uint8_t)c.uk[1];
            }
            certified = front_fast(c, r2, ru, theta, ir_fast);
            if (KEEP && certified && fabs(fabs(theta) - T(kHalfPiDown)) <= T(1e-11))
                certified = false;  // too close to call: take the reference's theta
        }
#endif
        if (!certified) {  // the reference's sequence (:462-525)
            ru = sqrt_rn(r2);
            ru = fmin(ru, T(kPi / 2.0));  // :467, f64::min semantics
            theta = ru;
            if (ru > PREC) {
                for (int i = 0; i < 10; ++i) {
                    T theta2 = theta * theta;
                    T theta4 = theta2 * theta2;
                    T theta6 = theta4 * theta2;
                    T theta8 = theta4 * theta4;
                    T k1t2 = k1 * theta2, k2t4 = k2 * theta4, k3t6 = k3 * theta6, k4t8 = k4 * theta8;
                    T f = theta * (T(1) + k1t2 + k2t4 + k3t6 + k4t8) - ru;
                    T fp = T(1) + (T(3) * k1t2) + (T(5) * k2t4) + (T(7) * k3t6) + (T(9) * k4t8);
                    if (fabs(fp) < T(kEps)) { converged = false; break; }
                    T delta = f / fp;
                    theta -= delta;
                    if (fabs(delta) < PREC) break;
                    if (i == 9) converged = false;
                }
            } else {
                if (ru > T(0)) converged = false;
                else { theta = T(0); }
            }
        }
        const bool small = fabs(ru) < T(kEps);
        T s, co;
        sincos_0_2(theta, &s, &co);  // polynomial on [0, 2], OCML sincos beyond
        // cos(theta) > 0, exactly (see kHalfPiDown); beyond |theta| = 2 the
        // sign of any faithful cos is right (no double lies that close to an
        // odd multiple of pi/2)
        const bool cos_pos = fabs(theta) <= T(2) ? fabs(theta) <= T(kHalfPiDown) : co > T(0);
#ifndef ACM_IEEE_MATH
        if constexpr (sizeof(T) == 8) {
            // Everything after the Newton loop only shapes the ray: no status
            // decision depends on it, and the ray is held to 1e-10 anyway
            // (sin / cos are polynomials).  1 / ru and 1 / |p| from rcp / rsq
            // + Newton (~1 ulp) instead of two IEEE divisions and a sqrt.
#ifndef ACM_AB_KB_NORMALIZE  // A/B build: normalise every certified ray (r05)
            if (certified && ru < T(kPi / 2.0)) {
                // (r06) not clamped: ru = |m| (to ~1 ulp, from rsq) and
                // (sin(theta) m / ru, cos(theta)) is a unit vector up to
                // rounding, so the reference's normalize() (:545-561) moves
                // it by ~1 ulp: no |p|, no rsq -- the 16 VALU instructions of
                // the normalisation, ~5% of the KB round trip.  (The clamped
                // ray, ru = pi/2 < |m|, is not unit: normalised below.)
                const T q = s * ir_fast;  // sin(theta) / ru
                X = mx * q;
                Y = my * q;
                Z = co;
                keep = converged && cos_pos;
                return ST_OK;
            }
#endif
            const T ir = certified ? ir_fast : (nr_range(ru) ? rcp_nr(ru) : T(1) / ru);
            const T xc = small ? T(0) : mx * ir;  // mx / ru
            const T yc = small ? T(0) : my * ir;
            const T px = s * xc, py = s * yc;
            const T n2 = px * px + py * py + co * co;
            const T in = nr_range(n2) ? rsq_nr(n2) : T(1) / sqrt_rn(n2);
            X = px * in;
            Y = py * in;
            Z = co * in;
            // |p| finite: z = cos / |p| is 0 (dropped) when |p| overflows
            keep = converged && cos_pos && n2 < T(INFINITY);
            return converged ? ST_OK : ST_NUMERICAL_ERROR;
        }
#endif
        const T mxy[2] = {mx, my};
        T c2[2];
        div_shared(mxy, ru, c2);  // mx / ru, my / ru
        T xc = small ? T(0) : c2[0];
        T yc = small ? T(0) : c2[1];
        T px = s * xc, py = s * yc;
        T n2 = px * px + py * py + co * co;
        T n = sqrt_rn(n2);
        const T nq[3] = {px, py, co};
        T q[3];
        div_shared(nq, n, q);
        X = q[0];
        Y = q[1];
        Z = q[2];
        keep = converged && cos_pos && n2 < T(INFINITY);
        return converged ? ST_OK : ST_NUMERICAL_ERROR;
    }
};

// ---------------------------------------------------------- Double Sphere
template <class T>
struct DoubleSphere {
    static constexpr int P = 6;  // fx fy cx cy alpha xi
    // double_sphere.rs:361-390 + check_projection_condition :177-184
    template <bool WJ, bool FAST = false, bool EXACT = false>
    __device__ static __forceinline__ uint8_t project(const Cam<T>& c, T x, T y, T z, T& u,
                                                      T& v, T* ju, T* jv) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T alpha = c.p[4], xi = c.p[5];
        T r_squared = (x * x) + (y * y);
        T d1 = sqrt_rn(r_squared + (z * z));
        T gamma = xi * d1 + z;
        T d2 = sqrt_rn(r_squared + gamma * gamma);
        T denom = alpha * d2 + (T(1) - alpha) * gamma;
        // w2 (from w1): a camera constant, computed once per camera with the
        // same IEEE operations (acm.hip unproject_consts, uk[1]; r05: it cost
        // a division and a square root per point)
        const T w2 = c.uk[1];
        const bool ok = !(denom < T(1e-3)) && (z > -w2 * d1);
        const T id = FAST ? T(1) / denom : T(0);
        T mx, my, yd = T(0);
        if (FAST) {
            mx = x * id;
            my = y * id;
        } else {
            yd = div2(x, y, denom, mx, my);  // x / denom, y / denom (:383-384)
        }
        u = fx * (mx) + cx;
        v = fy * (my) + cy;
        if (WJ) {
            T tu = FAST ? fx * mx * id : div_by_y(fx * mx, denom, yd);
            T tv = FAST ? fy * my * id : div_by_y(fy * my, denom, yd);
            T dda = d2 - gamma;
            T ddx = d1 * (alpha * gamma / d2 + (T(1) - alpha));
            ju[0] = mx; ju[1] = T(0); ju[2] = T(1); ju[3] = T(0);
            ju[4] = -tu * dda; ju[5] = -tu * ddx;
            jv[0] = T(0); jv[1] = my; jv[2] = T(0); jv[3] = T(1);
            jv[4] = -tv * dda; jv[5] = -tv * ddx;
        }
        return ok ? ST_OK : ST_POINT_IS_OUT_SIDE_IMAGE;
    }
    // double_sphere.rs:436-476 + check_unprojection_condition :200-209
    __device__ static __forceinline__ uint8_t unproject(const Cam<T>& c, T u, T v, T& X, T& Y,
                                                        T& Z) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T alpha = c.p[4], xi = c.p[5];
        T gamma_ds = T(1) - alpha;
        T mx = div_by_f(u - cx, fx, c.ifx);  // (u - cx) / fx
        T my = div_by_f(v - cy, fy, c.ify);
        T r_squared = (mx * mx) + (my * my);
        // c.uk[0] = 1 / (2 alpha - 1)
        const bool cond = !(alpha > T(0.5) && r_squared > c.uk[0]);
        const bool reject = alpha != T(0) && !cond;
        T mz = (T(1) - alpha * alpha * r_squared) /
               (alpha * sqrt_rn(T(1) - (T(2) * alpha - T(1)) * r_squared) + gamma_ds);
        T mz_squared = mz * mz;
        T num = mz * xi + sqrt_rn(mz_squared + (T(1) - xi * xi) * r_squared);
        T denom = mz_squared + r_squared;
        T coeff = num / denom;
        T px = coeff * mx, py = coeff * my, pz = coeff * mz - xi;
        T n = sqrt_rn(px * px + py * py + pz * pz);
        const T nq[3] = {px, py, pz};
        T q[3];
        div_shared(nq, n, q);
        X = q[0];
        Y = q[1];
        Z = q[2];
        return (reject || denom < T(1e-3)) ? ST_POINT_IS_OUT_SIDE_IMAGE : ST_OK;
    }
};

// -------------------------------------------------------------------- UCM
template <class T>
struct Ucm {
    static constexpr int P = 5;  // fx fy cx cy alpha
    // ucm.rs:297-316 + check_proj_condition :154-161
    template <bool WJ, bool FAST = false, bool EXACT = false>
    __device__ static __forceinline__ uint8_t project(const Cam<T>& c, T x, T y, T z, T& u,
                                                      T& v, T* ju, T* jv) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3], alpha = c.p[4];
        T d = sqrt_rn(x * x + y * y + z * z);
        T denom = alpha * d + (T(1) - alpha) * z;
        const T w = c.uk[2];  // per camera (acm.hip unproject_consts, r05)
        const bool ok = !(denom < T(1e-3)) && (z > -w * d);
        const T id = FAST ? T(1) / denom : T(0);
        T mx, my, yd = T(0);
        if (FAST) {
            mx = x * id;
            my = y * id;
        } else {
            yd = div2(x, y, denom, mx, my);  // x / denom, y / denom
        }
        u = fx * mx + cx;
        v = fy * my + cy;
        if (WJ) {
            T tu = FAST ? fx * mx * id : div_by_y(fx * mx, denom, yd);
            T tv = FAST ? fy * my * id : div_by_y(fy * my, denom, yd);
            T dda = d - z;
            ju[0] = mx; ju[1] = T(0); ju[2] = T(1); ju[3] = T(0); ju[4] = -tu * dda;
            jv[0] = T(0); jv[1] = my; jv[2] = T(0); jv[3] = T(1); jv[4] = -tv * dda;
        }
        return ok ? ST_OK : ST_POINT_IS_OUT_SIDE_IMAGE;
    }
    // ucm.rs:337-367 (+ :177-184); keeps the reference's denom = 1 - r^2 (:354)
    __device__ static __forceinline__ uint8_t unproject(const Cam<T>& c, T u, T v, T& X, T& Y,
                                                        T& Z) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3], alpha = c.p[4];
        T gamma = T(1) - alpha;
        T xi = c.uk[0];  // alpha / gamma
        T mx = div_by_f(u - cx, fx, c.ifx) * gamma;  // (u - cx) / fx * gamma
        T my = div_by_f(v - cy, fy, c.ify) * gamma;
        T r_squared = mx * mx + my * my;
        T num = xi + sqrt_rn(T(1) + (T(1) - xi * xi) * r_squared);
        T denom = T(1) - r_squared;
        // c.uk[1] = gamma * gamma / (2 alpha - 1)
        const bool cond = alpha > T(0.5) ? (r_squared <= c.uk[1]) : true;
        T coeff = num / denom;
        T px = coeff * mx, py = coeff * my, pz = coeff - xi;
        T n = sqrt_rn(px * px + py * py + pz * pz);
        const T nq[3] = {px, py, pz};
        T q[3];
        div_shared(nq, n, q);
        X = q[0];
        Y = q[1];
        Z = q[2];
        return (denom < T(1e-3) || !cond) ? ST_POINT_IS_OUT_SIDE_IMAGE : ST_OK;
    }
};

// ------------------------------------------------------------------- EUCM
template <class T>
struct Eucm {
    static constexpr int P = 6;  // fx fy cx cy alpha beta
    // eucm.rs:328-347 + check_proj_condition :167-177
    template <bool WJ, bool FAST = false, bool EXACT = false>
    __device__ static __forceinline__ uint8_t project(const Cam<T>& c, T x, T y, T z, T& u,
                                                      T& v, T* ju, T* jv) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T alpha = c.p[4], beta = c.p[5];
        T rr = x * x + y * y;
        T d = sqrt_rn(beta * rr + z * z);
        T denom = alpha * d + (T(1) - alpha) * z;
        bool cond = true;
        if (alpha > T(0.5)) {
            const T cc = c.uk[1];  // (alpha - 1) / (2 alpha - 1), per camera (r05)
            cond = !(z < denom * cc);
        }
        const bool ok = !(denom < T(1e-3)) && cond;
        const T id = FAST ? T(1) / denom : T(0);
        T mx, my, yd = T(0);
        if (FAST) {
            mx = x * id;
            my = y * id;
        } else {
            yd = div2(x, y, denom, mx, my);  // x / denom, y / denom
        }
        u = fx * mx + cx;
        v = fy * my + cy;
        if (WJ) {
            T tu = FAST ? fx * mx * id : div_by_y(fx * mx, denom, yd);
            T tv = FAST ? fy * my * id : div_by_y(fy * my, denom, yd);
            T dda = d - z;
            T ddb = alpha * rr / (T(2) * d);
            ju[0] = mx; ju[1] = T(0); ju[2] = T(1); ju[3] = T(0);
            ju[4] = -tu * dda; ju[5] = -tu * ddb;
            jv[0] = T(0); jv[1] = my; jv[2] = T(0); jv[3] = T(1);
            jv[4] = -tv * dda; jv[5] = -tv * ddb;
        }
        return ok ? ST_OK : ST_POINT_IS_OUT_SIDE_IMAGE;
    }
    // eucm.rs:368-398 (+ :194-200 precedence quirk (1/beta)*(2a-1))
    __device__ static __forceinline__ uint8_t unproject(const Cam<T>& c, T u, T v, T& X, T& Y,
                                                        T& Z) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3];
        const T alpha = c.p[4], beta = c.p[5];
        T mx = div_by_f(u - cx, fx, c.ifx);  // (u - cx) / fx
        T my = div_by_f(v - cy, fy, c.ify);
        T r_squared = mx * mx + my * my;
        T gamma = T(1) - alpha;
        T num = T(1) - r_squared * alpha * alpha * beta;
        T det = T(1) - (alpha - gamma) * beta * r_squared;
        T denom = gamma + alpha * sqrt_rn(det);
        // c.uk[0] = 1 / beta * (2 alpha - 1)
        const bool cond = !(alpha > T(0.5) && r_squared > c.uk[0]);
        T mz = num / denom;
        T n = sqrt_rn(mx * mx + my * my + mz * mz);
        const T nq[3] = {mx, my, mz};
        T q[3];
        div_shared(nq, n, q);
        X = q[0];
        Y = q[1];
        Z = q[2];
        return (det < T(1e-3) || !cond) ? ST_POINT_IS_OUT_SIDE_IMAGE : ST_OK;
    }
};

// -------------------------------------------------------------------- FOV
template <class T>
struct Fov {
    static constexpr int P = 5;  // fx fy cx cy w
    // fov.rs:284-316
    template <bool WJ, bool FAST = false, bool EXACT = false>
    __device__ static __forceinline__ uint8_t project(const Cam<T>& c, T x, T y, T z, T& u,
                                                      T& v, T* ju, T* jv) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3], wf = c.p[4];
        T r2 = x * x + y * y;
        T r = sqrt_rn(r2);
        const T tan_w_half = c.p[8];  // tan(w / 2), host-precomputed (acm.hip prep)
        T atan_wrd = EXACT ? atan2_exact(T(2) * tan_w_half * r, z)  // y >= 0
                           : atan2_ge0(T(2) * tan_w_half * r, z);
        const bool axis = r2 < T(kEpsSqrt);
        const T irw = FAST ? T(1) / (r * wf) : T(0);
        T rd = axis ? T(2) * tan_w_half / wf : (FAST ? atan_wrd * irw : atan_wrd / (r * wf));
        T mx = x * rd, my = y * rd;
        u = fx * mx + cx;
        v = fy * my + cy;
        if (WJ) {
            T drd;
            if (axis) {
                drd = ((T(1) + tan_w_half * tan_w_half) * wf - T(2) * tan_w_half) / (wf * wf);
            } else {
                T a = T(2) * tan_w_half * r;
                T datan = z * r * (T(1) + tan_w_half * tan_w_half) / (a * a + z * z);
                drd = FAST ? datan * irw - atan_wrd * irw / wf
                           : datan / (r * wf) - atan_wrd / (r * wf * wf);
            }
            ju[0] = mx; ju[1] = T(0); ju[2] = T(1); ju[3] = T(0); ju[4] = fx * x * drd;
            jv[0] = T(0); jv[1] = my; jv[2] = T(0); jv[3] = T(1); jv[4] = fy * y * drd;
        }
        return z < T(kEpsSqrt) ? ST_POINT_AT_CAMERA_CENTER : ST_OK;
    }
    // fov.rs:336-363
    __device__ static __forceinline__ uint8_t unproject(const Cam<T>& c, T u, T v, T& X, T& Y,
                                                        T& Z) {
        const T fx = c.p[0], fy = c.p[1], cx = c.p[2], cy = c.p[3], wf = c.p[4];
        const T tan_w_2 = c.p[8];  // tan(w / 2), host-precomputed
        T mul2 = tan_w_2 * T(2);
        T mx = div_by_f(u - cx, fx, c.ifx);  // (u - cx) / fx
        T my = div_by_f(v - cy, fy, c.ify);
#ifndef ACM_IEEE_MATH
        if constexpr (sizeof(T) == 8) {
            // Values-only fast form (uk[0] == 1; a per-call
            // ACM_REFERENCE_NEWTON sets NaN): rd and 1 / rd from rsq, sin / cos of rd w by sincos_0_2,
            // 1 / cos and 1 / |p| by rcp / rsq + Newton (~1-2 ulp each).  The
            // one decision, rd > sqrt(EPS) = 2^-26 (:320), is taken on r2
            // exactly: RN(sqrt(r2)) > 2^-26  <=>  r2 > 2^-52 (1 + 2^-52).
            const T r2 = mx * mx + my * my;
            if (c.uk[0] == c.uk[0] && r2 <= T(0x1p1000)) {
                T px = mx, py = my;
                if (mul2 > T(kEpsSqrt) && r2 > T(0x1.0000000000001p-52)) {
                    const T y = rsq_nr(r2);  // 1 / rd
                    T srw, crw;
                    sincos_0_2((r2 * y) * wf, &srw, &crw);
                    const T ru = srw * y * c.uk[1];  // sin(rd w) / (rd 2 tan(w / 2))
                    const T ic = nr_range(fabs(crw)) ? (crw < T(0) ? -rcp_nr(-crw) : rcp_nr(crw))
                                                     : T(1) / crw;
                    px = (mx * ru) * ic;
                    py = (my * ru) * ic;
                }
                const T n2 = fma(px, px, fma(py, py, T(1)));
                const T in = nr_range(n2) ? rsq_nr(n2) : T(1) / sqrt_rn(n2);
                X = px * in;
                Y = py * in;
                Z = in;
                return ST_OK;
            }
        }
#endif
        T rd = sqrt_rn(mx * mx + my * my);
        T px = mx, py = my;
        if (mul2 > T(kEpsSqrt) && rd > T(kEpsSqrt)) {
            T srw, crw;
            sincos(rd * wf, &srw, &crw);
            T ru = srw / (rd * mul2);
            const T nq[2] = {mx * ru, my * ru};
            T q[2];
            div_shared(nq, crw, q);  // (mx * ru) / crw, (my * ru) / crw
            px = q[0];
            py = q[1];
        }
        T n = sqrt_rn(px * px + py * py + T(1) * T(1));
        const T nq[2] = {px, py};
        T q[2];
        Z = div_shared(nq, n, q);  // X = px / n, Y = py / n, Z = 1 / n
        X = q[0];
        Y = q[1];
        return ST_OK;
    }
};

}  // namespace acm
