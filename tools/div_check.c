/* Exhaustive-style check of the shared-divisor division used by the HIP
 * kernels (camera_models.hpp div_rn): with y = RN(1/b) (an IEEE division),
 * q = RN(a*y), r = fma(-b, q, a), q' = fma(r, y, q) must equal RN(a/b) bit
 * for bit whenever |a|, |b| lie in [2^-500, 2^500].  Same IEEE binary64
 * arithmetic on x86 (mul, fma, div) as v_mul_f64 / v_fma_f64 / the IEEE
 * division sequence on gfx950.
 *
 *   div_check N MODE SEED   -> prints "mode M N n bad B", exit 1 if B > 0
 * MODE 0 random significands, 1 all-ones divisor significand, 2 short
 * divisor significands, 3 quotients near 1, 4 near-all-ones divisors,
 * 5 near-all-ones dividends over short divisors, 6 exponents at the guard
 * limits. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static double bits2d(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
static uint64_t d2bits(double d) { uint64_t b; memcpy(&b, &d, 8); return b; }
static uint64_t s[2] = {0x9E3779B97F4A7C15ull, 0xD1B54A32D192ED03ull};
static uint64_t rnd(void) {
    uint64_t s1 = s[0], s0 = s[1];
    s[0] = s0;
    s1 ^= s1 << 23;
    s[1] = s1 ^ s0 ^ (s1 >> 17) ^ (s0 >> 26);
    return s[1] + s0;
}

static double div_rn(double a, double y, double b) {
    double q = a * y;
    double r = fma(-b, q, a);
    return fma(r, y, q);
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    long n = atol(argv[1]);
    int mode = atoi(argv[2]);
    s[0] ^= (uint64_t)mode * 7919u + (uint64_t)atol(argv[3]);
    long bad = 0;
    for (long i = 0; i < n; i++) {
        uint64_t ma = rnd() & 0xFFFFFFFFFFFFFull, mb = rnd() & 0xFFFFFFFFFFFFFull;
        int ea = (int)(rnd() % 400) - 200, eb = (int)(rnd() % 400) - 200;
        if (mode == 1) mb = 0xFFFFFFFFFFFFFull;
        if (mode == 2) mb = rnd() & 0xFFull;
        if (mode == 3) { ma = mb ^ (rnd() & 0xFF); ea = eb + (int)(rnd() % 3) - 1; }
        if (mode == 4) mb = 0xFFFFFFFFFFFFFull - (rnd() & 0xFFFF);
        if (mode == 5) { ma = 0xFFFFFFFFFFFFFull - (rnd() & 0xFFFF); mb = rnd() & 0xFFFF; }
        if (mode == 6) { ea = (rnd() & 1) ? 499 : -500; eb = (rnd() & 1) ? 499 : -500; }
        double a = bits2d(((uint64_t)(ea + 1023) << 52) | ma) * ((rnd() & 1) ? -1.0 : 1.0);
        double b = bits2d(((uint64_t)(eb + 1023) << 52) | mb) * ((rnd() & 1) ? -1.0 : 1.0);
        double y = 1.0 / b;
        double q = div_rn(a, y, b), ref = a / b;
        if (d2bits(q) != d2bits(ref)) {
            if (bad < 5) printf("BAD a=%a b=%a q=%a ref=%a\n", a, b, q, ref);
            bad++;
        }
    }
    printf("mode %d N %ld bad %ld\n", mode, n, bad);
    return bad != 0;
}
