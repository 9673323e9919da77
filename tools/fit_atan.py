"""Coefficients of the polynomial atan used by k_fov_grid (acm.hip atan01):
degree-20 Chebyshev interpolant of atan(sqrt(s))/sqrt(s) on s in [0, 1],
computed with 60-digit mpmath, printed as hex floats split into the even
(c0, c2, ..., c20) and odd (c1, ..., c19) Horner chains.

  python tools/fit_atan.py            # print the two coefficient arrays
  python tools/fit_atan.py --check    # + max relative error vs glibc atan
                                      #   (C, fma, 2e8 arguments in [0, 1])
  python tools/fit_atan.py --sincos   # camera_models.hpp kSinS / kCosC: degree-10
                                      #   interpolants of sin(sqrt s)/sqrt s, cos(sqrt s)
                                      #   on s in [0, 4] (theta in [0, 2])
"""
import os
import subprocess
import sys
import tempfile

import mpmath as mp


def coefficients(deg=20):
    mp.mp.dps = 60

    def g(s):
        s = mp.mpf(s)
        if s == 0:
            return mp.mpf(1)
        r = mp.sqrt(s)
        return mp.atan(r) / r
    n = deg + 1
    nodes = [(mp.cos(mp.pi * (k + mp.mpf(1) / 2) / n) + 1) / 2 for k in range(n)]
    a = mp.matrix([[x ** j for j in range(n)] for x in nodes])
    c = mp.lu_solve(a, mp.matrix([g(x) for x in nodes]))
    cf = [float(c[j]) for j in range(n)]
    return cf[0::2], cf[1::2]


CHECK = r"""
#include <math.h>
#include <stdio.h>
static const double E[11] = {%s};
static const double O[10] = {%s};
static double atan01(double b) {
    double s = b * b, s2 = s * s, pe = E[10], po = O[9];
    for (int k = 9; k >= 0; --k) pe = fma(pe, s2, E[k]);
    for (int k = 8; k >= 0; --k) po = fma(po, s2, O[k]);
    return b * fma(po, s, pe);
}
int main(void) {
    double mx = 0, wb = 0;
    unsigned long long st = 88172645463325252ull;
    for (long i = 0; i < 200000000; i++) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        double b = (st >> 11) * 0x1p-53;
        if (i %% 4 == 0) b *= 1e-3;
        if (i == 0) b = 1.0;
        double r = atan(b);
        if (r == 0) continue;
        double e = fabs(atan01(b) - r) / fabs(r);
        if (e > mx) { mx = e; wb = b; }
    }
    printf("max rel err %%.3e at b=%%a\n", mx, wb);
    return 0;
}
"""


def sincos_coefficients(deg=10):
    mp.mp.dps = 60
    n = deg + 1
    nodes = [(mp.cos(mp.pi * (k + mp.mpf(1) / 2) / n) + 1) * 2 for k in range(n)]  # [0, 4]
    a = mp.matrix([[x ** j for j in range(n)] for x in nodes])

    def fs(s):
        return mp.mpf(1) if s == 0 else mp.sin(mp.sqrt(s)) / mp.sqrt(s)
    cs = mp.lu_solve(a, mp.matrix([fs(x) for x in nodes]))
    cc = mp.lu_solve(a, mp.matrix([mp.cos(mp.sqrt(x)) for x in nodes]))
    return [float(cs[j]) for j in range(n)], [float(cc[j]) for j in range(n)]


def main():
    if "--sincos" in sys.argv:
        s, c = sincos_coefficients()
        print("S:", ", ".join(v.hex() for v in s))
        print("C:", ", ".join(v.hex() for v in c))
        return
    e, o = coefficients()
    print("E:", ", ".join(v.hex() for v in e))
    print("O:", ", ".join(v.hex() for v in o))
    if "--check" in sys.argv:
        d = tempfile.mkdtemp()
        src = os.path.join(d, "c.c")
        with open(src, "w") as f:
            f.write(CHECK % (", ".join(v.hex() for v in e), ", ".join(v.hex() for v in o)))
        exe = os.path.join(d, "c")
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe, src, "-lm"], check=True)
        print(subprocess.run([exe], capture_output=True, text=True, check=True).stdout.strip())


if __name__ == "__main__":
    main()
