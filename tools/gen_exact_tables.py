"""Prints the double-double constant tables of csrc/exact_math.hpp (mpmath,
300-bit working precision): atan(k/64) for k = 0..64, the alternating odd
reciprocals (-1)^n / (2n+1) of the atan series, and pi/2.  Each value v is
stored as (hi, lo) with hi = RN(v), lo = RN(v - hi).

  python tools/gen_exact_tables.py
"""
import mpmath

mpmath.mp.prec = 300


def dd(x):
    hi = float(x)
    return hi, float(x - mpmath.mpf(hi))


def fmt(v):
    return f"{{{v[0].hex()}, {v[1].hex()}}}"


def main():
    tab = [fmt(dd(mpmath.atan(mpmath.mpf(k) / 64))) for k in range(65)]
    print("kAtanK64[65][2] = {")
    for i in range(0, 65, 2):
        print("    " + ", ".join(tab[i:i + 2]) + ",")
    print("};")
    print("kAtanSeries[8][2] = {")
    for n in range(8):
        print("    " + fmt(dd((-1) ** n / mpmath.mpf(2 * n + 1))) + ",")
    print("};")
    print("kPiHalf = " + fmt(dd(mpmath.pi / 2)))


if __name__ == "__main__":
    main()
