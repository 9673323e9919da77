"""Host check of the double-double atan2 (csrc/exact_math.hpp atan2_cr) that
the reference-exact KB / FOV projections use (undistort_image, acm_project
with ACM_EXACT_MATH): against 300-bit mpmath it must be the correctly
rounded atan2 on every argument tried, and where glibc's atan2 (the libm the
reference calls, kannala_brandt.rs:365, fov.rs:298) differs from it, glibc is
the one that misrounds (it is correctly rounded on ~99.8% of arguments)."""
import os
import subprocess

import mpmath
import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "apex-camera-models_amd", "csrc")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    d = tmp_path_factory.mktemp("xm")
    exe = str(d / "exact_math_driver")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-DACM_HD=", "-I", CSRC,
                    os.path.join(ROOT, "tests", "exact_math_driver.cpp"), "-o", exe], check=True)

    def run(y, x):
        inp, out = str(d / "in.bin"), str(d / "out.bin")
        np.stack([y, x], 1).astype(np.float64).tofile(inp)
        subprocess.run([exe, inp, out], check=True)
        r = np.fromfile(out, dtype=np.float64).reshape(-1, 2)
        return r[:, 0], r[:, 1]
    return run


def cr_atan2(y, x):
    with mpmath.workprec(300):
        return float(mpmath.atan2(mpmath.mpf(float(y)), mpmath.mpf(float(x))))


def adversarial():
    rng = np.random.default_rng(7)
    ys, xs = [], []
    # ratios on and next to the table nodes k/64 and the swap boundary y = x
    for k in range(65):
        for d in (-3, -1, 0, 1, 3):
            x = rng.uniform(0.5, 4.0, 8)
            q = np.nextafter(k / 64.0, 2.0) if d > 0 else k / 64.0
            q = q + d * 2.0 ** -52 * max(k / 64.0, 2.0 ** -40)
            ys.append(np.clip(q, 0, 1) * x)
            xs.append(x)
    x = rng.uniform(0.5, 4.0, 2000)
    ys += [x, np.nextafter(x, 0), np.nextafter(x, 10)]
    xs += [x, x, x]
    # tiny and huge radii / depths (KB axis neighbourhood, far points)
    e = rng.uniform(-60, 60, 4000)
    ys.append(2.0 ** e)
    xs.append(rng.uniform(0.5, 4.0, 4000))
    ys.append(rng.uniform(0.5, 4.0, 2000))
    xs.append(2.0 ** rng.uniform(-60, 60, 2000))
    ys.append(np.array([2.0 ** -1000, 2.0 ** -1074, 1e300, 1e-300, 5e-324, 1.0, 1e308]))
    xs.append(np.array([1.0, 1.0, 1e-300, 1e300, 1.0, 5e-324, 1e-308]))
    return np.concatenate(ys), np.concatenate(xs)


def test_atan2_cr_is_correctly_rounded(driver):
    rng = np.random.default_rng(20251205)
    y1, x1 = adversarial()
    n = 20000
    y2 = np.abs(rng.uniform(-2, 2, n)) * rng.uniform(0, 1, n) ** 2
    x2 = rng.uniform(1e-3, 4.0, n)
    y = np.concatenate([y1, y2])
    x = np.concatenate([x1, x2])
    cr, _ = driver(y, x)
    bad = [(a, b, c) for a, b, c in zip(y, x, cr) if c != cr_atan2(a, b)]
    assert not bad, bad[:10]


def test_glibc_disagreements_are_glibc_misroundings(driver):
    """2M bench-distribution arguments (KB: atan2(r, z), r = |(x, y)|,
    x, y ~ U[-1, 1), z ~ U[0.5, 4)): every point where glibc and atan2_cr
    differ is one where glibc is not correctly rounded."""
    rng = np.random.default_rng(11)
    n = 2_000_000
    r = np.hypot(rng.uniform(-1, 1, n), rng.uniform(-1, 1, n))
    z = rng.uniform(0.5, 4.0, n)
    cr, gl = driver(r, z)
    idx = np.nonzero(cr != gl)[0]
    assert len(idx) < 0.005 * n, len(idx)
    for i in idx:
        exact = cr_atan2(r[i], z[i])
        assert cr[i] == exact, (r[i], z[i])
        assert abs(gl[i] - exact) <= np.spacing(exact), (r[i], z[i])


def test_atan2_cr_domain(driver):
    y = np.array([0.0, 1.0, -1.0, 1.0, np.inf, 1.0, np.nan, 0.0])
    x = np.array([1.0, 0.0, 1.0, -1.0, 1.0, np.inf, 1.0, 1e-300])
    cr, _ = driver(y, x)
    assert cr[0] == 0.0 and cr[7] == 0.0
    assert np.isnan(cr[1:7]).all()
