"""CPU check of RadTan's host-certified Newton disk (acm.hip
radtan_newton_disk, exposed as acm_unproject_certificate): on the disk
x^2 + y^2 <= S the fast loop tests only s <= S per step, because the host
claims |det J| >= 1/16 and |j00| + |j11| + 2 |j01| <= 64 for every point of
it -- the conditions the fast loop's error analysis needs (camera_models.hpp
RadTan::newton_fast).  The claim is checked here on dense polar samples of
the disk (the edge included), with the Jacobian written as the reference
writes it (rad_tan.rs:470-491), for the reference's sample camera
(samples/rad_tan.yaml), the stress cameras of the GPU tests and a sweep of
random distortions.  The host code runs without a GPU."""
import ctypes
import os

import numpy as np
import pytest

from apex_camera_models import _lib

pytestmark = pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libacm.so not built")

RT_SAMPLE = [461.629, 460.152, 362.680, 246.049, -0.28340811, 0.07395907, 0.00019359,
             1.76187114e-05, 0.0]  # samples/rad_tan.yaml


def disk(params):
    L = _lib.load()
    cam = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam), 1, (ctypes.c_double * 9)(*params), 9,
                                 752, 480))
    out = (ctypes.c_double * 2)()
    _lib.check(L.acm_unproject_certificate(ctypes.byref(cam), out))
    return out[0], out[1]


def jac_ok(params, S, n_r=400, n_phi=720):
    k1, k2, p1, p2, k3 = params[4:]
    r = np.sqrt(S) * np.concatenate([np.linspace(0, 1, n_r), [1.0]])
    phi = np.linspace(0, 2 * np.pi, n_phi, endpoint=False)
    R, PH = np.meshgrid(r, phi)
    x, y = R * np.cos(PH), R * np.sin(PH)
    r2 = x * x + y * y
    r4 = r2 * r2
    rad = 1 + k1 * r2 + k2 * r4 + k3 * r4 * r2
    drdx, drdy = 2 * x, 2 * y
    dd = k1 + 2 * k2 * r2 + 3 * k3 * r4
    j00 = rad + x * dd * drdx + 2 * p1 * y + p2 * (drdx + 4 * x)
    j01 = x * dd * drdy + 2 * p1 * x + p2 * drdy
    j10 = y * dd * drdx + p1 * drdx + 2 * p2 * y
    j11 = rad + y * dd * drdy + p1 * (drdy + 4 * y) + 2 * p2 * x
    det = j00 * j11 - j10 * j01
    sj = np.abs(j00) + np.abs(j11) + np.abs(j01) + np.abs(j10)
    return float(np.abs(det).min()), float(sj.max())


def _check(params):
    S, fast = disk(params)
    if S == 0.0:
        return False
    assert 0 < S <= 4.0
    dmin, smax = jac_ok(params, S * (1 + 1e-6))
    assert dmin >= 1 / 16, (params, S, dmin)
    assert smax <= 64, (params, S, smax)
    return True


def test_sample_camera_disk():
    S, fast = disk(RT_SAMPLE)
    assert fast == 1.0
    # the config-4 pixels of the sample camera reach s ~ 1.3 (image corners)
    assert S >= 1.3, S
    assert _check(RT_SAMPLE)


@pytest.mark.parametrize("params", [
    [461.629, 460.152, 362.680, 246.049, -0.45, 0.12, 0.003, -0.002, -0.005],
    [461.629, 460.152, 362.680, 246.049, 0.3, -0.05, 0.01, 0.01, 0.002],
    [461.629, 460.152, 362.680, 246.049, -0.6, 0.45, 0.003, -0.002, -0.1],
])
def test_stress_cameras(params):
    _check(params)


def test_random_cameras():
    rng = np.random.default_rng(5)
    certified = 0
    for _ in range(60):
        k = [rng.uniform(-0.5, 0.5), rng.uniform(-0.2, 0.2), rng.uniform(-0.02, 0.02),
             rng.uniform(-0.02, 0.02), rng.uniform(-0.05, 0.05)]
        certified += _check(RT_SAMPLE[:4] + k)
    assert certified >= 30, certified


def test_other_models_have_no_disk():
    L = _lib.load()
    cam = _lib.AcmCamera()
    p = RT_SAMPLE[:4] + [0.0] * 4
    _lib.check(L.acm_camera_init(ctypes.byref(cam), 2, (ctypes.c_double * 8)(*p), 8, 512, 512))
    out = (ctypes.c_double * 2)(7.0, 7.0)
    _lib.check(L.acm_unproject_certificate(ctypes.byref(cam), out))
    assert list(out) == [0.0, 0.0]
