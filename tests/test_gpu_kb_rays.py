"""Kannala-Brandt sample_points on random cameras against the oracle (the
reference's own Newton loop per cell, point_sampling.rs:46-120 +
kannala_brandt.rs:445-562), covering every way the kernels form the ray of a
cell inside the host-certified kept interval (acm_sample_points_ray_fit):
mode 3 (the ray polynomials) including draws whose fit-error bound lands
near the 1e-13 gate, mode 2 (fitted guess + two Newton steps), and cameras
whose root-vs-iterate bound ef exceeds 1e-11, so the certified rays are off
and every cell takes the reference-iterate path.  Kept sets and
pixels bit-exact, rays within 1e-10."""
import ctypes

import numpy as np
import pytest

import oracle as O
from _backends import rel_err

pytestmark = pytest.mark.gpu
KB = 2


def _fit(params, w, h):
    from apex_camera_models import _lib
    L = _lib.load()
    cam = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam), KB, (ctypes.c_double * 8)(*params), 8, w, h))
    fit = (ctypes.c_double * 6)()
    _lib.check(L.acm_sample_points_ray_fit(ctypes.byref(cam), fit))
    cert = (ctypes.c_double * 5)()
    _lib.check(L.acm_sample_points_certificate(ctypes.byref(cam), cert))
    return list(fit), list(cert)


def _pick_cameras(w, h):
    """A seeded draw, sorted into the cases above (host-side fits only)."""
    rng = np.random.default_rng(2024)
    near_gate, mode2, ef_off, plain = [], [], [], []
    for _ in range(400):
        scale = rng.choice([0.05, 0.2])
        dist = list(rng.normal(0, [scale, scale * 0.5, scale * 0.2, scale * 0.05]))
        p = [200.0, 200.0, w / 2, h / 2] + dist
        (mode, M, ef, err, lo, hi), cert = _fit(p, w, h)
        if mode == 3 and 1e-14 < err <= 1e-13 and len(near_gate) < 3:
            near_gate.append(p)
        elif mode == 2 and len(mode2) < 2:
            mode2.append(p)
        elif mode == 0 and cert[0] == 1 and ef > 1e-11 and len(ef_off) < 2:
            ef_off.append(p)
        elif mode == 3 and len(plain) < 2:
            plain.append(p)
    return near_gate, mode2, ef_off, plain


def test_random_kb_cameras_sample_points_vs_oracle():
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, util
    w, h = 512, 512
    near_gate, mode2, ef_off, plain = _pick_cameras(w, h)
    assert len(near_gate) >= 2 and len(ef_off) >= 1 and len(plain) >= 1, \
        (len(near_gate), len(mode2), len(ef_off), len(plain))
    n = 250_000
    for p in near_gate + mode2 + ef_off + plain:
        m = KannalaBrandtModel._from_params(p, Resolution(w, h))
        uv, xyz = util.sample_points(m, n)
        torch.cuda.synchronize()
        uv0, xyz0, total = O.sample_points(KB, p, w, h, n)
        uv_h, xyz_h = uv.cpu().numpy(), xyz.cpu().numpy()
        assert uv_h.shape == uv0.shape, (p, uv_h.shape, uv0.shape)
        assert np.array_equal(uv_h, uv0), p
        assert rel_err(xyz_h, xyz0, floor=1.0) <= 1e-10, (p, rel_err(xyz_h, xyz0, floor=1.0))
