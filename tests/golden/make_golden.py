"""Generates tests/golden/golden_<model>.npz from the CPU oracle.

Inputs per model: the edge points of apex_camera_models.samples (every status
branch) + 2000 seeded points of the bench distribution + points projected
onto / around the image border; unproject inputs: a pixel grid over and
beyond the image (bounds checks), every projected uv, and the principal point.
Outputs: oracle project (uv, status, 2N x P Jacobian) and unproject (rays,
status).  The oracle itself is pinned by tests/test_oracle.py (reference
KATs + mpmath); these vectors freeze it and travel to the GPU box, where the
HIP kernels are compared against them.
Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle as O  # noqa: E402
from test_oracle import SAMPLES  # noqa: E402

EPS = 2.220446049250313e-16
EPS_SQRT = 1.4901161193847656e-08
EDGE = np.array([
    [0.0, 0.0, 0.0], [0.1, 0.2, -1.0], [0.0, 0.0, 1e-9], [0.0, 0.0, 1.0], [0.0, 0.0, -0.0],
    [0.3, -0.2, EPS], [0.3, -0.2, EPS / 2], [0.3, -0.2, EPS_SQRT],
    [0.3, -0.2, np.nextafter(EPS_SQRT, 0.0)], [0.3, -0.2, np.nextafter(EPS_SQRT, 1.0)],
    [1e-17, 0.0, 1.0], [0.0, 1e-300, 2.0], [EPS, 0.0, 1.0], [-EPS, EPS, 1.0],
    [5.0, 5.0, 0.01], [-5.0, 3.0, -0.5], [1.0, 0.0, -1.0], [0.0, 1.0, 0.0], [1e3, -1e3, 1.0],
    [0.5, 0.0, 2.0], [-0.5, 0.0, 2.0], [0.0, 0.5, 2.0], [0.0, -0.5, 2.0], [0.1, 0.1, 3.0],
    [0.5, -0.3, 2.0], [0.1, 0.2, 1.0], [np.inf, 0.0, 1.0], [0.0, 0.0, np.inf],
    [np.nan, 0.0, 1.0], [0.0, 0.0, np.nan],
])


def make(model):
    params, (w, h) = SAMPLES[model]
    rng = np.random.default_rng(20251205 + model)
    n = 2000
    rand = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(0.5, 4.0, n)], 1)
    wide = np.stack([rng.uniform(-3, 3, 500), rng.uniform(-3, 3, 500),
                     rng.uniform(-1.0, 2.0, 500)], 1)
    xyz = np.concatenate([EDGE, rand, wide])
    uv, st, J = O.project(model, params, w, h, xyz, want_jac=True)
    gx, gy = np.meshgrid(np.linspace(-20, w + 20, 41), np.linspace(-20, h + 20, 33))
    grid = np.stack([gx.ravel(), gy.ravel()], 1)
    border = np.array([[0.0, 0.0], [w - 1e-9, h - 1e-9], [float(w), 0.0], [0.0, float(h)],
                       [-1e-300, 5.0], [params[2], params[3]], [np.nan, 1.0]])
    uv_in = np.concatenate([grid, border, uv[st == 0]])
    rays, st2 = O.unproject(model, params, w, h, uv_in)
    return dict(params=np.array(params), res=np.array([w, h]), xyz=xyz, uv=uv,
                proj_status=st, jac=J, uv_in=uv_in, rays=rays, unproj_status=st2)


if __name__ == "__main__":
    out_dir = os.path.dirname(os.path.abspath(__file__))
    for m in range(7):
        d = make(m)
        np.savez_compressed(os.path.join(out_dir, f"golden_{m}.npz"), **d)
        print(m, "proj statuses", np.bincount(d["proj_status"], minlength=5),
              "unproj statuses", np.bincount(d["unproj_status"], minlength=5))
