"""undistort_image (src/util/undistort.rs:14-105) on the GPU vs the oracle,
every model, nearest and bilinear, own and custom target intrinsics:
byte-identical images.

The output bytes quantise the projected source coordinate with round() /
floor() (undistort.rs:61, :70, :100), so k_undistort projects with the
reference-exact math (camera_models.hpp EXACT: IEEE sqrt / divisions, and for
KB / FOV the correctly rounded atan2 of exact_math.hpp, which equals glibc's
wherever glibc is correctly rounded -- tests/test_gpu_exact.py).  On a
mismatch the test lists every differing pixel with both source coordinates
and whether glibc misrounded its atan2 argument."""
import numpy as np
import pytest

import oracle as O
from test_oracle import SAMPLES

pytestmark = pytest.mark.gpu


def _source_coords(model, params, w, h, tvec, be, pix):
    """oracle and GPU-EXACT source coordinates of output pixels pix (k, 2)"""
    import torch
    u, v = pix[:, 1].astype(np.float64), pix[:, 0].astype(np.float64)
    rays = np.stack([(u - tvec[2]) / tvec[0], (v - tvec[3]) / tvec[1], np.ones_like(u)], 1)
    uv0, st0, _ = O.project(model, params, w, h, rays)
    m = be._model(model, params, w, h)
    uv, st, _ = m.project_batch(torch.as_tensor(rays, device="cuda"), exact=True)
    return uv0, st0, uv.cpu().numpy(), st.cpu().numpy()


@pytest.mark.parametrize("bilinear", [0, 1])
@pytest.mark.parametrize("target_scale", [None, 0.5])
@pytest.mark.parametrize("model", range(7))
def test_undistort_vs_oracle(model, bilinear, target_scale):
    import torch
    from apex_camera_models import util
    from apex_camera_models.camera import Intrinsics
    from _backends import GpuBackend
    params, (w, h) = SAMPLES[model]
    rng = np.random.default_rng(model)
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    be = GpuBackend()
    m = be._model(model, params, w, h)
    target = None
    tvec = params[:4]
    if target_scale is not None:
        tvec = [params[0] * target_scale, params[1] * target_scale, params[2], params[3]]
        target = Intrinsics(*tvec)
    out = util.undistort_image(torch.as_tensor(img), m, target, bilinear).cpu().numpy()
    ref = O.undistort_image(model, params, w, h, tvec, bilinear, img)
    if not np.array_equal(out, ref):
        pix = np.argwhere((out != ref).any(axis=2))
        uv0, st0, uv, st = _source_coords(model, params, w, h, tvec, be, pix)
        rows = [f"(v={p[0]}, u={p[1]}) ref src {a.tolist()} st {s0}, gpu src {b.tolist()} st {s1}, "
                f"bytes ref {ref[p[0], p[1]].tolist()} gpu {out[p[0], p[1]].tolist()}"
                for p, a, b, s0, s1 in zip(pix[:20], uv0, uv, st0, st)]
        pytest.fail(f"{len(pix)} pixels differ:\n" + "\n".join(rows))


def test_undistort_source_coordinates_exact(golden_dir):
    """The source coordinate of every output pixel of the KB and FOV sample
    cameras (the only models with a transcendental): GPU EXACT projection vs
    oracle, bit for bit except at glibc atan2 misroundings (listed)."""
    from _backends import GpuBackend
    from test_gpu_exact import atan2_args, glibc_misrounds
    be = GpuBackend()
    for model in (2, 6):
        params, (w, h) = SAMPLES[model]
        for tvec in (params[:4], [params[0] * 0.5, params[1] * 0.5, params[2], params[3]]):
            pix = np.argwhere(np.ones((h, w), dtype=bool))
            uv0, st0, uv, st = _source_coords(model, params, w, h, tvec, be, pix)
            assert np.array_equal(st0, st)
            diff = np.nonzero(~((uv == uv0) | (np.isnan(uv) & np.isnan(uv0))).all(1))[0]
            rays = np.stack([(pix[diff, 1] - tvec[2]) / tvec[0], (pix[diff, 0] - tvec[3]) / tvec[1],
                             np.ones(len(diff))], 1)
            ya, xa = atan2_args(model, params, rays)
            assert all(glibc_misrounds(a, b) for a, b in zip(ya, xa)), diff[:10]
            assert len(diff) <= 0.005 * len(pix)


def test_undistort_rejects_mismatched_image():
    import torch
    from apex_camera_models import util
    from _backends import GpuBackend
    params, (w, h) = SAMPLES[3]
    m = GpuBackend()._model(3, params, w, h)
    with pytest.raises(util.UtilError):
        util.undistort_image(torch.zeros((10, 10, 3), dtype=torch.uint8), m)
