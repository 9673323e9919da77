"""undistort_image (src/util/undistort.rs:14-105) on the GPU vs the oracle,
every model, nearest and bilinear, own and custom target intrinsics.
Bit-exact for the models without transcendentals; KB/FOV projections can
differ from glibc by ulps, which may flip a rounding boundary: at most a
handful of pixels, each by at most one intensity level / one source pixel."""
import numpy as np
import pytest

import oracle as O
from test_oracle import SAMPLES

pytestmark = pytest.mark.gpu


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
    m = GpuBackend()._model(model, params, w, h)
    target = None
    tvec = params[:4]
    if target_scale is not None:
        tvec = [params[0] * target_scale, params[1] * target_scale, params[2], params[3]]
        target = Intrinsics(*tvec)
    out = util.undistort_image(torch.as_tensor(img), m, target, bilinear).cpu().numpy()
    ref = O.undistort_image(model, params, w, h, tvec, bilinear, img)
    diff = np.abs(out.astype(int) - ref.astype(int))
    if model in (2, 6):
        bad = (diff.max(axis=2) > 0).sum()
        assert bad <= 10, bad
        if not bilinear:
            return
        assert diff.max() <= 1
    else:
        assert np.array_equal(out, ref), int((diff > 0).sum())


def test_undistort_rejects_mismatched_image():
    import torch
    from apex_camera_models import util
    from _backends import GpuBackend
    params, (w, h) = SAMPLES[3]
    m = GpuBackend()._model(3, params, w, h)
    with pytest.raises(util.UtilError):
        util.undistort_image(torch.zeros((10, 10, 3), dtype=torch.uint8), m)
