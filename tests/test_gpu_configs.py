"""BASELINE.json configs 3 and 5 at their own scale on the GPU, checked
against the oracle (each well under a minute):

* config 5 -- `sample_points` on the KB sample camera with n = 1e8 requested
  cells (10000 x 10000 grid, point_sampling.rs:46-120): the kept count is the
  oracle's, the kept pixels are the oracle's in the oracle's order bit for
  bit, the rays within 1e-10 (KB's atan2 / sin / cos), and a row-range shard
  of the grid is bit-equal to its slice of the full run;
* config 3 -- KB -> Double Sphere conversion (camera_converter.rs:355-488:
  linear estimation + bounded LM) on the ~9.3M KB-sampled correspondences of
  n = 1e7: at the LM's final parameters the fused normal equations have the
  oracle's n_valid exactly and its JtJ, Jtr and cost within 1e-10.
"""
import numpy as np
import pytest

import oracle as O
from _backends import rel_err

pytestmark = pytest.mark.gpu
KB, DS = 2, 3


def _kb():
    from apex_camera_models import KannalaBrandtModel, Resolution, samples
    kp, (w, h) = samples.SAMPLES[KB]
    return KannalaBrandtModel._from_params(list(kp), Resolution(w, h)), kp, w, h


def test_config5_sample_points_1e8_cells():
    import torch
    from apex_camera_models import util
    from apex_camera_models.distributed import gpu_sample_points_range, grid_row_range
    m, kp, w, h = _kb()
    n = 100_000_000
    uv, xyz = util.sample_points(m, n)
    uv0, xyz0, total = O.sample_points(KB, kp, w, h, n)
    assert total == 100_000_000
    assert uv.shape[0] == uv0.shape[0] == 92_935_075
    uv_h, xyz_h = uv.cpu().numpy(), xyz.cpu().numpy()
    assert np.array_equal(uv_h, uv0)
    assert rel_err(xyz_h, xyz0, floor=1.0) <= 1e-10
    # a row-range shard (rows 3000..3999 of 10000) equals its slice of the full run
    c0, c1 = grid_row_range(10_000, 10_000, 3, 10)
    su, sx = gpu_sample_points_range(m, n)(c0, c1)
    lo = int(np.searchsorted(uv_h[:, 1], (3000 + 0.5) * (h / 10_000)))
    k = su.shape[0]
    assert torch.equal(su, uv[lo:lo + k]) and torch.equal(sx, xyz[lo:lo + k])


def test_config3_kb_to_ds_conversion_9m():
    import torch
    from apex_camera_models import conversion, factors, util
    from apex_camera_models.camera import Resolution
    m, kp, w, h = _kb()
    uv, xyz = util.sample_points(m, 10_000_000)
    n = xyz.shape[0]
    assert n > 9_000_000
    met = conversion.convert(m, "double_sphere", xyz, uv)
    assert met.convergence_status == "Converged", met.lm_termination
    assert met.final_reprojection_error.n_valid == n
    assert met.final_reprojection_error.mean < 0.02  # README.md:163 reports 0.008 px
    p = met.model.params()
    f = factors.DoubleSphereCameraParamsFactor(xyz, uv, Resolution(w, h))
    out = torch.empty((6 * 6 + 6 + 2,), dtype=torch.float64, device="cuda")
    f.normal_equations(p, out)
    got = out.cpu().numpy()
    JtJ, Jtr, cost, nv = O.normal_equations(DS, p, w, h, xyz.cpu().numpy(), uv.cpu().numpy())
    assert int(got[-1]) == nv == n
    ref = np.concatenate([JtJ.ravel(), Jtr, [cost]])
    scale = np.maximum(np.abs(ref), np.abs(ref).max() * 1e-6)
    assert (np.abs(got[:-1] - ref) / scale).max() <= 1e-10
