"""BASELINE.json configs 3, 4 and 5 at their own scale on the GPU, checked
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


@pytest.mark.parametrize("model", range(6))
def test_config4_round_trip_6_25m(model):
    """BASELINE config 4 at its own per-GPU size: the project -> unproject
    round trip of 6.25M synthetic points (the bench distribution, 0.1% edge
    points) for each of the six north-star models, through the fused entry
    the bench leg times (acm_project_unproject).  On a strided 200k
    subsample both statuses are bit-exact against the oracle's project
    followed by its unproject of its own pixels, uv / rays within 1e-10,
    values bit-exact for the models without a transcendental
    (test_gpu_parity.check_round_trip_vs_oracle); over all 6.25M points the
    round trip preserves the direction the way
    tests/projection_accuracy.rs:49-74 asserts (|dot - 1| < 1e-6) -- except
    UCM, whose reference unprojection keeps the 1 - r^2 quirk (ucm.rs:354):
    there the GPU round trip equals the oracle's on the subsample instead."""
    import torch
    from apex_camera_models import samples
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    from test_gpu_parity import check_round_trip_vs_oracle
    names = {0: "pinhole", 1: "rad_tan", 2: "kannala_brandt", 3: "double_sphere", 4: "ucm",
             5: "eucm"}
    n = 6_250_000
    params, (w, h) = samples.SAMPLES[model]
    m = MODEL_CLASSES[names[model]]._from_params(list(params), Resolution(w, h))
    # rank 3's shard of config 4's 50M-point global batch, as the bench leg slices it
    lo = 3 * n
    pts = samples.synthetic_points_device(8 * n)[lo:lo + n].contiguous()
    uv, st, ray, st2 = m.project_unproject_batch(pts)
    torch.cuda.synchronize()
    sub = torch.arange(0, n, n // 200_000, device="cuda")
    check_round_trip_vs_oracle(model, params, w, h, pts[sub].cpu().numpy(),
                               uv[sub].cpu().numpy(), st[sub].cpu().numpy(),
                               ray[sub].cpu().numpy(), st2[sub].cpu().numpy())
    ok = (st == 0) & (st2 == 0) & torch.isfinite(pts).all(1)
    assert int(ok.sum()) > 0.8 * n
    pn = pts[ok] / torch.linalg.norm(pts[ok], dim=1, keepdim=True)
    dot = (pn * ray[ok]).sum(1)
    if model == 4:
        assert float((dot - 1).abs().max()) > 1e-6  # the quirk is there, as in the oracle
    else:
        assert float((dot - 1).abs().max()) < 1e-6


def test_config5_kb_to_ds_on_92_9m_correspondences():
    """BASELINE config 5 at its own size: the KB sample camera's 1e8-cell
    sample_points (92,935,075 correspondences) -> Double Sphere conversion
    (camera_converter.rs:355-488: linear estimation + bounded LM, all on the
    GPU).  At the final parameters the fused normal equations over all
    92.9M points have the oracle's n_valid exactly, and on a strided 1M
    subsample the GPU's JtJ / Jtr / cost equal the oracle's within 1e-10.
    Then the config's f32-vs-f64 sweep over all 92.9M points."""
    import torch
    from apex_camera_models import conversion, factors, util
    from apex_camera_models.camera import Resolution
    m, kp, w, h = _kb()
    uv, xyz, cs = util.sample_points(m, 100_000_000, cells=True)
    n = xyz.shape[0]
    assert n == 92_935_075
    met = conversion.convert(m, "double_sphere", xyz, uv, cells=cs)
    assert met.convergence_status == "Converged", met.lm_termination
    # (r06) the cell form at scale: the fused normal equations from the 4-B
    # cells equal the pixel form's over all 92.9M points, bit for bit
    import ctypes
    from apex_camera_models import _lib
    from apex_camera_models.camera import _stream_handle
    L = _lib.load()
    cam = met.model.acm_camera()
    wsb = L.acm_normal_equations_workspace_size(DS, n)
    ws = torch.empty(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    a = torch.empty(44, dtype=torch.float64, device="cuda")
    b = torch.empty(44, dtype=torch.float64, device="cuda")
    _lib.check(L.acm_normal_equations(ctypes.byref(cam), n, xyz.data_ptr(), 0, uv.data_ptr(), 0,
                                      a.data_ptr(), ws.data_ptr(), wsb, _stream_handle()))
    _lib.check(L.acm_normal_equations_cells(ctypes.byref(cam), n, xyz.data_ptr(), 0,
                                            cs.cells.data_ptr(), ctypes.byref(cs.grid), 0,
                                            b.data_ptr(), ws.data_ptr(), wsb, _stream_handle()))
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int64), b.view(torch.int64))
    del ws, cs
    assert met.final_reprojection_error.n_valid == n
    assert met.final_reprojection_error.mean < 0.02  # README.md:163 reports 0.008 px
    p = met.model.params()
    out = torch.empty((6 * 6 + 6 + 2,), dtype=torch.float64, device="cuda")
    factors.DoubleSphereCameraParamsFactor(xyz, uv, Resolution(w, h)).normal_equations(p, out)
    nv_all = int(out[-1].item())
    # the oracle's n_valid over all 92.9M (DS projection status only)
    _, st0, _ = O.project(DS, p, w, h, xyz.cpu().numpy())
    assert nv_all == int((st0 == 0).sum()) == n
    sub = torch.arange(0, n, 93, device="cuda")
    xs, us = xyz[sub].contiguous(), uv[sub].contiguous()
    factors.DoubleSphereCameraParamsFactor(xs, us, Resolution(w, h)).normal_equations(p, out)
    got = out.cpu().numpy()
    JtJ, Jtr, cost, nv = O.normal_equations(DS, p, w, h, xs.cpu().numpy(), us.cpu().numpy())
    assert int(got[-1]) == nv == len(sub)
    ref = np.concatenate([JtJ.ravel(), Jtr, [cost]])
    scale = np.maximum(np.abs(ref), np.abs(ref).max() * 1e-6)
    assert (np.abs(got[:-1] - ref) / scale).max() <= 1e-10
    # BASELINE config 5's f32-vs-f64 tolerance sweep at scale: the DS
    # projection at the optimum over all 92.9M correspondences in f32
    # (acm_project_f32) agrees with the f64 path on every status, and its
    # pixels are within 1e-4 relative (floor 1 px; measured 7.5e-5)
    ds = met.model
    uv64, st64, _ = ds.project_batch(xyz)
    uv32, st32, _ = ds.project_batch(xyz.to(torch.float32))
    assert uv32.dtype == torch.float32
    assert int((st64 != st32).sum()) == 0
    both = (st64 == 0) & (st32 == 0)
    d = ((uv32.double() - uv64).abs() / uv64.abs().clamp(min=1.0)).max(dim=1).values
    worst = float(torch.where(both, d, torch.zeros_like(d)).max())
    assert 0.0 < worst < 1e-4, worst
