"""The cell form of grid-sampled correspondences (r06).

sample_points' pixels are cell centres, ((j + 0.5) * cw, (i + 0.5) * ch)
(point_sampling.rs:56-78), so a kept point can be handed to the solver as
its cell c = i * ncx + j (4 B) instead of its pixel (16 B).  The cell forms
must give the pixel forms' results bit for bit: the cells written by every
sample_points path decode to the stored pixels exactly, the normal
equations (JtJ, Jtr, cost, n_valid) are identical, and the LM takes the
same iterates (bin/camera_converter.rs:410-420)."""
import ctypes

import numpy as np
import pytest

from test_oracle import SAMPLES

pytestmark = pytest.mark.gpu
KB = 2


def _decode(cells, grid):
    c = cells.astype(np.int64) & 0xFFFFFFFF
    i, j = c // grid.num_cells_x, c % grid.num_cells_x
    cw = float(grid.width) / float(grid.num_cells_x)
    ch = float(grid.height) / float(grid.num_cells_y)
    return np.stack([(j.astype(np.float64) + 0.5) * cw, (i.astype(np.float64) + 0.5) * ch], 1)


@pytest.mark.parametrize("model", [KB, 1, 3, 4, 5, 6, 0])
@pytest.mark.parametrize("mode", [-1, 0, 1])
def test_sample_points_cells_decode_to_the_pixels(model, mode):
    """acm_sample_points_cells: the same pixels and rays as
    acm_sample_points_ex, and cells that decode to the pixels bit for bit --
    for the segment paths that write them (auto: two-pass, RadTan's
    speculative pass) and the ones that derive them (SAMPLE_FUSED 0, 1)."""
    from apex_camera_models import _lib, util
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    names = {0: "pinhole", 1: "rad_tan", 2: "kannala_brandt", 3: "double_sphere", 4: "ucm",
             5: "eucm", 6: "fov"}
    params, (w, h) = SAMPLES[model]
    m = MODEL_CLASSES[names[model]]._from_params(params, Resolution(w, h))
    L = _lib.load()
    prev = L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, mode)
    try:
        uv0, xyz0 = util.sample_points(m, 150_000)
        uv, xyz, cs = util.sample_points(m, 150_000, cells=True)
    finally:
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, prev)
    uv0, xyz0, uv, xyz = (t.cpu().numpy() for t in (uv0, xyz0, uv, xyz))
    assert np.array_equal(uv, uv0) and np.array_equal(xyz, xyz0, equal_nan=True)
    cells = cs.cells.cpu().numpy()
    assert cells.shape[0] == uv.shape[0] > 1000
    assert np.array_equal(_decode(cells, cs.grid).view(np.int64), uv.view(np.int64))
    assert (np.diff(cells.astype(np.int64) & 0xFFFFFFFF) > 0).all()  # grid order


def _camera(mid):
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    names = {0: "pinhole", 1: "rad_tan", 2: "kannala_brandt", 3: "double_sphere", 4: "ucm",
             5: "eucm", 6: "fov"}
    params, (w, h) = SAMPLES[mid]
    p = list(params)
    p[0] *= 1.01  # off the optimum: nonzero residuals
    return MODEL_CLASSES[names[mid]]._from_params(p, Resolution(w, h)).acm_camera()


@pytest.mark.parametrize("target", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("policy", [0, 1])
def test_normal_equations_cells_bit_identical(target, policy):
    """acm_normal_equations_cells == acm_normal_equations on KB-sampled
    correspondences, every target model and both invalid-point policies:
    JtJ, Jtr, cost and n_valid bit for bit."""
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, util
    from apex_camera_models.camera import _stream_handle
    L = _lib.load()
    kp, (w, h) = SAMPLES[KB]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz, cs = util.sample_points(src, 400_003, cells=True)
    n = xyz.shape[0]
    cam = _camera(target)
    P = cam.num_params
    R = P * P + P + 2
    wsb = L.acm_normal_equations_workspace_size(target, n)
    ws = torch.empty(wsb // 8 + 1, dtype=torch.float64, device="cuda")
    a = torch.empty(R, dtype=torch.float64, device="cuda")
    b = torch.empty(R, dtype=torch.float64, device="cuda")
    _lib.check(L.acm_normal_equations(ctypes.byref(cam), n, xyz.data_ptr(), 0, uv.data_ptr(),
                                      policy, a.data_ptr(), ws.data_ptr(), wsb, _stream_handle()))
    _lib.check(L.acm_normal_equations_cells(ctypes.byref(cam), n, xyz.data_ptr(), 0,
                                            cs.cells.data_ptr(), ctypes.byref(cs.grid), policy,
                                            b.data_ptr(), ws.data_ptr(), wsb, _stream_handle()))
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int64), b.view(torch.int64))
    assert a[-1].item() > 1000  # enough valid points to mean something


@pytest.mark.parametrize("target", ["double_sphere", "kannala_brandt", "rad_tan", "ucm", "eucm",
                                    "fov"])
def test_convert_cells_same_iterates(target):
    """conversion.convert(cells=...) (the LM through acm_lm_optimize_cells)
    == convert() on the pixels: parameters, iterations and every error
    statistic bit for bit."""
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, util
    kp, (w, h) = SAMPLES[KB]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz, cs = util.sample_points(src, 60_000, cells=True)
    a = conversion.convert(src, target, xyz, uv)
    b = conversion.convert(src, target, xyz, uv, cells=cs)
    assert a.model.params() == b.model.params()
    assert (a.lm_iterations, a.lm_termination) == (b.lm_iterations, b.lm_termination)
    for fa, fb in ((a.final_reprojection_error, b.final_reprojection_error),
                   (a.initial_reprojection_error, b.initial_reprojection_error)):
        for k in ("rmse", "min", "max", "mean", "stddev", "median", "n_valid"):
            va, vb = getattr(fa, k), getattr(fb, k)
            assert va == vb or (va != va and vb != vb), (k, va, vb)


def test_sharded_cells_world1_is_the_1gpu_path():
    """The sharded entry points with the cell form at world 1 (local
    collective): the 1-GPU pixel path's bits."""
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, util
    from apex_camera_models.distributed import LocalCollective
    kp, (w, h) = SAMPLES[KB]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz, cs = util.sample_points(src, 60_000, cells=True)
    a = conversion.convert(src, "double_sphere", xyz, uv)
    b = conversion.convert(src, "double_sphere", xyz, uv, collective=LocalCollective(), cells=cs)
    assert a.model.params() == b.model.params()
    assert a.final_reprojection_error == b.final_reprojection_error
    assert a.initial_reprojection_error == b.initial_reprojection_error


def test_cell_form_argument_checks():
    import torch
    from apex_camera_models import _lib
    from apex_camera_models.camera import _stream_handle
    L = _lib.load()
    cam = _camera(3)
    ws = torch.empty(1 << 16, dtype=torch.float64, device="cuda")
    out = torch.empty(64, dtype=torch.float64, device="cuda")
    pts = torch.zeros((4, 3), dtype=torch.float64, device="cuda")
    cells = torch.zeros(4, dtype=torch.int32, device="cuda")
    for g in (_lib.CellGrid(0, 5, 512, 512), _lib.CellGrid(70000, 70000, 512, 512),
              _lib.CellGrid(5, 5, 0, 512)):
        rc = L.acm_normal_equations_cells(ctypes.byref(cam), 4, pts.data_ptr(), 0,
                                          cells.data_ptr(), ctypes.byref(g), 0, out.data_ptr(),
                                          ws.data_ptr(), ws.numel() * 8, _stream_handle())
        assert rc == _lib.ERR_INVALID_ARGUMENT
    assert L.acm_normal_equations_cells(ctypes.byref(cam), 4, pts.data_ptr(), 0, None,
                                        ctypes.byref(_lib.CellGrid(5, 5, 512, 512)), 0,
                                        out.data_ptr(), ws.data_ptr(), ws.numel() * 8,
                                        _stream_handle()) == _lib.ERR_INVALID_ARGUMENT
