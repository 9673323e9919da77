"""Mirror of the reference's hot-path utilities (src/util/).

`sample_points` (point_sampling.rs:46-120) and `compute_reprojection_error`
(error_metrics.rs:62-121), both evaluated by libacm.so kernels on device
tensors.
"""
from __future__ import annotations

import ctypes
import dataclasses
from dataclasses import dataclass

import torch

from . import _lib
from .camera import CameraModel, InvalidParams, NumericalError, _as_device_f64, _stream_handle


class UtilError(Exception):
    pass


class ZeroProjectionPoints(UtilError):
    def __init__(self):
        super().__init__("Zero projection points")


@dataclass
class ProjectionError:
    rmse: float
    min: float
    max: float
    mean: float
    stddev: float
    median: float
    n_valid: int = 0


@dataclass
class CellSample:
    """The cell form of grid-sampled correspondences (r06): cells[k] = i * ncx
    + j is the grid cell of points_2d[k] (point_sampling.rs:56-78), a uint32
    instead of the 16-B pixel -- what conversion.convert(cells=...) hands the
    LM (acm_lm_optimize_cells: the same iterates, 12 B per point less read per
    evaluation)."""
    cells: torch.Tensor  # (M,) int32 device tensor holding the uint32 cell ids
    grid: object         # _lib.CellGrid


def sample_points(camera_model: CameraModel, n: int, reference_newton: bool = False,
                  cells: bool = False, cell_range=None):
    """Grid of ~n pixel-cell centres, unprojected; keeps Ok && z > 0, in order.

    Returns (points_2d (M,2), points_3d (M,3)) float64 device tensors, and
    with cells=True a third item, the CellSample of the same points.
    reference_newton=True: ACM_REFERENCE_NEWTON for this call.  cell_range:
    (begin, end) cells of the grid (a multi-GPU shard), default all.
    """
    L = _lib.load()
    cam = camera_model.acm_camera()
    ncx, ncy = ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(L.acm_sample_points_grid(cam.width, cam.height, n, ctypes.byref(ncx),
                                        ctypes.byref(ncy)))
    c0, c1 = cell_range if cell_range is not None else (0, ncx.value * ncy.value)
    cap = max(c1 - c0, 1)
    dev = torch.device("cuda")
    uv = torch.empty((cap, 2), dtype=torch.float64, device=dev)
    xyz = torch.empty((cap, 3), dtype=torch.float64, device=dev)
    counts = torch.zeros((2,), dtype=torch.int64, device=dev)
    ws_bytes = L.acm_sample_points_workspace_size(ctypes.byref(cam), n)
    ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=dev)
    flags = _lib.REFERENCE_NEWTON if reference_newton else 0
    cl = None
    if cells:
        cl = torch.empty((cap,), dtype=torch.int32, device=dev)
        _lib.check(L.acm_sample_points_cells(ctypes.byref(cam), n, c0, c1, flags, uv.data_ptr(),
                                             xyz.data_ptr(), cl.data_ptr(), counts.data_ptr(),
                                             ws.data_ptr(), ws_bytes, _stream_handle()))
    else:
        _lib.check(L.acm_sample_points_ex(ctypes.byref(cam), n, c0, c1, flags, uv.data_ptr(),
                                          xyz.data_ptr(), counts.data_ptr(), ws.data_ptr(),
                                          ws_bytes, _stream_handle()))
    m = int(counts[0].item())
    if cells:
        grid = _lib.CellGrid(ncx.value, ncy.value, cam.width, cam.height)
        return uv[:m], xyz[:m], CellSample(cl[:m], grid)
    return uv[:m], xyz[:m]


def reprojection_stats(camera_model: CameraModel, points3d, points2d, errors=None):
    """Device result [rmse, min, max, mean, stddev, n_valid, sum, sumsq]."""
    L = _lib.load()
    p3 = _as_device_f64(points3d, 3)
    p2 = _as_device_f64(points2d, 2)
    n = p3.shape[0]
    if p2.shape[0] != n:
        raise ValueError("points3d and points2d must have the same number of columns")
    ws_bytes = L.acm_reprojection_stats_workspace_size(n)
    ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=p3.device)
    out = torch.empty((8,), dtype=torch.float64, device=p3.device)
    cam = camera_model.acm_camera()
    _lib.check(L.acm_reprojection_stats(ctypes.byref(cam), n, p3.data_ptr(), _lib.LAYOUT_AOS,
                                        p2.data_ptr(), out.data_ptr(),
                                        errors.data_ptr() if errors is not None else None,
                                        ws.data_ptr(), ws_bytes, _stream_handle()))
    return out


def compute_reprojection_error(camera_model: CameraModel, points3d, points2d,
                               collective=None, cells=None) -> ProjectionError:
    """error_metrics.rs:62-121: one acm_reprojection_error call (the
    statistics and the median, whose first radix histogram the statistics
    pass counts) and one device -> host read of its 9 doubles.

    collective (distributed.RcclCollective / TorchCollective, r06): the
    points are this rank's shard, and the result is the union's
    (acm_reprojection_error_sharded), the same on every rank.  cells (r06):
    the CellSample of points2d -- the pass reads the 4-B cells (same bits)."""
    L = _lib.load()
    p3 = _as_device_f64(points3d, 3)
    p2 = _as_device_f64(points2d, 2)
    n = p3.shape[0]
    if p2.shape[0] != n:
        raise ValueError("points3d and points2d must have the same number of columns")
    res = torch.empty((9,), dtype=torch.float64, device=p3.device)
    cam = camera_model.acm_camera()
    cl, grid = _cell_args(cells, n)
    if collective is not None:
        ws_bytes = L.acm_reprojection_error_sharded_workspace_size(n, collective.c.world)
        ws = _workspace(ws_bytes, p3.device)
        _lib.check(L.acm_reprojection_error_sharded(
            ctypes.byref(cam), n, p3.data_ptr() if n else None, _lib.LAYOUT_AOS,
            p2.data_ptr() if n else None, cl, grid, res.data_ptr(), None,
            ctypes.byref(collective.c), ws.data_ptr(), ws_bytes, _stream_handle()))
    elif cells is not None:
        ws_bytes = L.acm_reprojection_error_workspace_size(n)
        ws = _workspace(ws_bytes, p3.device)
        _lib.check(L.acm_reprojection_error_cells(ctypes.byref(cam), n, p3.data_ptr(),
                                                  _lib.LAYOUT_AOS, cl, grid, res.data_ptr(), None,
                                                  ws.data_ptr(), ws_bytes, _stream_handle()))
    else:
        ws_bytes = L.acm_reprojection_error_workspace_size(n)
        ws = _workspace(ws_bytes, p3.device)
        _lib.check(L.acm_reprojection_error(ctypes.byref(cam), n, p3.data_ptr(), _lib.LAYOUT_AOS,
                                            p2.data_ptr(), res.data_ptr(), None, ws.data_ptr(),
                                            ws_bytes, _stream_handle()))
    out = res.cpu().tolist()
    n_valid = int(out[5])
    if n_valid == 0:
        raise ZeroProjectionPoints()
    return ProjectionError(rmse=out[0], min=out[1], max=out[2], mean=out[3], stddev=out[4],
                           median=out[8], n_valid=n_valid)


def _workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(((nbytes + 7) // 8,), dtype=torch.float64, device=device)


def _cell_args(cells, n):
    """(cells pointer, grid reference) for the C-ABI's nullable cell-form
    arguments (None, None without a CellSample)."""
    if cells is None:
        return None, None
    if cells.cells.shape[0] != n:
        raise ValueError("cells and points_3d must have the same number of points")
    return (cells.cells.data_ptr() if n else None), ctypes.byref(cells.grid)


def initial_error_and_linear_estimation(model: CameraModel, points3d, points2d,
                                        defer_median: bool = False, collective=None,
                                        cells=None):
    """convert_to_*'s opening (camera_converter.rs:371-375): the reprojection
    error of `model` as given, then `model.linear_estimation` -- for the TSQR
    models one pass over the correspondences (acm_linear_estimation_with_error_async).
    Raises like the two calls in that order: ZeroProjectionPoints first, then
    the estimation's InvalidParams / NumericalError.

    defer_median=True (conversion.convert, r05): returns (error, finish) at
    once, `error.median` NaN; the median is still running on the stream and
    finish() returns the completed ProjectionError -- call it after the next
    synchronising step (the LM), so no host round trip separates the opening
    from the LM's first evaluation.

    collective (r06): the points are this rank's shard and everything is
    over the union (acm_linear_estimation_with_error_sharded: one all-gather
    of each rank's factor and statistics, the distributed median); every
    rank gets the same model.  cells (r06): the CellSample of points2d --
    the fused pass reads the 4-B cells (same bits)."""
    L = _lib.load()
    p3 = _as_device_f64(points3d, 3)
    p2 = _as_device_f64(points2d, 2)
    n = p3.shape[0]
    if p2.shape[0] != n:  # as linear_estimation raises it (kannala_brandt.rs:168-172 & co)
        raise InvalidParams("Number of 2D and 3D points must match")
    if collective is not None:
        ws_bytes = L.acm_linear_estimation_with_error_sharded_workspace_size(
            model.MODEL_ID, n, collective.c.world)
    else:
        ws_bytes = L.acm_linear_estimation_with_error_workspace_size(model.MODEL_ID, n)
    if ws_bytes == 0:
        raise InvalidParams(f"{model.NAME} has no GPU linear_estimation")
    ws = _workspace(ws_bytes, p3.device)
    # NaN until written: an early error return of the C call leaves it so
    res = torch.full((9,), float("nan"), dtype=torch.float64, device=p3.device)
    host = (ctypes.c_double * 8)(*([float("nan")] * 8))
    cam = model.acm_camera()
    cl, grid = _cell_args(cells, n)
    if collective is not None:
        rc = L.acm_linear_estimation_with_error_sharded(
            ctypes.byref(cam), n, p3.data_ptr() if n else None, _lib.LAYOUT_AOS,
            p2.data_ptr() if n else None, cl, grid, res.data_ptr(), host,
            ctypes.byref(collective.c), ws.data_ptr(), ws_bytes, _stream_handle())
    elif cells is not None:
        rc = L.acm_linear_estimation_with_error_cells_async(
            ctypes.byref(cam), n, p3.data_ptr(), _lib.LAYOUT_AOS, p2.data_ptr(), cl, grid,
            res.data_ptr(), host, ws.data_ptr(), ws_bytes, _stream_handle())
    else:
        rc = L.acm_linear_estimation_with_error_async(ctypes.byref(cam), n, p3.data_ptr(),
                                                      _lib.LAYOUT_AOS, p2.data_ptr(),
                                                      res.data_ptr(), host, ws.data_ptr(),
                                                      ws_bytes, _stream_handle())
    if rc not in (_lib.ACM_SUCCESS, _lib.ERR_INVALID_PARAMS, _lib.ERR_NUMERICAL):
        _lib.check(rc)
    out = list(host)
    if out[5] != out[5]:  # the initial error was never computed: the call's own error
        if rc == _lib.ERR_NUMERICAL:
            raise NumericalError(_lib.last_error())
        raise InvalidParams(_lib.last_error())
    n_valid = int(out[5])
    if n_valid == 0:
        raise ZeroProjectionPoints()
    if rc == _lib.ERR_INVALID_PARAMS:
        raise InvalidParams(_lib.last_error())
    if rc == _lib.ERR_NUMERICAL:
        raise NumericalError(_lib.last_error())
    model._set_params(list(cam.params)[: model.NUM_PARAMS])
    err = ProjectionError(rmse=out[0], min=out[1], max=out[2], mean=out[3], stddev=out[4],
                          median=float("nan"), n_valid=n_valid)

    def finish(err=err, res=res, ws=ws):  # ws: the median reads it until the stream passes
        return dataclasses.replace(err, median=float(res[8].item()))
    if defer_median:
        return err, finish
    return finish()


def reprojection_median(errors: torch.Tensor, n_valid: int) -> float:
    """Median of the valid (non-NaN) errors (error_metrics.rs:104-111)."""
    L = _lib.load()
    out = torch.empty((1,), dtype=torch.float64, device=errors.device)
    ws_bytes = L.acm_median_workspace_size(errors.numel())
    ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=errors.device)
    _lib.check(L.acm_median_valid(errors.numel(), errors.data_ptr(), None, n_valid, out.data_ptr(),
                                  ws.data_ptr(), ws_bytes, _stream_handle()))
    return float(out.item())


NEAREST, BILINEAR = 0, 1


def undistort_image(input_image, camera_model: CameraModel, target_intrinsics=None,
                    interpolation: int = BILINEAR):
    """`undistort_image` (src/util/undistort.rs:14-49): input_image (H, W, 3)
    uint8 (device or host), returns the (H, W, 3) uint8 device tensor."""
    res = camera_model.get_resolution()
    img = input_image if isinstance(input_image, torch.Tensor) else torch.as_tensor(input_image)
    img = img.to("cuda", torch.uint8).contiguous()
    if img.dim() != 3 or img.shape[2] != 3:
        raise UtilError("expected an (H, W, 3) RGB8 image")
    h, w = img.shape[0], img.shape[1]
    if w != res.width or h != res.height:  # :23-28
        raise UtilError(f"Image {w}x{h} doesn't match model {res.width}x{res.height}")
    out = torch.empty_like(img)
    cam = camera_model.acm_camera()
    t = None
    if target_intrinsics is not None:
        ti = target_intrinsics
        t = (ctypes.c_double * 4)(ti.fx, ti.fy, ti.cx, ti.cy)
    _lib.check(_lib.load().acm_undistort_image(ctypes.byref(cam), t, interpolation,
                                               img.data_ptr(), out.data_ptr(),
                                               _stream_handle()))
    return out


# ------------------------------------------------- validate_conversion_accuracy
@dataclass
class RegionValidation:
    name: str
    input_projection: object  # (u, v) or None
    output_projection: object
    error: float


@dataclass
class ValidationResults:
    center_error: float
    near_center_error: float
    mid_region_error: float
    edge_region_error: float
    far_edge_error: float
    average_error: float
    max_error: float
    status: str
    region_data: list


_REGIONS = (("Center", 0.5), ("Near Center", 0.55), ("Mid Region", 0.65),
            ("Edge Region", 0.8), ("Far Edge", 0.95))
_VALIDATION_CACHE = {}
_VALIDATION_CACHE_MAX = 64


def _validation_buffers(width: int, height: int):
    """The five test pixels of a resolution, resident on the device, and the
    device / pinned-host result buffers of validate_conversion_accuracy
    (cached per resolution, device, stream and thread: the call then launches
    three kernels and copies twice, without building tensors on the host).
    Two calls on one device from different threads or streams get different
    buffers, so neither overwrites the other's results between the copies
    and the synchronisation; the cache is bounded."""
    import threading
    key = (int(width), int(height), torch.cuda.current_device(),
           torch.cuda.current_stream().cuda_stream, threading.get_ident())
    if key not in _VALIDATION_CACHE:
        if len(_VALIDATION_CACHE) >= _VALIDATION_CACHE_MAX:
            _VALIDATION_CACHE.clear()
        w, h = float(width), float(height)
        k = len(_REGIONS)
        pix = torch.tensor([[w * f, h * f] for _, f in _REGIONS], dtype=torch.float64,
                           device="cuda")
        _VALIDATION_CACHE[key] = (
            pix, torch.empty((3 * k,), dtype=torch.uint8, device="cuda"),
            torch.empty((2 * k, 2), dtype=torch.float64, device="cuda"),
            torch.empty((3 * k,), dtype=torch.uint8).pin_memory(),
            torch.empty((2 * k, 2), dtype=torch.float64).pin_memory())
    return _VALIDATION_CACHE[key]


def validate_conversion_accuracy(output_model: CameraModel,
                                 input_model: CameraModel) -> ValidationResults:
    """`validate_conversion_accuracy` (validation.rs:92-213): the five
    diagonal test pixels (0.5 .. 0.95 of the input resolution) are
    unprojected with the input model and the rays projected with both models
    (one batched kernel call each); error = ||input_proj - output_proj||."""
    import math
    res = input_model.get_resolution()
    k = len(_REGIONS)
    pix, st_d, uv_d, st_h, uv_h = _validation_buffers(res.width, res.height)
    rays, _ = input_model.unproject_batch(pix, out=(None, st_d[:k]))
    input_model.project_batch(rays, out=(uv_d[:k], st_d[k:2 * k], None))
    output_model.project_batch(rays, out=(uv_d[k:], st_d[2 * k:], None))
    # two async copies into pinned host memory and one stream synchronisation
    st_h.copy_(st_d, non_blocking=True)
    uv_h.copy_(uv_d, non_blocking=True)
    torch.cuda.current_stream().synchronize()
    st = st_h.tolist()
    uvl = uv_h.tolist()
    rays_ok, ok_in, ok_out = st[:k], st[k:2 * k], st[2 * k:]
    a, b = uvl[:k], uvl[k:]
    total, max_error, valid = 0.0, 0.0, 0
    errs, data = [], []
    for i, (name, _) in enumerate(_REGIONS):
        if rays_ok[i] == 0 and ok_in[i] == 0 and ok_out[i] == 0:  # :120-143
            du, dv = a[i][0] - b[i][0], a[i][1] - b[i][1]
            e = math.sqrt(du * du + dv * dv)
            total += e
            max_error = max(max_error, e)
            valid += 1
            errs.append(e)
            data.append(RegionValidation(name, tuple(a[i]), tuple(b[i]), e))
        else:  # :144-182: any failure -> NaN, no projections recorded
            errs.append(float("nan"))
            data.append(RegionValidation(name, None, None, float("nan")))
    avg = total / valid if valid > 0 else float("nan")
    if math.isnan(avg):  # :192-200
        status = "NEEDS IMPROVEMENT"
    elif avg < 0.001:
        status = "EXCELLENT"
    elif avg < 0.1:
        status = "GOOD"
    else:
        status = "NEEDS IMPROVEMENT"
    return ValidationResults(*errs, average_error=avg, max_error=max_error, status=status,
                             region_data=data)
