"""Multi-GPU execution of the hot path: one process per GPU, torch.distributed
for the (tiny) exchange steps -- backend "nccl" is RCCL over xGMI on MI355X,
"gloo" in the CPU tests.

The path shards trivially: every point is independent.
  * project / unproject / residual: contiguous shards, no collective at all;
  * LM normal equations: each rank reduces its shard on the GPU to
    P(P+1)/2 + P + 2 <= 56 doubles; ONE all-reduce(sum) of that vector per
    evaluation (448 B: latency-bound, link bandwidth irrelevant) before the
    host solve, so every rank takes identical LM steps;
  * reprojection statistics: each rank reduces its shard on the GPU to the
    8-double acm_reprojection_stats / acm_error_stats result; ONE all-gather
    of those, then libacm's rank-ordered Chan merge
    (acm_reprojection_stats_merge) -- every rank gets the same bits; the
    median is the exact distributed radix select (one all-reduce of a
    histogram per pass);
  * sample_points: ranks take contiguous row ranges of the cell grid, and
    concatenation in rank order (offsets from an all-gather of the kept
    counts) reproduces the serial order of point_sampling.rs:88-103.

The local evaluators are injectable (defaults: libacm.so kernels), which is
how the gloo tests run the same exchange logic on the CPU.
"""
from __future__ import annotations

import ctypes
from typing import Callable, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard of ceil(n / world) items (the last may be shorter)."""
    per = (n + world - 1) // world
    lo = min(rank * per, n)
    return lo, min(lo + per, n)


def grid_row_range(ncx: int, ncy: int, rank: int, world: int) -> Tuple[int, int]:
    """Cell range [begin, end) of whole grid rows for `rank`."""
    r0, r1 = shard_range(ncy, rank, world)
    return r0 * ncx, r1 * ncx


# ------------------------------------------------------------- device views
class _DeviceArray:
    def __init__(self, ptr: int, count: int):
        self.__cuda_array_interface__ = {"shape": (count,), "typestr": "<f8",
                                         "data": (ptr, False), "version": 3}


def device_view(ptr: int, count: int) -> torch.Tensor:
    """Zero-copy float64 tensor over a device pointer (same HIP runtime)."""
    return torch.as_tensor(_DeviceArray(ptr, count), device="cuda")


def rccl_allreduce(group=None) -> Callable:
    """Callback for acm_lm_optimize / LevenbergMarquardt.optimize(allreduce=...):
    sums the device normal-equation vector across ranks with RCCL."""

    def cb(_ctx, dev_ptr, count, _stream):
        try:
            t = device_view(int(dev_ptr), int(count))
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            return 0
        except Exception:  # report to the C++ driver as a failed callback
            return -1

    return cb


# ------------------------------------------------------ the collectives
class TorchCollective:
    """acm_collective (include/acm.h) whose all-reduce / all-gather are
    torch.distributed calls on zero-copy views of libacm's device buffers --
    any backend, including gloo ranks that share one GPU (the tests).  Each
    collective is a ctypes callback into Python; RcclCollective is the
    production form with none."""

    def __init__(self, group=None):
        from . import _lib
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self._views = {}

        def view(ptr, count):
            key = (int(ptr), int(count))
            t = self._views.get(key)
            if t is None:
                if len(self._views) > 64:
                    self._views.clear()
                t = self._views[key] = device_view(int(ptr), int(count))
            return t

        def allreduce(_ctx, ptr, count, _stream):
            try:
                dist.all_reduce(view(ptr, count), op=dist.ReduceOp.SUM, group=group)
                return 0
            except Exception:  # noqa: BLE001 -- a failed callback, reported by libacm
                return -1

        def allgather(_ctx, send, recv, count, _stream):
            try:
                r = view(recv, count * self.world)
                dist.all_gather(list(r.split(int(count))), view(send, count), group=group)
                return 0
            except Exception:  # noqa: BLE001
                return -1

        self._ar = _lib.ALLREDUCE_FN(allreduce)  # kept alive with the struct
        self._ag = _lib.ALLGATHER_FN(allgather)
        self.c = _lib.AcmCollective(self._ar, self._ag, None, self.rank, self.world)

    def close(self):
        self._views.clear()


class RcclCollective:
    """acm_collective over an RCCL communicator that libacm drives itself
    (acm_rccl_init): rank 0 makes the unique id, torch.distributed
    broadcasts it once, every rank joins with its own GPU current.  The LM's
    all-reduce per evaluation and the median's histogram all-reduces are
    then RCCL calls on the stream from C -- no Python per collective.  One
    GPU per rank (RCCL refuses two ranks on one device)."""

    def __init__(self, group=None):
        from . import _lib
        L = _lib.load()
        self.c = None
        if dist.is_available() and dist.is_initialized():
            self.world = dist.get_world_size(group)
            self.rank = dist.get_rank(group)
        else:  # no process group: a 1-rank communicator (bench.py's world-1 leg)
            self.world, self.rank = 1, 0
        ok = int(bool(L.acm_rccl_available()))
        if self.world > 1:  # the same answer on every rank (see below)
            dev = torch.device("cuda", torch.cuda.current_device()) \
                if dist.get_backend(group) == "nccl" else torch.device("cpu")
            t = torch.tensor([ok], dtype=torch.int32, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
            ok = int(t.item())
        if not ok:
            raise RuntimeError("librccl.so.1 is not loadable on every rank: no RCCL collective")
        self.c = None
        uid = (ctypes.c_uint8 * _lib.RCCL_UNIQUE_ID_BYTES)()
        rc = L.acm_rccl_unique_id(uid) if self.rank == 0 else 0
        obj = [rc, bytes(uid)]
        if self.world > 1:
            # every rank learns whether rank 0 could make the id, so a failure
            # raises on all ranks alike instead of leaving the others blocked
            # in the communicator's rendezvous
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(obj, src=src, group=group)
        if obj[0] != 0:
            raise RuntimeError(f"acm_rccl_unique_id failed on rank 0 ({obj[0]})")
        uid = (ctypes.c_uint8 * _lib.RCCL_UNIQUE_ID_BYTES).from_buffer_copy(obj[1])
        self.c = _lib.AcmCollective()
        _lib.check(L.acm_rccl_init(uid, self.world, self.rank, ctypes.byref(self.c)))

    def close(self):
        from . import _lib
        if self.c is not None and self.c.ctx:
            _lib.check(_lib.load().acm_rccl_destroy(ctypes.byref(self.c)))
        self.c = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


class LocalCollective:
    """The 1-rank acm_collective with no callbacks: the sharded entry points
    then run every merge and the median locally (tests: the sharded path's
    bits at world 1 without any communicator)."""

    def __init__(self):
        from . import _lib
        self.world, self.rank = 1, 0
        self.c = _lib.AcmCollective(_lib.ALLREDUCE_FN(), _lib.ALLGATHER_FN(), None, 0, 1)

    def close(self):
        pass


def make_collective(group=None):
    """The sharded conversion's collective for `group`: RcclCollective under
    the nccl (RCCL) backend with one GPU per rank, else TorchCollective --
    also when RCCL cannot be set up; RcclCollective raises on every rank
    alike before the communicator's rendezvous, so the fallback is taken by
    all ranks together (the bench line names the collective it used)."""
    if dist.get_backend(group) == "nccl":
        try:
            return RcclCollective(group)
        except RuntimeError:
            pass
    return TorchCollective(group)


# ------------------------------------------------------- normal equations
def allreduce_normal_equations(vec: torch.Tensor, group=None) -> torch.Tensor:
    """In-place sum of the packed [JtJ | Jtr | cost | n_valid] vector."""
    dist.all_reduce(vec, op=dist.ReduceOp.SUM, group=group)
    return vec


# --------------------------------------------------- reprojection statistics
STAT_KEYS = ("rmse", "min", "max", "mean", "stddev", "n_valid", "sum", "sumsq")


def local_reprojection_result(errors) -> torch.Tensor:
    """acm_reprojection_stats' 8-double result [rmse, min, max, mean, stddev,
    n_valid, sum, sumsq] of one shard's per-point errors computed on the
    host (NaN = invalid) -- for shards whose errors come from elsewhere, e.g.
    the CPU oracle in the gloo tests."""
    import numpy as np
    e = np.asarray(errors.cpu() if isinstance(errors, torch.Tensor) else errors,
                   dtype=np.float64)
    v = e[~np.isnan(e)]
    n = float(v.size)
    if n == 0:
        return torch.tensor([np.nan, np.inf, -np.inf, np.nan, np.nan, 0.0, 0.0, 0.0],
                            dtype=torch.float64)
    s, ss = float(v.sum()), float((v * v).sum())
    mean = s / n
    return torch.tensor([(ss / n) ** 0.5, float(v.min()), float(v.max()), mean,
                         (float(((v - mean) ** 2).sum()) / n) ** 0.5, n, s, ss],
                        dtype=torch.float64)


def merge_reprojection_stats(local_result: torch.Tensor, group=None) -> dict:
    """error_metrics.rs:86-111 over the union of every rank's shard: ONE
    all-gather of each rank's 8-double acm_reprojection_stats result, then
    libacm's rank-ordered merge (acm_reprojection_stats_merge: sums, extrema,
    Chan's update of (n, mean, M2)) -- every rank computes the same numbers
    bit for bit.  No mask copy, no per-statistic all-reduce, no second
    variance pass over the errors."""
    import ctypes

    from . import _lib
    world = dist.get_world_size(group)
    be = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if be == "nccl" else \
        torch.device("cpu")
    mine = local_result.reshape(8).to(dev, torch.float64).contiguous()
    allr = [torch.empty((8,), dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(allr, mine, group=group)
    parts = torch.stack(allr).cpu().contiguous()
    out = (ctypes.c_double * 8)()
    _lib.check(_lib.load().acm_reprojection_stats_merge(
        world, ctypes.cast(parts.data_ptr(), ctypes.POINTER(ctypes.c_double)), out))
    d = dict(zip(STAT_KEYS, list(out)))
    d["n_valid"] = int(d["n_valid"])
    return d


def device_error_stats(errors: torch.Tensor) -> torch.Tensor:
    """acm_error_stats: the 8-double statistics result of one shard's device
    error vector (NaN = invalid), reduced on the GPU -- no host copy."""
    from . import _lib
    from .camera import _stream_handle
    L = _lib.load()
    e = errors.contiguous()
    n = e.numel()
    out = torch.empty((8,), dtype=torch.float64, device=e.device)
    ws_bytes = L.acm_error_stats_workspace_size(n)
    ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=e.device)
    _lib.check(L.acm_error_stats(n, e.data_ptr() if n else None, out.data_ptr(), ws.data_ptr(),
                                 ws_bytes, _stream_handle()))
    return out


def combine_reprojection_stats(local_errors: torch.Tensor, group=None) -> dict:
    """Statistics of the union of every rank's per-point errors (NaN =
    invalid) via merge_reprojection_stats.  Device errors are reduced on the
    GPU (acm_error_stats) and also get the exact median of the union
    (distributed_median); host errors (the gloo tests' oracle shards) take
    local_reprojection_result."""
    if local_errors.is_cuda:
        local = device_error_stats(local_errors.to(torch.float64))
    else:
        local = local_reprojection_result(local_errors)
    out = merge_reprojection_stats(local, group)
    if local_errors.is_cuda and out["n_valid"] > 0:
        out["median"] = distributed_median(local_errors, out["n_valid"], group)
    return out


def distributed_median(local_errors: torch.Tensor, n_valid_global: int, group=None) -> float:
    """Exact median of the union of every rank's non-NaN errors
    (error_metrics.rs:103-111): acm_median_valid_allreduce, one all-reduce of
    the 2 x 2048-bin histogram per radix pass (6 x 32 KB, latency-bound)."""
    import ctypes

    from . import _lib
    from .camera import _stream_handle
    L = _lib.load()
    e = local_errors.contiguous()
    out = torch.empty((1,), dtype=torch.float64, device=e.device)
    ws_bytes = L.acm_median_workspace_size(e.numel())
    ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=e.device)
    cb = _lib.ALLREDUCE_FN(rccl_allreduce(group))
    _lib.check(L.acm_median_valid_allreduce(e.numel(), e.data_ptr() if e.numel() else None,
                                            None, n_valid_global, out.data_ptr(), ws.data_ptr(),
                                            ws_bytes, cb, None, _stream_handle()))
    return float(out.item())


# ---------------------------------------------------- linear estimation
def distributed_linear_estimation(model, points_3d, points_2d, group=None) -> None:
    """`XModel::linear_estimation` over the union of every rank's
    correspondences.  KB/RadTan/DS/UCM/EUCM: each rank reduces its shard's
    [A | b] rows to a (k+1)^2 TSQR factor on the GPU, the factors are
    all-gathered and folded in rank order (acm_linear_system_r_merge), and
    every rank solves the same system (acm_linear_estimation_solve).  FOV:
    the all-reduced grid search.  Updates the model in place, identically on
    every rank."""
    import ctypes

    from . import _lib
    from .camera import InvalidParams, NumericalError, _as_device_f64, _stream_handle
    if model.NAME == "fov":
        return distributed_fov_linear_estimation(model, points_3d, points_2d, group)
    L = _lib.load()
    p3 = _as_device_f64(points_3d, 3)
    p2 = _as_device_f64(points_2d, 2)
    if p3.shape[0] != p2.shape[0]:
        raise InvalidParams("Number of 2D and 3D points must match")
    n = p3.shape[0]
    mid = model.MODEL_ID
    k = L.acm_linear_system_columns(mid)
    if k < 0:
        raise InvalidParams(f"{model.NAME} has no linear_estimation")
    S = (k + 1) * (k + 2) // 2
    dev = p3.device
    ws_bytes = L.acm_linear_system_qr_workspace_size(mid, n)
    ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=dev)
    r_dev = torch.zeros((S + 2,), dtype=torch.float64, device=dev)  # R | err | n
    err = torch.zeros((1,), dtype=torch.int32, device=dev)
    cam = model.acm_camera()
    _lib.check(L.acm_linear_system_qr(ctypes.byref(cam), n, p3.data_ptr() if n else None,
                                      _lib.LAYOUT_AOS, p2.data_ptr() if n else None,
                                      r_dev.data_ptr(), err.data_ptr(), ws.data_ptr(), ws_bytes,
                                      _stream_handle()))
    r_dev[S] = err[0].to(torch.float64)
    r_dev[S + 1] = float(n)
    world = dist.get_world_size(group)
    parts = [torch.empty_like(r_dev) for _ in range(world)]
    dist.all_gather(parts, r_dev, group=group)
    host = [p.cpu().tolist() for p in parts]
    R = (ctypes.c_double * S)(*host[0][:S])
    for h in host[1:]:
        _lib.check(L.acm_linear_system_r_merge(mid, R, (ctypes.c_double * S)(*h[:S])))
    any_err = int(any(h[S] != 0.0 for h in host))
    n_total = int(sum(h[S + 1] for h in host))
    rc = L.acm_linear_estimation_solve(ctypes.byref(cam), n_total, R, any_err)
    if rc == _lib.ERR_INVALID_PARAMS:
        raise InvalidParams(_lib.last_error())
    if rc == _lib.ERR_NUMERICAL:
        raise NumericalError(_lib.last_error())
    _lib.check(rc)
    model._set_params(list(cam.params)[: model.NUM_PARAMS])


def distributed_reprojection_error(model, points_3d, points_2d, group=None):
    """`compute_reprojection_error` (error_metrics.rs:62-121) over the union of
    every rank's correspondences (GPU per-point errors, all-reduced sums and
    extrema, distributed exact median)."""
    from . import util
    from .camera import _as_device_f64
    p3 = _as_device_f64(points_3d, 3)
    errors = torch.empty((p3.shape[0],), dtype=torch.float64, device=p3.device)
    local = util.reprojection_stats(model, p3, points_2d, errors)  # this shard, on the GPU
    st = merge_reprojection_stats(local, group)
    if st["n_valid"] == 0:  # error_metrics.rs:82-84, on every rank alike
        raise util.ZeroProjectionPoints()
    st["median"] = distributed_median(errors, st["n_valid"], group)
    return util.ProjectionError(rmse=st["rmse"], min=st["min"], max=st["max"], mean=st["mean"],
                                stddev=st["stddev"], median=st["median"], n_valid=st["n_valid"])


# ------------------------------------------------------ FOV grid search
def distributed_fov_linear_estimation(model, points_3d, points_2d, group=None) -> None:
    """FovModel::linear_estimation (fov.rs:153-251) over the union of every
    rank's correspondences: each rank runs the 290-value grid on its shard
    (acm_fov_grid_errors), the 2 x 290 sums are all-reduced, and every rank
    selects the same w (acm_fov_grid_select).  Updates model.w in place."""
    import ctypes

    from . import _lib
    from .camera import InvalidParams, _as_device_f64, _stream_handle
    L = _lib.load()
    p3 = _as_device_f64(points_3d, 3)
    p2 = _as_device_f64(points_2d, 2)
    if p3.shape[0] != p2.shape[0]:
        raise InvalidParams("Number of 2D and 3D points must match")
    n = p3.shape[0]
    total = torch.tensor([float(n)], dtype=torch.float64, device=p3.device)
    dist.all_reduce(total, op=dist.ReduceOp.SUM, group=group)
    if float(total) < 2:  # fov.rs:166-171
        raise InvalidParams("Need at least 2 point correspondences for linear estimation")
    ws_bytes = L.acm_fov_grid_workspace_size(n)
    ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=p3.device)
    sums = torch.empty((2 * _lib.FOV_GRID_SIZE,), dtype=torch.float64, device=p3.device)
    cam = model.acm_camera()
    _lib.check(L.acm_fov_grid_errors(ctypes.byref(cam), n, p3.data_ptr() if n else None,
                                     _lib.LAYOUT_AOS, p2.data_ptr() if n else None,
                                     sums.data_ptr(), ws.data_ptr(), ws_bytes, _stream_handle()))
    dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    host = (ctypes.c_double * (2 * _lib.FOV_GRID_SIZE))(*sums.cpu().tolist())
    rc = L.acm_fov_grid_select(ctypes.byref(cam), host)
    if rc == _lib.ERR_INVALID_PARAMS:
        raise InvalidParams(_lib.last_error())
    _lib.check(rc)
    model._set_params(list(cam.params)[: model.NUM_PARAMS])


# ------------------------------------------------------------ sample_points
def sharded_sample_points(ncx: int, ncy: int, rank: int, world: int,
                          local_fn: Callable[[int, int], Tuple[torch.Tensor, torch.Tensor]],
                          group=None):
    """Run `local_fn(cell_begin, cell_end) -> (uv (m,2), xyz (m,3))` on this
    rank's grid rows; return (uv, xyz, global_offset, global_total) so that
    the rank-ordered concatenation equals the serial sample_points output."""
    c0, c1 = grid_row_range(ncx, ncy, rank, world)
    out = local_fn(c0, c1)
    uv = out[0]
    m = torch.tensor([uv.shape[0]], dtype=torch.int64, device=uv.device)
    counts = [torch.zeros_like(m) for _ in range(world)]
    dist.all_gather(counts, m, group=group)
    counts = [int(c) for c in counts]
    return (*out, sum(counts[:rank]), sum(counts))


def gpu_sample_points_range(model, n_requested: int, cells: bool = False):
    """local_fn for sharded_sample_points backed by acm_sample_points_range
    (cells=True: util.sample_points' cell form, (uv, xyz, CellSample) with
    the global cell ids of the shard's rows)."""
    from . import _lib
    from .camera import _stream_handle
    L = _lib.load()
    cam = model.acm_camera()
    if cells:
        from . import util
        return lambda c0, c1: util.sample_points(model, n_requested, cells=True,
                                                 cell_range=(c0, c1))

    def fn(c0, c1):
        cells = max(c1 - c0, 0)
        dev = torch.device("cuda")
        uv = torch.empty((max(cells, 1), 2), dtype=torch.float64, device=dev)
        xyz = torch.empty((max(cells, 1), 3), dtype=torch.float64, device=dev)
        counts = torch.zeros((2,), dtype=torch.int64, device=dev)
        ws_bytes = L.acm_sample_points_workspace_size(ctypes.byref(cam), n_requested)
        ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=dev)
        _lib.check(L.acm_sample_points_range(ctypes.byref(cam), n_requested, c0, c1,
                                             uv.data_ptr(), xyz.data_ptr(), counts.data_ptr(),
                                             ws.data_ptr(), ws_bytes, _stream_handle()))
        m = int(counts[0].item())
        return uv[:m], xyz[:m]

    return fn
