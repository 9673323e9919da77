"""Multi-GPU execution of the hot path: one process per GPU, torch.distributed
for the (tiny) exchange steps -- backend "nccl" is RCCL over xGMI on MI355X,
"gloo" in the CPU tests.

The path shards trivially: every point is independent.
  * project / unproject / residual: contiguous shards, no collective at all;
  * LM normal equations: each rank reduces its shard on the GPU to
    P(P+1)/2 + P + 2 <= 56 doubles; ONE all-reduce(sum) of that vector per
    evaluation (448 B: latency-bound, link bandwidth irrelevant) before the
    host solve, so every rank takes identical LM steps;
  * reprojection statistics: all-reduce of [sum, sumsq, count] (sum), min,
    max, then of sum (e - mean)^2 -- the reference's two-pass stddev;
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


# ------------------------------------------------------- normal equations
def allreduce_normal_equations(vec: torch.Tensor, group=None) -> torch.Tensor:
    """In-place sum of the packed [JtJ | Jtr | cost | n_valid] vector."""
    dist.all_reduce(vec, op=dist.ReduceOp.SUM, group=group)
    return vec


# --------------------------------------------------- reprojection statistics
def combine_reprojection_stats(local_errors: torch.Tensor, group=None) -> dict:
    """error_metrics.rs:86-101 over the union of all ranks' valid errors
    (local_errors: this rank's per-point errors, NaN = failed projection).
    The median needs a distributed select and is computed by the caller."""
    valid = local_errors[~torch.isnan(local_errors)]
    dev = local_errors.device
    s = torch.stack([valid.sum(), (valid * valid).sum(),
                     torch.tensor(float(valid.numel()), dtype=torch.float64, device=dev)])
    mn = valid.min() if valid.numel() else torch.tensor(float("inf"), dtype=torch.float64,
                                                         device=dev)
    mx = valid.max() if valid.numel() else torch.tensor(float("-inf"), dtype=torch.float64,
                                                         device=dev)
    mn, mx = mn.clone().reshape(1), mx.clone().reshape(1)
    dist.all_reduce(s, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=group)
    n = float(s[2])
    mean = float(s[0]) / n
    var = ((valid - mean) ** 2).sum().reshape(1)
    dist.all_reduce(var, op=dist.ReduceOp.SUM, group=group)
    return {"rmse": (float(s[1]) / n) ** 0.5, "min": float(mn), "max": float(mx), "mean": mean,
            "stddev": (float(var) / n) ** 0.5, "n_valid": int(n)}


# ------------------------------------------------------------ sample_points
def sharded_sample_points(ncx: int, ncy: int, rank: int, world: int,
                          local_fn: Callable[[int, int], Tuple[torch.Tensor, torch.Tensor]],
                          group=None):
    """Run `local_fn(cell_begin, cell_end) -> (uv (m,2), xyz (m,3))` on this
    rank's grid rows; return (uv, xyz, global_offset, global_total) so that
    the rank-ordered concatenation equals the serial sample_points output."""
    c0, c1 = grid_row_range(ncx, ncy, rank, world)
    uv, xyz = local_fn(c0, c1)
    m = torch.tensor([uv.shape[0]], dtype=torch.int64, device=uv.device)
    counts = [torch.zeros_like(m) for _ in range(world)]
    dist.all_gather(counts, m, group=group)
    counts = [int(c) for c in counts]
    return uv, xyz, sum(counts[:rank]), sum(counts)


def gpu_sample_points_range(model, n_requested: int):
    """local_fn for sharded_sample_points backed by acm_sample_points_range."""
    from . import _lib
    from .camera import _stream_handle
    L = _lib.load()
    cam = model.acm_camera()

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
