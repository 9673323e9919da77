"""Levenberg-Marquardt model conversion (the apex-solver call sites of
bin/camera_converter.rs:381-420, :516-557, :655-698, :797-832, :928-965),
driven by libacm.so's C++ LM (csrc/solver.hip) over the fused GPU normal
equations.

`LevenbergMarquardtConfig` keeps apex-solver's builder surface
(`with_max_iterations`, `with_cost_tolerance`, ...).  For multi-GPU runs pass
`collective=distributed.make_collective(group)`: each rank holds its shard of
the correspondences and the (<= 92-double) normal-equation vector is summed
across ranks before every host solve (RCCL from C under the nccl backend).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional, Sequence, Tuple

import torch

from . import _lib
from .camera import CameraModel, _as_device_f64, _stream_handle


@dataclass
class LevenbergMarquardtConfig:
    max_iterations: int = 100
    cost_tolerance: float = 1e-6
    parameter_tolerance: float = 1e-8
    gradient_tolerance: float = 1e-6
    initial_damping: float = 1e-4
    invalid_policy: int = _lib.INVALID_SKIP

    def with_max_iterations(self, v):
        self.max_iterations = int(v)
        return self

    def with_cost_tolerance(self, v):
        self.cost_tolerance = float(v)
        return self

    def with_parameter_tolerance(self, v):
        self.parameter_tolerance = float(v)
        return self

    def with_gradient_tolerance(self, v):
        self.gradient_tolerance = float(v)
        return self

    def with_verbose(self, _v):
        return self


@dataclass
class LmResult:
    parameters: list
    iterations: int
    termination: str
    evaluations: int
    initial_cost: float
    final_cost: float
    n_valid: int


# camera_converter.rs set_variable_bounds per target model (index -> (lo, hi))
_INTR = {0: (1.0, 2000.0), 1: (1.0, 2000.0), 2: (0.0, 2000.0), 3: (0.0, 2000.0)}
CONVERTER_BOUNDS: Dict[str, Dict[int, Tuple[float, float]]] = {
    "double_sphere": {**_INTR, 4: (1e-6, 1.0), 5: (-5.0, 5.0)},          # :395-400
    "kannala_brandt": {**_INTR, 4: (-5.0, 5.0), 5: (-5.0, 5.0), 6: (-5.0, 5.0),
                       7: (-5.0, 5.0)},                                     # :536-543
    "rad_tan": {**_INTR, 4: (-5.0, 5.0), 5: (-5.0, 5.0), 6: (-1.0, 1.0), 7: (-1.0, 1.0),
                8: (-5.0, 5.0)},                                            # :676-684
    "ucm": {**_INTR, 4: (1e-6, 10.0)},                                      # :813-817
    "eucm": {**_INTR, 4: (1e-6, 1.0), 5: (1e-6, 5.0)},                      # :945-950
    "fov": {**_INTR, 4: (1e-6, 3.0)},                                       # :1076-1080
}


class LevenbergMarquardt:
    def __init__(self, config: Optional[LevenbergMarquardtConfig] = None):
        self.config = config or LevenbergMarquardtConfig()

    @classmethod
    def with_config(cls, config):
        return cls(config)

    def optimize(self, model: CameraModel, points_3d, points_2d,
                 bounds: Optional[Dict[int, Tuple[float, float]]] = None,
                 allreduce: Optional[Callable] = None, collective=None,
                 cells=None) -> LmResult:
        """Optimise model's factor-order parameters in place over the
        (local shard of the) correspondences.  collective (r06; e.g.
        distributed.RcclCollective): its all-reduce sums the normal
        equations of every evaluation across the ranks, from C; allreduce:
        a bare Python callback (acm_allreduce_fn) instead.  cells (r06):
        the util.CellSample of points_2d (grid-sampled correspondences):
        every evaluation reads the 4-B cells instead of the pixels
        (acm_lm_optimize_cells; the same iterates)."""
        L = _lib.load()
        p3 = _as_device_f64(points_3d, 3)
        p2 = _as_device_f64(points_2d, 2)
        n = p3.shape[0]
        cfg = _lib.LmConfig()
        L.acm_lm_default_config(ctypes.byref(cfg))
        c = self.config
        cfg.max_iterations = c.max_iterations
        cfg.cost_tolerance = c.cost_tolerance
        cfg.parameter_tolerance = c.parameter_tolerance
        cfg.gradient_tolerance = c.gradient_tolerance
        cfg.initial_damping = c.initial_damping
        cfg.invalid_policy = c.invalid_policy
        if bounds:
            cfg.has_bounds = 1
            for k, (lo, hi) in bounds.items():
                cfg.lower[k] = lo
                cfg.upper[k] = hi
        ws_bytes = L.acm_lm_workspace_size(model.MODEL_ID, n)
        ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=p3.device)
        cam = model.acm_camera()
        summ = _lib.LmSummary()
        ctx = None
        if collective is not None:
            cb, ctx = collective.c.allreduce, collective.c.ctx
        elif allreduce is not None:
            cb = _lib.ALLREDUCE_FN(allreduce)
        else:
            cb = _lib.ALLREDUCE_FN()
        if cells is not None:
            if cells.cells.shape[0] != n:
                raise ValueError("cells and points_3d must have the same number of points")
            _lib.check(L.acm_lm_optimize_cells(ctypes.byref(cam), n, p3.data_ptr() if n else None,
                                               _lib.LAYOUT_AOS,
                                               cells.cells.data_ptr() if n else None,
                                               ctypes.byref(cells.grid), ctypes.byref(cfg), cb,
                                               ctx, ctypes.byref(summ), ws.data_ptr(), ws_bytes,
                                               _stream_handle()))
        else:
            _lib.check(L.acm_lm_optimize(ctypes.byref(cam), n, p3.data_ptr() if n else None,
                                         _lib.LAYOUT_AOS, p2.data_ptr() if n else None,
                                         ctypes.byref(cfg), cb, ctx,
                                         ctypes.byref(summ), ws.data_ptr(), ws_bytes,
                                         _stream_handle()))
        params = list(cam.params)[: model.NUM_PARAMS]
        model._set_params(params)
        return LmResult(parameters=params, iterations=summ.iterations,
                        termination=_lib.LM_TERMINATION.get(summ.termination, "?"),
                        evaluations=summ.evaluations, initial_cost=summ.initial_cost,
                        final_cost=summ.final_cost, n_valid=int(summ.n_valid))
