"""Model conversion pipeline of bin/camera_converter.rs (convert_to_*,
:355-1163): sample correspondences from the input model, initialise the
target, linear estimation, bounded LM, reprojection errors -- all on the GPU
through libacm.so.  Report formatting, validation tables and image-quality
metrics (reporting.rs, validation.rs, image_quality.rs) are out of scope."""
from __future__ import annotations

import time
from dataclasses import dataclass

from . import _lib, util
from .camera import (CameraModel, DoubleSphereModel, EucmModel, FovModel, Intrinsics,
                     KannalaBrandtModel, RadTanModel, UcmModel)
from .optimizer import CONVERTER_BOUNDS, LevenbergMarquardt, LevenbergMarquardtConfig


@dataclass
class ConversionMetrics:
    model: CameraModel
    model_name: str
    final_reprojection_error: util.ProjectionError
    initial_reprojection_error: util.ProjectionError
    optimization_time_ms: float
    convergence_status: str
    lm_iterations: int = 0
    lm_termination: str = ""
    validation_results: object = None  # util.ValidationResults (validation.rs)


# initial target parameters (camera_converter.rs:364-369, :500-505, :639-644,
# :781-785, :911-916, :1045-1049)
def _init_target(name, src: CameraModel):
    i = src.get_intrinsics()
    res = src.get_resolution()
    intr = Intrinsics(i.fx, i.fy, i.cx, i.cy)
    if name == "double_sphere":
        return DoubleSphereModel(intr, res, 0.5, 0.1)
    if name == "kannala_brandt":
        return KannalaBrandtModel(intr, res, [0.0] * 4)
    if name == "rad_tan":
        return RadTanModel(intr, res, [0.0] * 5)
    if name == "ucm":
        return UcmModel(intr, res, 0.5)
    if name == "eucm":
        return EucmModel(intr, res, 0.5, 1.0)
    if name == "fov":
        return FovModel(intr, res, 1.0)
    raise ValueError(name)


DISPLAY = {"double_sphere": "Double Sphere", "kannala_brandt": "Kannala-Brandt",
           "rad_tan": "Radial-Tangential", "ucm": "Unified Camera Model",
           "eucm": "Extended Unified Camera Model", "fov": "Field-of-View"}


def convert(input_model: CameraModel, target: str, points_3d, points_2d,
            config: LevenbergMarquardtConfig = None, collective=None,
            cells=None) -> ConversionMetrics:
    """One `convert_to_<target>` (e.g. convert_to_double_sphere :355-488).

    Multi-GPU (r06): pass this rank's shard of the correspondences and a
    `collective` (distributed.make_collective(group): RCCL driven from libacm
    under the nccl backend).  The opening (initial error + linear
    estimation, one fused pass per shard and one all-gather), the LM's
    normal equations (one all-reduce per evaluation) and the final
    reprojection error then all run over the union of the shards,
    identically on every rank, with the same structure as on one GPU.

    cells (r06): the util.CellSample of points_2d when the correspondences
    come from sample_points(..., cells=True): the opening, the LM's
    evaluations and the final error read the 4-B cells instead of the 16-B
    pixels -- the same results, bit for bit."""
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    model = _init_target(target, input_model)
    # the initial error and the linear estimation in one pass (r04); its
    # median completes on the stream while the LM starts (r05)
    initial, finish_initial = util.initial_error_and_linear_estimation(
        model, points_3d, points_2d, defer_median=True, collective=collective, cells=cells)
    cfg = config or LevenbergMarquardtConfig()
    status = "Converged"
    res = None
    try:
        res = LevenbergMarquardt(cfg).optimize(model, points_3d, points_2d,
                                               bounds=CONVERTER_BOUNDS[target],
                                               collective=collective, cells=cells)
        if res.termination == "Failed":
            status = "Linear Only"
    except _lib.AcmError as e:
        # camera_converter.rs:443: the solver's Err(_) => "Linear Only".  Only
        # a numerical failure of the solve is that; a device fault
        # (ACM_ERR_HIP, incl. a failed all-reduce), a bad argument or a too
        # small workspace is not a solver outcome and propagates.
        if e.code != _lib.ERR_NUMERICAL:
            raise
        status = "Linear Only"
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    initial = finish_initial()
    final = util.compute_reprojection_error(model, points_3d, points_2d, collective=collective,
                                            cells=cells)
    # camera_converter.rs:425-438; failed regions come back as NaN (no raise)
    validation = util.validate_conversion_accuracy(model, input_model)
    return ConversionMetrics(model=model, model_name=DISPLAY[target],
                             final_reprojection_error=final, initial_reprojection_error=initial,
                             optimization_time_ms=ms, convergence_status=status,
                             lm_iterations=res.iterations if res else 0,
                             lm_termination=res.termination if res else "",
                             validation_results=validation)


def convert_all(input_model: CameraModel, num_points: int = 500,
                targets=("double_sphere", "kannala_brandt", "rad_tan", "ucm", "eucm", "fov")):
    """camera_converter.rs main (:127-350): sample_points once (:189), then
    every target conversion except the input's own model (:225-340)."""
    points_2d, points_3d = util.sample_points(input_model, num_points)
    return {t: convert(input_model, t, points_3d, points_2d) for t in targets
            if t != input_model.NAME}
