"""ctypes binding of libacm.so (the C-ABI declared in include/acm.h).

The product path runs only through this library: there is no CPU fallback.
If libacm.so is missing, importing the package raises -- build it with
``python -c "import __graft_entry__ as g; g.build()"`` (or ``make -C
apex-camera-models_amd``).

torch is imported first on purpose: torch ships its own libamdhip64.so.7 and
libacm.so links the same SONAME, so loading torch first makes both share ONE
HIP runtime (device pointers and streams from torch are then valid here).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module doc)

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# ACM_LIB_PATH: load another build of the same C-ABI (the tools' diagnostic
# and A/B builds, e.g. lib/libacm_ieee.so); default: the in-tree libacm.so
LIB_PATH = os.environ.get("ACM_LIB_PATH") or os.path.join(_PKG_ROOT, "lib", "libacm.so")

# model ids / codes (include/acm.h)
PINHOLE, RADTAN, KANNALA_BRANDT, DOUBLE_SPHERE, UCM, EUCM, FOV = range(7)
LAYOUT_AOS, LAYOUT_SOA = 0, 1
EXACT_MATH = 0x100  # OR-ed into acm_project's layout (include/acm.h)
REFERENCE_NEWTON = 0x200  # OR-ed into acm_unproject's layout / acm_sample_points_ex's flags
INVALID_SKIP, INVALID_SENTINEL = 0, 1
MAX_PARAMS = 9

ACM_SUCCESS = 0
ERR_INVALID_MODEL = -1
ERR_INVALID_PARAMS = -2
ERR_INVALID_ARGUMENT = -3
ERR_HIP = -4
ERR_WORKSPACE_TOO_SMALL = -5


class LmConfig(ctypes.Structure):
    _fields_ = [
        ("max_iterations", ctypes.c_int32),
        ("invalid_policy", ctypes.c_int32),
        ("cost_tolerance", ctypes.c_double),
        ("parameter_tolerance", ctypes.c_double),
        ("gradient_tolerance", ctypes.c_double),
        ("initial_damping", ctypes.c_double),
        ("has_bounds", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("lower", ctypes.c_double * 9),
        ("upper", ctypes.c_double * 9),
    ]


class LmSummary(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int32),
        ("termination", ctypes.c_int32),
        ("evaluations", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("initial_cost", ctypes.c_double),
        ("final_cost", ctypes.c_double),
        ("n_valid", ctypes.c_double),
    ]


ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.c_void_p)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_size_t, ctypes.c_void_p)


class AcmCollective(ctypes.Structure):
    """acm_collective (include/acm.h, r06): the sharded conversion's
    stream-ordered all-reduce / all-gather over device f64 buffers."""
    _fields_ = [
        ("allreduce", ALLREDUCE_FN),
        ("allgather", ALLGATHER_FN),
        ("ctx", ctypes.c_void_p),
        ("rank", ctypes.c_int32),
        ("world", ctypes.c_int32),
    ]


RCCL_UNIQUE_ID_BYTES = 128


class CellGrid(ctypes.Structure):
    """acm_cell_grid (include/acm.h, r06): the grid of a cell-form sample."""
    _fields_ = [
        ("num_cells_x", ctypes.c_uint32),
        ("num_cells_y", ctypes.c_uint32),
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
    ]
TUNE_PROJECT_VARIANT, TUNE_RESIDUAL_NT, TUNE_NE_WAVES, TUNE_FOV_UNROLL, TUNE_NE_UNROLL = 0, 1, 2, 3, 4
TUNE_ALIGN_J, TUNE_NT_LOADS, TUNE_NT_LOADS_UNPROJECT, TUNE_LM_HOST_RESULT = 5, 6, 7, 8
TUNE_SAMPLE_FUSED, TUNE_UNPROJECT_RCP, TUNE_SAMPLE_PATIENCE = 9, 10, 11
TUNE_NEWTON_FAST = 12  # removed in round 3: acm_set_tuning rejects it (use REFERENCE_NEWTON)
TUNE_UNPROJECT_PPT = 13
TUNE_SAMPLE_CERT = 14
TUNE_SAMPLE_WRITE = 15
TUNE_LM_DEVICE = 16  # removed in r05 (acm_set_tuning: ACM_ERR_NOT_SUPPORTED)
TUNE_ROUND_TRIP = 17  # r05: acm_project_unproject PPT + 8 x ray stores (same outputs)
ERR_NOT_SUPPORTED = -6
ERR_NUMERICAL = -7
LM_TERMINATION = {0: "MaxIterations", 1: "CostTolerance", 2: "ParameterTolerance",
                  3: "GradientTolerance", 4: "Failed"}


class AcmCamera(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int32),
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("num_params", ctypes.c_uint32),
        ("params", ctypes.c_double * MAX_PARAMS),
    ]


FOV_GRID_SIZE = 290  # ACM_FOV_GRID_SIZE

EXPORTED_SYMBOLS = (
    "acm_num_params",
    "acm_camera_init",
    "acm_validate_params",
    "acm_project",
    "acm_project_f32",
    "acm_unproject",
    "acm_residual_jacobian",
    "acm_normal_equations_workspace_size",
    "acm_normal_equations",
    "acm_reprojection_stats_workspace_size",
    "acm_reprojection_stats",
    "acm_reprojection_stats_merge",
    "acm_project_unproject",
    "acm_reprojection_error_workspace_size",
    "acm_reprojection_error",
    "acm_linear_estimation_with_error_workspace_size",
    "acm_linear_estimation_with_error",
    "acm_linear_estimation_with_error_async",
    "acm_error_stats_workspace_size",
    "acm_error_stats",
    "acm_linear_system_columns",
    "acm_linear_system_qr_workspace_size",
    "acm_linear_system_qr",
    "acm_linear_estimation_workspace_size",
    "acm_linear_estimation",
    "acm_linear_system_r_merge",
    "acm_linear_estimation_solve",
    "acm_fov_grid_workspace_size",
    "acm_fov_grid_errors",
    "acm_fov_grid_select",
    "acm_lm_default_config",
    "acm_lm_workspace_size",
    "acm_lm_optimize",
    "acm_normal_equations_cells",
    "acm_reprojection_error_cells",
    "acm_linear_estimation_with_error_cells_async",
    "acm_lm_optimize_cells",
    "acm_sample_points_cells",
    "acm_rccl_available",
    "acm_rccl_unique_id",
    "acm_rccl_init",
    "acm_rccl_destroy",
    "acm_linear_estimation_with_error_sharded_workspace_size",
    "acm_linear_estimation_with_error_sharded",
    "acm_reprojection_error_sharded_workspace_size",
    "acm_reprojection_error_sharded",
    "acm_median_workspace_size",
    "acm_median_valid",
    "acm_median_valid_allreduce",
    "acm_sample_points_grid",
    "acm_sample_points_workspace_size",
    "acm_sample_points",
    "acm_sample_points_range",
    "acm_sample_points_ex",
    "acm_sample_points_certificate",
    "acm_unproject_certificate",
    "acm_sample_points_ray_poly",
    "acm_sample_points_ray_fit",
    "acm_undistort_image",
    "acm_set_device",
    "acm_device_malloc",
    "acm_device_free",
    "acm_memcpy_htod",
    "acm_memcpy_dtoh",
    "acm_stream_synchronize",
    "acm_set_tuning",
    "acm_last_hip_error",
    "acm_last_error",
    "acm_version",
)

_lib = None


from ._buildinfo import source_sha256  # noqa: E402,F401  (bench.py's traffic check)


class AcmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libacm error {code}: {msg}")
        self.code = code


def load():
    """Load libacm.so and declare every C-ABI signature (fails loudly)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libacm.so not found at {LIB_PATH}: the HIP extension is not built "
            "(run __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    cam_p = ctypes.POINTER(AcmCamera)
    vp = ctypes.c_void_p
    sz = ctypes.c_size_t
    i = ctypes.c_int
    L.acm_num_params.argtypes = [i]
    L.acm_num_params.restype = i
    L.acm_camera_init.argtypes = [cam_p, i, ctypes.POINTER(ctypes.c_double), sz,
                                  ctypes.c_uint32, ctypes.c_uint32]
    L.acm_camera_init.restype = i
    L.acm_validate_params.argtypes = [cam_p]
    L.acm_validate_params.restype = i
    L.acm_project.argtypes = [cam_p, sz, vp, i, vp, vp, vp, vp]
    L.acm_project.restype = i
    L.acm_project_f32.argtypes = [cam_p, sz, vp, i, vp, vp, vp, vp]
    L.acm_project_f32.restype = i
    L.acm_unproject.argtypes = [cam_p, sz, vp, vp, i, vp, vp]
    L.acm_unproject.restype = i
    L.acm_residual_jacobian.argtypes = [cam_p, sz, vp, i, vp, i, vp, vp, vp, vp]
    L.acm_residual_jacobian.restype = i
    L.acm_normal_equations_workspace_size.argtypes = [i, sz]
    L.acm_normal_equations_workspace_size.restype = sz
    L.acm_normal_equations.argtypes = [cam_p, sz, vp, i, vp, i, vp, vp, sz, vp]
    L.acm_normal_equations.restype = i
    L.acm_reprojection_stats_workspace_size.argtypes = [sz]
    L.acm_reprojection_stats_workspace_size.restype = sz
    L.acm_reprojection_stats_merge.argtypes = [sz, ctypes.POINTER(ctypes.c_double),
                                               ctypes.POINTER(ctypes.c_double)]
    L.acm_reprojection_stats_merge.restype = i
    L.acm_error_stats_workspace_size.argtypes = [sz]
    L.acm_error_stats_workspace_size.restype = sz
    L.acm_error_stats.argtypes = [sz, vp, vp, vp, sz, vp]
    L.acm_error_stats.restype = i
    L.acm_reprojection_stats.argtypes = [cam_p, sz, vp, i, vp, vp, vp, vp, sz, vp]
    L.acm_reprojection_stats.restype = i
    L.acm_project_unproject.argtypes = [cam_p, sz, vp, i, vp, vp, vp, vp, vp]
    L.acm_project_unproject.restype = i
    L.acm_reprojection_error_workspace_size.argtypes = [sz]
    L.acm_reprojection_error_workspace_size.restype = sz
    L.acm_reprojection_error.argtypes = [cam_p, sz, vp, i, vp, vp, vp, vp, sz, vp]
    L.acm_reprojection_error.restype = i
    L.acm_linear_estimation_with_error_workspace_size.argtypes = [i, sz]
    L.acm_linear_estimation_with_error_workspace_size.restype = sz
    L.acm_linear_estimation_with_error.argtypes = [cam_p, sz, vp, i, vp, vp, vp, sz, vp]
    L.acm_linear_estimation_with_error.restype = i
    L.acm_linear_estimation_with_error_async.argtypes = [cam_p, sz, vp, i, vp, vp, vp, vp, sz, vp]
    L.acm_linear_estimation_with_error_async.restype = i
    L.acm_sample_points_grid.argtypes = [ctypes.c_uint32, ctypes.c_uint32, sz,
                                         ctypes.POINTER(ctypes.c_uint32),
                                         ctypes.POINTER(ctypes.c_uint32)]
    L.acm_sample_points_grid.restype = i
    L.acm_sample_points_workspace_size.argtypes = [cam_p, sz]
    L.acm_sample_points_workspace_size.restype = sz
    L.acm_sample_points.argtypes = [cam_p, sz, vp, vp, vp, vp, sz, vp]
    L.acm_sample_points.restype = i
    L.acm_sample_points_range.argtypes = [cam_p, sz, sz, sz, vp, vp, vp, vp, sz, vp]
    L.acm_sample_points_range.restype = i
    L.acm_sample_points_ex.argtypes = [cam_p, sz, sz, sz, i, vp, vp, vp, vp, sz, vp]
    L.acm_sample_points_ex.restype = i
    L.acm_sample_points_certificate.argtypes = [cam_p, ctypes.POINTER(ctypes.c_double)]
    L.acm_sample_points_certificate.restype = i
    L.acm_unproject_certificate.argtypes = [cam_p, ctypes.POINTER(ctypes.c_double)]
    L.acm_unproject_certificate.restype = i
    L.acm_sample_points_ray_poly.argtypes = [cam_p, ctypes.POINTER(ctypes.c_double)]
    L.acm_sample_points_ray_poly.restype = i
    L.acm_sample_points_ray_fit.argtypes = [cam_p, ctypes.POINTER(ctypes.c_double)]
    L.acm_sample_points_ray_fit.restype = i
    L.acm_linear_system_columns.argtypes = [i]
    L.acm_linear_system_columns.restype = i
    L.acm_linear_system_qr_workspace_size.argtypes = [i, sz]
    L.acm_linear_system_qr_workspace_size.restype = sz
    L.acm_linear_system_qr.argtypes = [cam_p, sz, vp, i, vp, vp, vp, vp, sz, vp]
    L.acm_linear_system_qr.restype = i
    L.acm_linear_estimation_workspace_size.argtypes = [i, sz]
    L.acm_linear_estimation_workspace_size.restype = sz
    L.acm_linear_estimation.argtypes = [cam_p, sz, vp, i, vp, vp, sz, vp]
    L.acm_linear_estimation.restype = i
    L.acm_linear_system_r_merge.argtypes = [i, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_double)]
    L.acm_linear_system_r_merge.restype = i
    L.acm_linear_estimation_solve.argtypes = [cam_p, sz, ctypes.POINTER(ctypes.c_double), i]
    L.acm_linear_estimation_solve.restype = i
    L.acm_fov_grid_workspace_size.argtypes = [sz]
    L.acm_fov_grid_workspace_size.restype = sz
    L.acm_fov_grid_errors.argtypes = [cam_p, sz, vp, i, vp, vp, vp, sz, vp]
    L.acm_fov_grid_errors.restype = i
    L.acm_fov_grid_select.argtypes = [cam_p, ctypes.POINTER(ctypes.c_double)]
    L.acm_fov_grid_select.restype = i
    L.acm_lm_default_config.argtypes = [ctypes.POINTER(LmConfig)]
    L.acm_lm_default_config.restype = None
    L.acm_lm_workspace_size.argtypes = [i, sz]
    L.acm_lm_workspace_size.restype = sz
    L.acm_lm_optimize.argtypes = [cam_p, sz, vp, i, vp, ctypes.POINTER(LmConfig), ALLREDUCE_FN,
                                  vp, ctypes.POINTER(LmSummary), vp, sz, vp]
    L.acm_lm_optimize.restype = i
    grid_p = ctypes.POINTER(CellGrid)
    L.acm_normal_equations_cells.argtypes = [cam_p, sz, vp, i, vp, grid_p, i, vp, vp, sz, vp]
    L.acm_normal_equations_cells.restype = i
    L.acm_lm_optimize_cells.argtypes = [cam_p, sz, vp, i, vp, grid_p, ctypes.POINTER(LmConfig),
                                        ALLREDUCE_FN, vp, ctypes.POINTER(LmSummary), vp, sz, vp]
    L.acm_lm_optimize_cells.restype = i
    L.acm_sample_points_cells.argtypes = [cam_p, sz, sz, sz, i, vp, vp, vp, vp, vp, sz, vp]
    L.acm_sample_points_cells.restype = i
    L.acm_reprojection_error_cells.argtypes = [cam_p, sz, vp, i, vp, grid_p, vp, vp, vp, sz, vp]
    L.acm_reprojection_error_cells.restype = i
    L.acm_linear_estimation_with_error_cells_async.argtypes = [cam_p, sz, vp, i, vp, vp, grid_p,
                                                              vp, vp, vp, sz, vp]
    L.acm_linear_estimation_with_error_cells_async.restype = i
    coll_p = ctypes.POINTER(AcmCollective)
    L.acm_rccl_available.argtypes = []
    L.acm_rccl_available.restype = i
    L.acm_rccl_unique_id.argtypes = [vp]
    L.acm_rccl_unique_id.restype = i
    L.acm_rccl_init.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, coll_p]
    L.acm_rccl_init.restype = i
    L.acm_rccl_destroy.argtypes = [coll_p]
    L.acm_rccl_destroy.restype = i
    L.acm_linear_estimation_with_error_sharded_workspace_size.argtypes = [i, sz, ctypes.c_int32]
    L.acm_linear_estimation_with_error_sharded_workspace_size.restype = sz
    L.acm_linear_estimation_with_error_sharded.argtypes = [cam_p, sz, vp, i, vp, vp, grid_p, vp,
                                                           vp, coll_p, vp, sz, vp]
    L.acm_linear_estimation_with_error_sharded.restype = i
    L.acm_reprojection_error_sharded_workspace_size.argtypes = [sz, ctypes.c_int32]
    L.acm_reprojection_error_sharded_workspace_size.restype = sz
    L.acm_reprojection_error_sharded.argtypes = [cam_p, sz, vp, i, vp, vp, grid_p, vp, vp, coll_p,
                                                 vp, sz, vp]
    L.acm_reprojection_error_sharded.restype = i
    L.acm_median_workspace_size.argtypes = [sz]
    L.acm_median_workspace_size.restype = sz
    L.acm_median_valid.argtypes = [sz, vp, vp, ctypes.c_uint64, vp, vp, sz, vp]
    L.acm_median_valid.restype = i
    L.acm_median_valid_allreduce.argtypes = [sz, vp, vp, ctypes.c_uint64, vp, vp, sz,
                                             ALLREDUCE_FN, vp, vp]
    L.acm_median_valid_allreduce.restype = i
    L.acm_undistort_image.argtypes = [cam_p, ctypes.POINTER(ctypes.c_double), i, vp, vp, vp]
    L.acm_undistort_image.restype = i
    L.acm_set_device.argtypes = [i]
    L.acm_set_device.restype = i
    L.acm_device_malloc.argtypes = [ctypes.POINTER(vp), sz]
    L.acm_device_malloc.restype = i
    L.acm_device_free.argtypes = [vp]
    L.acm_device_free.restype = i
    L.acm_memcpy_htod.argtypes = [vp, vp, sz, vp]
    L.acm_memcpy_htod.restype = i
    L.acm_memcpy_dtoh.argtypes = [vp, vp, sz, vp]
    L.acm_memcpy_dtoh.restype = i
    L.acm_stream_synchronize.argtypes = [vp]
    L.acm_stream_synchronize.restype = i
    L.acm_set_tuning.argtypes = [i, i]
    L.acm_set_tuning.restype = i
    L.acm_last_hip_error.argtypes = []
    L.acm_last_hip_error.restype = i
    L.acm_last_error.argtypes = []
    L.acm_last_error.restype = ctypes.c_char_p
    L.acm_version.argtypes = []
    L.acm_version.restype = ctypes.c_char_p
    _lib = L
    return L


def check(rc: int) -> int:
    if rc < 0:
        msg = load().acm_last_error().decode(errors="replace")
        raise AcmError(rc, msg)
    return rc


def last_error() -> str:
    return load().acm_last_error().decode(errors="replace")
