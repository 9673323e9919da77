"""apex_camera_models -- MI355X-native drop-in for the reference crate's hot path.

Module layout mirrors the reference crate (`apex_camera_models::camera`,
`::util`, and apex-solver's `factors`).  Every numeric operation runs in the
HIP kernels of libacm.so (gfx950) through its C-ABI (include/acm.h); importing
this package loads that library and raises if it is missing.
"""
from . import _lib

_lib.load()  # fail loudly at import if the HIP extension is not built

from . import camera, factors, util  # noqa: E402
from .camera import (CameraModel, CameraModelError, DoubleSphereModel, EucmModel,  # noqa: E402
                     FovModel, Intrinsics, KannalaBrandtModel, PinholeModel, RadTanModel,
                     Resolution, UcmModel)

__all__ = [
    "camera", "factors", "util", "CameraModel", "CameraModelError", "DoubleSphereModel",
    "EucmModel", "FovModel", "Intrinsics", "KannalaBrandtModel", "PinholeModel", "RadTanModel",
    "Resolution", "UcmModel",
]
