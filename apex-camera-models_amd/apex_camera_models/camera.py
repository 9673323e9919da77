"""Host-side mirror of the reference's `camera` module over libacm.so.

Mirrors /root/reference/src/camera/mod.rs: the `CameraModel` trait
(:241-340), `Intrinsics` (:53-62), `Resolution` (:68-73), `CameraModelError`
(:80-113), `validation::validate_intrinsics` (:362-371) and the model structs
(pinhole.rs, rad_tan.rs, kannala_brandt.rs, double_sphere.rs, ucm.rs,
eucm.rs, fov.rs) with the same names, argument meaning and error behaviour.

The reference's per-point `project`/`unproject` return `Result`; here
`project(point)` / `unproject(point)` raise the matching `CameraModelError`
subclass.  The batched drop-in (`project_batch`, `unproject_batch`) takes and
returns device tensors and a per-point status vector instead of `Result`s.
All numerics run in the HIP kernels of libacm.so; this module only marshals.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib

# ------------------------------------------------------------------ errors


class CameraModelError(Exception):
    """Base of the CameraModelError variants (src/camera/mod.rs:80-113)."""


class ProjectionOutSideImage(CameraModelError):
    def __init__(self):
        super().__init__("Projection is outside the image")


class PointIsOutSideImage(CameraModelError):
    def __init__(self):
        super().__init__("Input point is outside the image")


class PointAtCameraCenter(CameraModelError):
    def __init__(self):
        super().__init__("z is close to zero, point is at camera center")


class FocalLengthMustBePositive(CameraModelError):
    def __init__(self):
        super().__init__("Focal length must be positive")


class PrincipalPointMustBeFinite(CameraModelError):
    def __init__(self):
        super().__init__("Principal point must be finite")


class InvalidParams(CameraModelError):
    def __init__(self, msg: str):
        super().__init__(f"Invalid camera parameters: {msg}")
        self.msg = msg


class YamlError(CameraModelError):
    def __init__(self, msg: str):
        super().__init__(f"Failed to load YAML: {msg}")


class IOError_(CameraModelError):
    def __init__(self, msg: str):
        super().__init__(f"IO Error: {msg}")


class NumericalError(CameraModelError):
    def __init__(self, msg: str = "numerical error"):
        super().__init__(f"NumericalError: {msg}")


STATUS_OK = 0
STATUS_PROJECTION_OUT_SIDE_IMAGE = 1
STATUS_POINT_IS_OUT_SIDE_IMAGE = 2
STATUS_POINT_AT_CAMERA_CENTER = 3
STATUS_NUMERICAL_ERROR = 4


def status_to_error(code: int) -> Optional[CameraModelError]:
    if code == STATUS_OK:
        return None
    if code == STATUS_PROJECTION_OUT_SIDE_IMAGE:
        return ProjectionOutSideImage()
    if code == STATUS_POINT_IS_OUT_SIDE_IMAGE:
        return PointIsOutSideImage()
    if code == STATUS_POINT_AT_CAMERA_CENTER:
        return PointAtCameraCenter()
    return NumericalError("point failed to (un)project")


# ------------------------------------------------------------ value types


@dataclass
class Intrinsics:
    fx: float
    fy: float
    cx: float
    cy: float


@dataclass
class Resolution:
    width: int
    height: int


class validation:  # noqa: N801  (mirrors `pub mod validation`)
    @staticmethod
    def validate_intrinsics(intr: Intrinsics) -> None:
        """src/camera/mod.rs:362-371."""
        if intr.fx <= 0.0 or intr.fy <= 0.0:
            raise FocalLengthMustBePositive()
        if not math.isfinite(intr.cx) or not math.isfinite(intr.cy):
            raise PrincipalPointMustBeFinite()


def _as_device_f64(t, cols: int) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(t, dtype=torch.float64)
    if t.device.type != "cuda":
        t = t.to("cuda")
    t = t.to(torch.float64).reshape(-1, cols).contiguous()
    return t


def _stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


# ------------------------------------------------------------------ trait


class CameraModel:
    """Mirror of `pub trait CameraModel` (src/camera/mod.rs:241-340)."""

    MODEL_ID: int = -1
    NAME: str = ""
    NUM_PARAMS: int = 0
    _VALIDATE_IN_NEW = False  # Pinhole / RadTan run validate_params in new()

    def __init__(self, intrinsics: Intrinsics, resolution: Resolution):
        self.intrinsics = intrinsics
        self.resolution = resolution

    # --- construction (XModel::new(&DVector)) ----------------------------
    @classmethod
    def new(cls, parameters: Sequence[float]):
        parameters = [float(p) for p in parameters]
        if len(parameters) != cls.NUM_PARAMS:
            raise InvalidParams(f"Expected {cls.NUM_PARAMS} parameters, got {len(parameters)}")
        m = cls._from_params(parameters, Resolution(0, 0))
        if cls._VALIDATE_IN_NEW:
            m.validate_params()
        return m

    @classmethod
    def _from_params(cls, params: List[float], res: Resolution):
        raise NotImplementedError

    def _distortion_params(self) -> List[float]:
        raise NotImplementedError

    # --- trait surface ---------------------------------------------------
    def params(self) -> List[float]:
        """Factor-order parameter vector (camera_converter.rs:385-392 & co)."""
        i = self.intrinsics
        return [i.fx, i.fy, i.cx, i.cy] + list(self._distortion_params())

    def get_resolution(self) -> Resolution:
        return Resolution(self.resolution.width, self.resolution.height)

    def get_intrinsics(self) -> Intrinsics:
        i = self.intrinsics
        return Intrinsics(i.fx, i.fy, i.cx, i.cy)

    def get_distortion(self) -> List[float]:
        return list(self._distortion_params())

    def get_model_name(self) -> str:
        return self.NAME

    def validate_params(self) -> None:
        validation.validate_intrinsics(self.intrinsics)

    # --- C-ABI camera ----------------------------------------------------
    def acm_camera(self) -> _lib.AcmCamera:
        cam = _lib.AcmCamera()
        cam.model = self.MODEL_ID
        cam.width = int(self.resolution.width) & 0xFFFFFFFF
        cam.height = int(self.resolution.height) & 0xFFFFFFFF
        cam.num_params = self.NUM_PARAMS
        for k, p in enumerate(self.params()):
            cam.params[k] = p
        return cam

    # --- batched drop-in (device tensors) --------------------------------
    def project_batch(self, points_3d, jacobian: bool = False, layout: str = "aos",
                      out: Optional[Tuple[torch.Tensor, ...]] = None, exact: bool = False):
        """Batched `CameraModel::project` (mod.rs:256) (+ dense 2N x P Jacobian).

        points_3d: (N,3) float64 on the GPU (AoS, = nalgebra Matrix3xX) or, with
        layout="soa", (3,N).  Returns (uv (N,2), status (N,) uint8, jac) where
        jac is (P,N,2) -- memory identical to a 2N x P column-major DMatrix --
        or None.  Failed points: uv = NaN, J = 0, status = error code.
        A float32 input tensor selects the f32 kernels (acm_project_f32).
        exact=True: ACM_EXACT_MATH (reference-exact KB / FOV math, include/acm.h).
        """
        lay = _lib.LAYOUT_SOA if layout == "soa" else _lib.LAYOUT_AOS
        pts = points_3d if isinstance(points_3d, torch.Tensor) else torch.as_tensor(
            points_3d, dtype=torch.float64)
        dt = torch.float32 if pts.dtype == torch.float32 else torch.float64
        pts = pts.to("cuda", dt)
        if lay == _lib.LAYOUT_SOA:
            pts = pts.reshape(3, -1).contiguous()
            n = pts.shape[1]
        else:
            pts = pts.reshape(-1, 3).contiguous()
            n = pts.shape[0]
        if out is not None:
            uv, st, jac = out
        else:
            uv = torch.empty((n, 2), dtype=dt, device=pts.device)
            st = torch.empty((n,), dtype=torch.uint8, device=pts.device)
            jac = (torch.empty((self.NUM_PARAMS, n, 2), dtype=dt, device=pts.device)
                   if jacobian else None)
        cam = self.acm_camera()
        fn = _lib.load().acm_project_f32 if dt == torch.float32 else _lib.load().acm_project
        if exact and dt == torch.float64:
            lay |= _lib.EXACT_MATH
        _lib.check(fn(ctypes.byref(cam), n, pts.data_ptr(), lay, uv.data_ptr(), st.data_ptr(),
                      jac.data_ptr() if jac is not None else None, _stream_handle()))
        return uv, st, jac

    def unproject_batch(self, points_2d, layout: str = "aos", reference_newton: bool = False,
                        out: Optional[Tuple[Optional[torch.Tensor], ...]] = None):
        """Batched `CameraModel::unproject` (mod.rs:271).  Returns (rays, status).
        reference_newton=True: ACM_REFERENCE_NEWTON for this call (the
        reference's own Newton loops; include/acm.h).  out = (rays, status):
        preallocated outputs (either may be None)."""
        uv = _as_device_f64(points_2d, 2)
        n = uv.shape[0]
        lay = _lib.LAYOUT_SOA if layout == "soa" else _lib.LAYOUT_AOS
        if reference_newton:
            lay |= _lib.REFERENCE_NEWTON
        rays, st = out if out is not None else (None, None)
        if rays is None:
            rays = torch.empty((n, 3) if layout != "soa" else (3, n), dtype=torch.float64,
                               device=uv.device)
        if st is None:
            st = torch.empty((n,), dtype=torch.uint8, device=uv.device)
        cam = self.acm_camera()
        _lib.check(_lib.load().acm_unproject(ctypes.byref(cam), n, uv.data_ptr(),
                                              rays.data_ptr(), lay, st.data_ptr(),
                                              _stream_handle()))
        return rays, st

    def project_unproject_batch(self, points_3d, layout: str = "aos"):
        """Project then unproject every point in one pass (acm_project_unproject;
        the per-point loop of tests/projection_accuracy.rs:49-73 over
        mod.rs:256 and :271, BASELINE config 4).  Returns (uv, status, rays,
        ray_status): the pixels as project_batch writes them (NaN for failed
        projections) and the unprojection of those same pixels."""
        lay = _lib.LAYOUT_SOA if layout == "soa" else _lib.LAYOUT_AOS
        if lay == _lib.LAYOUT_AOS:
            pts = _as_device_f64(points_3d, 3)
        else:
            pts = torch.as_tensor(points_3d, dtype=torch.float64).to("cuda").reshape(
                3, -1).contiguous()
        n = pts.shape[0] if lay == _lib.LAYOUT_AOS else pts.shape[1]
        uv = torch.empty((n, 2), dtype=torch.float64, device=pts.device)
        st = torch.empty((n,), dtype=torch.uint8, device=pts.device)
        rays = torch.empty((n, 3) if lay == _lib.LAYOUT_AOS else (3, n), dtype=torch.float64,
                           device=pts.device)
        st2 = torch.empty((n,), dtype=torch.uint8, device=pts.device)
        cam = self.acm_camera()
        _lib.check(_lib.load().acm_project_unproject(ctypes.byref(cam), n, pts.data_ptr(), lay,
                                                      uv.data_ptr(), st.data_ptr(),
                                                      rays.data_ptr(), st2.data_ptr(),
                                                      _stream_handle()))
        return uv, st, rays, st2

    # --- linear_estimation (GPU TSQR + host k x k SVD solve) ---------------
    def linear_estimation(self, points_3d, points_2d) -> None:
        """`XModel::linear_estimation(&Matrix3xX, &Matrix2xX)` (kannala_brandt.rs:164-272,
        double_sphere.rs:225-290, ucm.rs:200-258, eucm.rs:216-288, rad_tan.rs:153-234).
        Updates the distortion parameters in place; raises InvalidParams /
        NumericalError like the reference."""
        L = _lib.load()
        p3 = _as_device_f64(points_3d, 3)
        p2 = _as_device_f64(points_2d, 2)
        if p3.shape[0] != p2.shape[0]:
            raise InvalidParams("Number of 2D and 3D points must match")
        n = p3.shape[0]
        ws_bytes = L.acm_linear_estimation_workspace_size(self.MODEL_ID, n)
        if ws_bytes == 0:
            raise InvalidParams(f"{self.NAME} has no GPU linear_estimation")
        ws = torch.empty(((ws_bytes + 7) // 8,), dtype=torch.float64, device=p3.device)
        cam = self.acm_camera()
        rc = L.acm_linear_estimation(ctypes.byref(cam), n, p3.data_ptr(), _lib.LAYOUT_AOS,
                                     p2.data_ptr(), ws.data_ptr(), ws_bytes, _stream_handle())
        if rc == _lib.ERR_INVALID_PARAMS:
            raise InvalidParams(_lib.last_error())
        if rc == _lib.ERR_NUMERICAL:
            raise NumericalError(_lib.last_error())
        _lib.check(rc)
        self._set_params(list(cam.params)[: self.NUM_PARAMS])

    def _set_params(self, p: List[float]) -> None:
        upd = self._from_params(p, self.resolution)
        self.__dict__.update({k: v for k, v in upd.__dict__.items() if k != "resolution"})

    # --- per-point reference surface --------------------------------------
    def project(self, point_3d):
        """`fn project(&self, &Vector3) -> Result<Vector2, CameraModelError>`."""
        uv, st, _ = self.project_batch(torch.as_tensor([list(map(float, point_3d))],
                                                       dtype=torch.float64))
        err = status_to_error(int(st[0].item()))
        if err is not None:
            raise err
        return uv[0].cpu().tolist()

    def unproject(self, point_2d):
        """`fn unproject(&self, &Vector2) -> Result<Vector3, CameraModelError>`."""
        rays, st = self.unproject_batch(torch.as_tensor([list(map(float, point_2d))],
                                                        dtype=torch.float64))
        err = status_to_error(int(st[0].item()))
        if err is not None:
            raise err
        return rays[0].cpu().tolist()

    # --- YAML (cam0 format, mod.rs:412-578) -------------------------------
    @classmethod
    def load_from_yaml(cls, path: str):
        from .yaml_io import load_camera_yaml
        return load_camera_yaml(cls, path)

    def save_to_yaml(self, path: str) -> None:
        from .yaml_io import save_camera_yaml
        save_camera_yaml(self, path)

    def __repr__(self):
        i = self.intrinsics
        return (f"{type(self).__name__}[fx: {i.fx} fy: {i.fy} cx: {i.cx} cy: {i.cy} "
                f"distortion: {self.get_distortion()}]")


# ------------------------------------------------------------------ models


class PinholeModel(CameraModel):
    """src/camera/pinhole.rs."""
    MODEL_ID, NAME, NUM_PARAMS = _lib.PINHOLE, "pinhole", 4
    _VALIDATE_IN_NEW = True

    @classmethod
    def _from_params(cls, p, res):
        return cls(Intrinsics(*p[:4]), res)

    def _distortion_params(self):
        return []


class RadTanModel(CameraModel):
    """src/camera/rad_tan.rs; distortions = [k1, k2, p1, p2, k3]."""
    MODEL_ID, NAME, NUM_PARAMS = _lib.RADTAN, "rad_tan", 9
    _VALIDATE_IN_NEW = True

    def __init__(self, intrinsics, resolution, distortions):
        super().__init__(intrinsics, resolution)
        self.distortions = [float(d) for d in distortions]

    @classmethod
    def _from_params(cls, p, res):
        return cls(Intrinsics(*p[:4]), res, p[4:9])

    def _distortion_params(self):
        return list(self.distortions)


class KannalaBrandtModel(CameraModel):
    """src/camera/kannala_brandt.rs; distortions = [k1, k2, k3, k4]."""
    MODEL_ID, NAME, NUM_PARAMS = _lib.KANNALA_BRANDT, "kannala_brandt", 8

    def __init__(self, intrinsics, resolution, distortions):
        super().__init__(intrinsics, resolution)
        self.distortions = [float(d) for d in distortions]

    @classmethod
    def _from_params(cls, p, res):
        return cls(Intrinsics(*p[:4]), res, p[4:8])

    def _distortion_params(self):
        return list(self.distortions)


class DoubleSphereModel(CameraModel):
    """src/camera/double_sphere.rs; get_distortion() = [alpha, xi] (:636-638)."""
    MODEL_ID, NAME, NUM_PARAMS = _lib.DOUBLE_SPHERE, "double_sphere", 6

    def __init__(self, intrinsics, resolution, alpha, xi):
        super().__init__(intrinsics, resolution)
        self.alpha = float(alpha)
        self.xi = float(xi)

    @classmethod
    def _from_params(cls, p, res):
        return cls(Intrinsics(*p[:4]), res, p[4], p[5])

    def _distortion_params(self):
        return [self.alpha, self.xi]

    def validate_params(self):
        """double_sphere.rs:592-607."""
        super().validate_params()
        if self.alpha <= 0.0 or self.alpha > 1.0:
            raise InvalidParams("alpha must be in (0, 1]")
        if not math.isfinite(self.xi):
            raise InvalidParams("xi must be finite")


class UcmModel(CameraModel):
    """src/camera/ucm.rs; distortion = [alpha]."""
    MODEL_ID, NAME, NUM_PARAMS = _lib.UCM, "ucm", 5

    def __init__(self, intrinsics, resolution, alpha):
        super().__init__(intrinsics, resolution)
        self.alpha = float(alpha)

    @classmethod
    def _from_params(cls, p, res):
        return cls(Intrinsics(*p[:4]), res, p[4])

    def _distortion_params(self):
        return [self.alpha]

    def validate_params(self):
        """ucm.rs:467-477."""
        super().validate_params()
        if not math.isfinite(self.alpha):
            raise InvalidParams("alpha must be finite")


class EucmModel(CameraModel):
    """src/camera/eucm.rs; distortion = [alpha, beta]."""
    MODEL_ID, NAME, NUM_PARAMS = _lib.EUCM, "eucm", 6

    def __init__(self, intrinsics, resolution, alpha, beta):
        super().__init__(intrinsics, resolution)
        self.alpha = float(alpha)
        self.beta = float(beta)

    @classmethod
    def _from_params(cls, p, res):
        return cls(Intrinsics(*p[:4]), res, p[4], p[5])

    def _distortion_params(self):
        return [self.alpha, self.beta]

    def validate_params(self):
        """eucm.rs:501-517."""
        super().validate_params()
        if not math.isfinite(self.alpha):
            raise InvalidParams("alpha must be finite")
        if not math.isfinite(self.beta):
            raise InvalidParams("beta must be finite")


class FovModel(CameraModel):
    """src/camera/fov.rs; distortion = [w]."""
    MODEL_ID, NAME, NUM_PARAMS = _lib.FOV, "fov", 5

    def __init__(self, intrinsics, resolution, w):
        super().__init__(intrinsics, resolution)
        self.w = float(w)

    @classmethod
    def _from_params(cls, p, res):
        return cls(Intrinsics(*p[:4]), res, p[4])

    def _distortion_params(self):
        return [self.w]

    def validate_params(self):  # fov.rs:457-468
        super().validate_params()
        if not math.isfinite(self.w) or self.w <= 2.220446049250313e-16 or self.w > 3.0:
            raise InvalidParams(f"w must be in range (epsilon, 3.0], got {self.w}")


MODEL_CLASSES = {
    "pinhole": PinholeModel,
    "rad_tan": RadTanModel,
    "radtan": RadTanModel,
    "kannala_brandt": KannalaBrandtModel,
    "kb": KannalaBrandtModel,
    "double_sphere": DoubleSphereModel,
    "ds": DoubleSphereModel,
    "ucm": UcmModel,
    "eucm": EucmModel,
    "fov": FovModel,
}
