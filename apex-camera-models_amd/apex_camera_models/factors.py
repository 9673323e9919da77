"""Batched drop-in for apex-solver's `*CameraParamsFactor`.

The reference registers ONE residual block per conversion holding all N
correspondences (bin/camera_converter.rs:378-382, :513, :652, :794, :925,
:1058): `XCameraParamsFactor::new(points_3d.clone(), points_2d.clone())`.
Each LM iteration linearises it: residual (2N) and dense Jacobian (2N x P)
with respect to the camera parameter vector (factor order).  apex-solver
0.1.5's source is not in the image, so the conventions are documented, not
pinned: r = project(p_i; params) - uv_i, J = d project / d params, and
invalid points follow `invalid_policy` (see include/acm.h).

`linearize` materialises r and J (the factor surface); `normal_equations`
is the fused MI355X form the LM driver uses (JtJ, Jtr, cost without writing
r or J to HBM).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .camera import (CameraModel, DoubleSphereModel, EucmModel, FovModel, KannalaBrandtModel,
                     PinholeModel, RadTanModel, UcmModel, Intrinsics, Resolution, _as_device_f64,
                     _stream_handle)


class CameraParamsFactor:
    MODEL: type = CameraModel

    def __init__(self, points_3d, points_2d, resolution: Resolution = None,
                 invalid_policy: int = _lib.INVALID_SKIP):
        self.points_3d = _as_device_f64(points_3d, 3)
        self.points_2d = _as_device_f64(points_2d, 2)
        if self.points_3d.shape[0] != self.points_2d.shape[0]:
            raise ValueError("Number of 2D and 3D points must match")
        self.resolution = resolution or Resolution(0, 0)
        self.invalid_policy = invalid_policy
        self._ws = None

    @property
    def num_points(self) -> int:
        return self.points_3d.shape[0]

    def _camera(self, params):
        params = [float(p) for p in params]
        m = self.MODEL._from_params(params, self.resolution)
        return m.acm_camera()

    def linearize(self, params, compute_jacobian: bool = True):
        """Returns (residual (2N,), jacobian (2N, P) column-major view or None)."""
        n = self.num_points
        P = self.MODEL.NUM_PARAMS
        dev = self.points_3d.device
        res = torch.empty((n, 2), dtype=torch.float64, device=dev)
        jac = (torch.empty((P, n, 2), dtype=torch.float64, device=dev)
               if compute_jacobian else None)
        cam = self._camera(params)
        _lib.check(_lib.load().acm_residual_jacobian(
            ctypes.byref(cam), n, self.points_3d.data_ptr(), _lib.LAYOUT_AOS,
            self.points_2d.data_ptr(), self.invalid_policy, res.data_ptr(),
            jac.data_ptr() if jac is not None else None, None, _stream_handle()))
        r = res.reshape(-1)
        J = jac.reshape(P, 2 * n).t() if jac is not None else None  # (2N, P), col-major
        return r, J

    def normal_equations(self, params, result: torch.Tensor = None):
        """Fused JtJ (P,P), Jtr (P,), cost = 0.5*sum r^2, n_valid -- on device."""
        n = self.num_points
        P = self.MODEL.NUM_PARAMS
        L = _lib.load()
        need = L.acm_normal_equations_workspace_size(self.MODEL.MODEL_ID, n)
        if self._ws is None or self._ws.numel() * 8 < need:
            self._ws = torch.empty(((need + 7) // 8,), dtype=torch.float64,
                                   device=self.points_3d.device)
        if result is None:
            result = torch.empty((P * P + P + 2,), dtype=torch.float64,
                                 device=self.points_3d.device)
        cam = self._camera(params)
        _lib.check(L.acm_normal_equations(
            ctypes.byref(cam), n, self.points_3d.data_ptr(), _lib.LAYOUT_AOS,
            self.points_2d.data_ptr(), self.invalid_policy, result.data_ptr(),
            self._ws.data_ptr(), self._ws.numel() * 8, _stream_handle()))
        return result

    @staticmethod
    def unpack_normal_equations(result: torch.Tensor, P: int):
        JtJ = result[: P * P].reshape(P, P)
        Jtr = result[P * P: P * P + P]
        cost = result[P * P + P]
        n_valid = result[P * P + P + 1]
        return JtJ, Jtr, cost, n_valid


class PinholeCameraParamsFactor(CameraParamsFactor):
    MODEL = PinholeModel


class RadTanCameraParamsFactor(CameraParamsFactor):
    MODEL = RadTanModel


class KannalaBrandtCameraParamsFactor(CameraParamsFactor):
    MODEL = KannalaBrandtModel


class DoubleSphereCameraParamsFactor(CameraParamsFactor):
    MODEL = DoubleSphereModel


class UcmCameraParamsFactor(CameraParamsFactor):
    MODEL = UcmModel


class EucmCameraParamsFactor(CameraParamsFactor):
    MODEL = EucmModel


class FovCameraParamsFactor(CameraParamsFactor):
    MODEL = FovModel


__all__ = [
    "CameraParamsFactor", "PinholeCameraParamsFactor", "RadTanCameraParamsFactor",
    "KannalaBrandtCameraParamsFactor", "DoubleSphereCameraParamsFactor",
    "UcmCameraParamsFactor", "EucmCameraParamsFactor", "FovCameraParamsFactor", "Intrinsics",
]
