"""CPU parity oracle for the batched camera-model hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg, as the checker / the timed CPU
restatement.  The product path (``libacm.so`` and the ``apex_camera_models``
package) never imports or links this module.

Thin numpy/ctypes wrapper over ``oracle/build/liboracle.so`` (built from
``oracle/acm_oracle.c`` by ``oracle/Makefile``), an operation-for-operation C
restatement of the reference's Rust per-point code (file:line citations in the
C source).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
# -O3 build of the same source: the timed CPU baseline (bench.py cpu_baseline)
_LIB_O3_PATH = os.path.join(_HERE, "build", "liboracle_o3.so")

PINHOLE, RADTAN, KB, DS, UCM, EUCM, FOV = range(7)
NUM_PARAMS = {PINHOLE: 4, RADTAN: 9, KB: 8, DS: 6, UCM: 5, EUCM: 6, FOV: 5}

_libs = {}


def build() -> str:
    """Compile liboracle.so and liboracle_o3.so (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib(opt: str = "O2"):
    """The oracle library: opt="O2" (the parity checker) or "O3" (the same
    source at -O3, the timed CPU baseline)."""
    path = _LIB_O3_PATH if opt == "O3" else _LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        dp = ctypes.POINTER(ctypes.c_double)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        sz = ctypes.c_size_t
        u32 = ctypes.c_uint32
        L.oracle_project_jacobian.argtypes = [ctypes.c_int, dp, u32, u32, dp, dp, dp]
        L.oracle_project_jacobian.restype = ctypes.c_int
        L.oracle_unproject.argtypes = [ctypes.c_int, dp, u32, u32, dp, dp]
        L.oracle_unproject.restype = ctypes.c_int
        L.oracle_project_batch.argtypes = [ctypes.c_int, dp, u32, u32, sz, dp, dp, u8p, dp]
        L.oracle_project_batch.restype = None
        L.oracle_unproject_batch.argtypes = [ctypes.c_int, dp, u32, u32, sz, dp, dp, u8p]
        L.oracle_unproject_batch.restype = None
        L.oracle_residual_jacobian_batch.argtypes = [
            ctypes.c_int, dp, u32, u32, sz, dp, dp, ctypes.c_int, dp, dp, u8p]
        L.oracle_residual_jacobian_batch.restype = None
        L.oracle_normal_equations.argtypes = [
            ctypes.c_int, dp, u32, u32, sz, dp, dp, ctypes.c_int, dp, dp, dp,
            ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_normal_equations.restype = None
        L.oracle_reprojection_error.argtypes = [ctypes.c_int, dp, u32, u32, sz, dp, dp, dp]
        L.oracle_reprojection_error.restype = sz
        L.oracle_sample_points.argtypes = [ctypes.c_int, dp, u32, u32, sz, sz, dp, dp,
                                           ctypes.POINTER(sz)]
        L.oracle_sample_points.restype = sz
        L.oracle_linear_estimation_system.argtypes = [ctypes.c_int, dp, sz, dp, dp, dp, dp]
        L.oracle_linear_estimation_system.restype = ctypes.c_int
        L.oracle_fov_grid_search.argtypes = [dp, sz, dp, dp, dp, dp]
        L.oracle_fov_grid_search.restype = ctypes.c_double
        L.oracle_undistort_image.argtypes = [ctypes.c_int, dp, u32, u32, dp, ctypes.c_int,
                                             u8p, u8p]
        L.oracle_undistort_image.restype = None
        _libs[path] = L
    return _libs[path]


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _u8p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def project(model, params, w, h, xyz, want_jac=False):
    """Batch project.  xyz (N,3) -> uv (N,2), status (N,) u8, jac (P, N, 2) or None.

    jac memory layout equals nalgebra's 2N x P column-major DMatrix.
    """
    params = _f64(params)
    xyz = _f64(xyz).reshape(-1, 3)
    n = xyz.shape[0]
    P = NUM_PARAMS[model]
    uv = np.empty((n, 2))
    st = np.empty(n, dtype=np.uint8)
    jac = np.empty((P, n, 2)) if want_jac else None
    lib().oracle_project_batch(model, _dp(params), w, h, n, _dp(xyz), _dp(uv), _u8p(st),
                               _dp(jac) if want_jac else None)
    return uv, st, jac


def unproject(model, params, w, h, uv):
    params = _f64(params)
    uv = _f64(uv).reshape(-1, 2)
    n = uv.shape[0]
    xyz = np.empty((n, 3))
    st = np.empty(n, dtype=np.uint8)
    lib().oracle_unproject_batch(model, _dp(params), w, h, n, _dp(uv), _dp(xyz), _u8p(st))
    return xyz, st


def residual_jacobian(model, params, w, h, xyz, uv_obs, policy=0, want_jac=True):
    params = _f64(params)
    xyz = _f64(xyz).reshape(-1, 3)
    uv_obs = _f64(uv_obs).reshape(-1, 2)
    n = xyz.shape[0]
    P = NUM_PARAMS[model]
    res = np.empty((n, 2))
    jac = np.empty((P, n, 2)) if want_jac else None
    st = np.empty(n, dtype=np.uint8)
    lib().oracle_residual_jacobian_batch(model, _dp(params), w, h, n, _dp(xyz), _dp(uv_obs),
                                         policy, _dp(res), _dp(jac) if want_jac else None,
                                         _u8p(st))
    return res, jac, st


def normal_equations(model, params, w, h, xyz, uv_obs, policy=0):
    params = _f64(params)
    xyz = _f64(xyz).reshape(-1, 3)
    uv_obs = _f64(uv_obs).reshape(-1, 2)
    P = NUM_PARAMS[model]
    JtJ = np.empty((P, P))
    Jtr = np.empty(P)
    cost = ctypes.c_double()
    nv = ctypes.c_uint64()
    lib().oracle_normal_equations(model, _dp(params), w, h, xyz.shape[0], _dp(xyz),
                                  _dp(uv_obs), policy, _dp(JtJ), _dp(Jtr),
                                  ctypes.byref(cost), ctypes.byref(nv))
    return JtJ, Jtr, cost.value, nv.value


def reprojection_error(model, params, w, h, xyz, uv):
    """Returns (stats dict, n_valid); stats None when no projection succeeded."""
    params = _f64(params)
    xyz = _f64(xyz).reshape(-1, 3)
    uv = _f64(uv).reshape(-1, 2)
    out = np.empty(6)
    m = lib().oracle_reprojection_error(model, _dp(params), w, h, xyz.shape[0], _dp(xyz),
                                        _dp(uv), _dp(out))
    if m == 0:
        return None, 0
    keys = ("rmse", "min", "max", "mean", "stddev", "median")
    return dict(zip(keys, out.tolist())), m


def sample_points(model, params, w, h, n):
    """Returns (uv (M,2), xyz (M,3), grid_total)."""
    params = _f64(params)
    width, height = float(w), float(h)
    ncx = int(round(np.sqrt(n * (width / height))))
    ncy = int(round(np.sqrt(n * (height / width))))
    cap = max(ncx * ncy, 1)
    uv = np.empty((cap, 2))
    xyz = np.empty((cap, 3))
    total = ctypes.c_size_t()
    m = lib().oracle_sample_points(model, _dp(params), w, h, n, cap, _dp(uv), _dp(xyz),
                                   ctypes.byref(total))
    return uv[:m].copy(), xyz[:m].copy(), total.value


def linear_estimation_system(model, params, xyz, uv):
    params = _f64(params)
    xyz = _f64(xyz).reshape(-1, 3)
    uv = _f64(uv).reshape(-1, 2)
    n = xyz.shape[0]
    A = np.zeros((2 * n, 4))
    b = np.zeros(2 * n)
    k = lib().oracle_linear_estimation_system(model, _dp(params), n, _dp(xyz), _dp(uv),
                                              _dp(A), _dp(b))
    if k < 0:
        return None, None, k
    return A.reshape(-1)[: 2 * n * k].reshape(2 * n, k).copy(), b, k


def fov_grid_search(params, xyz, uv):
    """FOV linear_estimation grid search (fov.rs:153-251).  Returns
    (best_w or None if n < 2, error_sum (290,), valid_count (290,))."""
    params = _f64(params)
    xyz = _f64(xyz).reshape(-1, 3)
    uv = _f64(uv).reshape(-1, 2)
    s = np.zeros(290)
    c = np.zeros(290)
    w = lib().oracle_fov_grid_search(_dp(params), xyz.shape[0], _dp(xyz), _dp(uv), _dp(s),
                                     _dp(c))
    return (None if w < 0 else w), s, c


FOV_GRID = np.arange(10, 300) / 100.0


def undistort_image(model, params, w, h, target, bilinear, img):
    """img: (h, w, 3) uint8 -> (h, w, 3) uint8 (src/util/undistort.rs:14-49)."""
    params = _f64(params)
    target = _f64(target)
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.empty_like(img)
    lib().oracle_undistort_image(model, _dp(params), w, h, _dp(target), int(bilinear),
                                 _u8p(img), _u8p(out))
    return out
