"""CPU-side checks of the drop-in boundary (no GPU needed): libacm.so builds,
loads, exports every ACM_API symbol declared in include/acm.h, and its host
logic (parameter counts, XModel::new / validate_params semantics, argument
validation, sample grid) mirrors the reference."""
import ctypes
import math
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    text = open(os.path.join(ROOT, "include", "acm.h")).read()
    return sorted(set(re.findall(r"ACM_API\s+[\w\s\*]+?\b(acm_\w+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    from apex_camera_models import _lib
    L = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.EXPORTED_SYMBOLS)
    assert b"gfx950" in L.acm_version()


def test_num_params():
    from apex_camera_models import _lib
    L = _lib.load()
    assert [L.acm_num_params(m) for m in range(7)] == [4, 9, 8, 6, 5, 6, 5]
    assert L.acm_num_params(7) == -1


def _init(model, params, w=752, h=480):
    from apex_camera_models import _lib
    cam = _lib.AcmCamera()
    arr = (ctypes.c_double * max(len(params), 1))(*params)
    rc = _lib.load().acm_camera_init(ctypes.byref(cam), model, arr, len(params), w, h)
    return rc, cam


def test_camera_init_param_count_errors():
    # tests/model_conversions.rs:162-169: wrong parameter counts -> InvalidParams
    from apex_camera_models import _lib
    import kat_suite
    from _backends import MODEL_IDS
    cases = [(MODEL_IDS[k["model"]], k["n"]) for k in kat_suite.KATS["param_count_errors"]]
    assert (6, 4) in cases  # fov.rs:750-756
    for model, n in cases:
        rc, _ = _init(model, [500.0] * n)
        assert rc == _lib.ERR_INVALID_PARAMS
    assert "Expected" in _lib.last_error()
    rc, cam = _init(2, [1.0] * 8)
    assert rc == 0 and cam.num_params == 8 and cam.width == 752


def test_camera_init_validates_pinhole_like_reference():
    # tests/model_conversions.rs:172-186 (PinholeModel::new runs validate_params)
    from apex_camera_models import _lib
    for p in ([-500.0, 500.0, 320.0, 240.0], [0.0, 500.0, 320.0, 240.0],
              [500.0, 500.0, math.inf, 240.0], [500.0, 500.0, 320.0, math.nan]):
        rc, _ = _init(0, p)
        assert rc == _lib.ERR_INVALID_PARAMS


def test_validate_params_reference_kats():
    """tests/golden/reference_kats.json "validate_params" (pinhole: the
    reference runs it inside new(); FOV: fov.rs:668-714) through the C-ABI's
    acm_validate_params, whose codes mirror CameraModelError (acm.h)."""
    import kat_suite
    from _backends import MODEL_IDS, parse_params
    from apex_camera_models import _lib
    L = _lib.load()
    code = {"Valid": 0, "FocalLengthMustBePositive": 4, "PrincipalPointMustBeFinite": 5,
            "InvalidParams": 6}
    n_fov = 0
    for k in kat_suite.KATS["validate_params"]:
        p = parse_params(k["params"])
        cam = _lib.AcmCamera()
        cam.model, cam.width, cam.height, cam.num_params = MODEL_IDS[k["model"]], 752, 480, len(p)
        for i, v in enumerate(p):
            cam.params[i] = v
        assert L.acm_validate_params(ctypes.byref(cam)) == code[k["error"]], k["src"]
        n_fov += k["model"] == "fov"
    assert n_fov == 6


def test_validate_params_codes():
    from apex_camera_models import _lib
    L = _lib.load()
    _, cam = _init(3, [350.0, 350.0, 320.0, 240.0, 0.58, -0.18])
    assert L.acm_validate_params(ctypes.byref(cam)) == 0
    cam.params[4] = 0.0  # double_sphere.rs:811-829: alpha must be in (0, 1]
    assert L.acm_validate_params(ctypes.byref(cam)) == 6
    cam.params[4] = 0.5
    cam.params[5] = math.nan  # xi must be finite
    assert L.acm_validate_params(ctypes.byref(cam)) == 6
    cam.params[5] = 0.1
    cam.params[0] = 0.0  # FocalLengthMustBePositive
    assert L.acm_validate_params(ctypes.byref(cam)) == 4


def test_argument_validation_before_any_launch():
    from apex_camera_models import _lib
    L = _lib.load()
    _, cam = _init(2, [1.0] * 8)
    # n == 0 is a no-op success (empty batch), bad layout / model rejected
    assert L.acm_project(ctypes.byref(cam), 0, None, 0, None, None, None, None) == 0
    assert L.acm_project(ctypes.byref(cam), 10, None, 0, None, None, None, None) == \
        _lib.ERR_INVALID_ARGUMENT
    assert L.acm_project(ctypes.byref(cam), 0, None, 7, None, None, None, None) == \
        _lib.ERR_INVALID_ARGUMENT
    cam.model = 42
    assert L.acm_project(ctypes.byref(cam), 0, None, 0, None, None, None, None) == \
        _lib.ERR_INVALID_MODEL
    _, cam = _init(3, [350.0, 350.0, 320.0, 240.0, 0.58, -0.18])
    assert L.acm_normal_equations(ctypes.byref(cam), 100, 1, 0, 1, 0, 1, 1, 8, None) == \
        _lib.ERR_WORKSPACE_TOO_SMALL
    assert L.acm_residual_jacobian(ctypes.byref(cam), 1, 1, 0, 1, 5, 1, None, None, None) == \
        _lib.ERR_INVALID_ARGUMENT


@pytest.mark.parametrize("w,h,n", [(752, 480, 100), (512, 512, 100_000_000), (752, 480, 500),
                                   (752, 480, 2), (640, 480, 1)])
def test_sample_grid_matches_reference_formula(w, h, n):
    # point_sampling.rs:53-54: round(sqrt(n * w/h)) x round(sqrt(n * h/w))
    from apex_camera_models import _lib
    ncx, ncy = ctypes.c_uint32(), ctypes.c_uint32()
    assert _lib.load().acm_sample_points_grid(w, h, n, ctypes.byref(ncx), ctypes.byref(ncy)) == 0
    assert ncx.value == int(round(math.sqrt(n * (w / h))))
    assert ncy.value == int(round(math.sqrt(n * (h / w))))


def test_workspace_sizes():
    from apex_camera_models import _lib
    L = _lib.load()
    D = 8 - 4  # KB: structured normal-equation sums, 10 + 5D + D(D+1)/2 + 2
    K = 10 + 5 * D + D * (D + 1) // 2 + 2
    assert L.acm_normal_equations_workspace_size(2, 10_000_000) == (2048 + 1) * K * 8
    assert L.acm_reprojection_stats_workspace_size(1000) >= 1000 * 8
    assert L.acm_median_workspace_size(10) >= 10 * 8  # candidate buffer sized for n


def test_tuning_knobs_validate_and_restore():
    """acm_set_tuning (benchmark A/B knobs, results identical for every
    setting) rejects out-of-range values and returns the previous value."""
    from apex_camera_models import _lib
    L = _lib.load()
    cases = {_lib.TUNE_PROJECT_VARIANT: ([-1, 0, 1, 2, 3, 4, 5, 6, 7], [-2, 8]),
             _lib.TUNE_RESIDUAL_NT: ([-1, 0, 1], [2]),
             _lib.TUNE_NE_WAVES: ([0, 1, 3, 4], [2, 5]),
             _lib.TUNE_FOV_UNROLL: ([-1, 0, 1, 2, 4], [-2, 3, 5, 8]),
             _lib.TUNE_NE_UNROLL: ([0, 1, 2, 3, 4, 5], [6, -1]),
             _lib.TUNE_ALIGN_J: ([-1, 0, 1], [2]),
             _lib.TUNE_NT_LOADS: ([-1, 0, 1], [2]),
             _lib.TUNE_NT_LOADS_UNPROJECT: ([-1, 0, 1], [2]),
             _lib.TUNE_LM_HOST_RESULT: ([-1, 0, 1, 2, 3], [4, -2]),
             _lib.TUNE_SAMPLE_FUSED: ([-1, 0, 1, 2, 3, 4], [5, -2]),
             _lib.TUNE_UNPROJECT_RCP: ([-1, 0, 1], [2, -2]),
             _lib.TUNE_SAMPLE_CERT: ([-1, 0], [1, -2]),
             _lib.TUNE_SAMPLE_WRITE: ([-1, 1, 2, 3, 4, 5], [6, -2]),
             _lib.TUNE_UNPROJECT_PPT: ([-1, 1, 2, 3], [0, 4, -2]),
             _lib.TUNE_ROUND_TRIP: ([-1, 1, 2, 4, 9, 10, 12, 17, 18, 20], [0, 3, 8, 21, -2])}
    for key, (good, bad) in cases.items():
        first = L.acm_set_tuning(key, good[0])
        assert first >= -1, key
        prev = good[0]
        for v in good[1:]:
            assert L.acm_set_tuning(key, v) == prev, (key, v)
            prev = v
        for v in bad:
            assert L.acm_set_tuning(key, v) == _lib.ERR_INVALID_ARGUMENT, (key, v)
        assert L.acm_set_tuning(key, first) == prev  # a rejected value changed nothing
    assert L.acm_set_tuning(99, 0) == _lib.ERR_INVALID_ARGUMENT
    # numerics are per call since round 3: the old process-wide knob is gone
    assert L.acm_set_tuning(_lib.TUNE_NEWTON_FAST, 0) == _lib.ERR_NOT_SUPPORTED
    # the device-resident LM (r04) is gone since round 5
    assert L.acm_set_tuning(16, 1) == _lib.ERR_NOT_SUPPORTED


def test_tuning_defaults_match_the_header():
    """every knob's default, read in a fresh process as
    the previous value acm_set_tuning returns, equals the one include/acm.h
    documents (its "Defaults (...)" list; r04's header called
    ACM_TUNE_LM_DEVICE's -1 "on" while the code took it as off)."""
    import subprocess
    import sys
    text = open(os.path.join(ROOT, "include", "acm.h")).read()
    block = re.search(r"Defaults \(the value acm_set_tuning returns.*?\):(.*?)\.\n", text,
                      re.S).group(1)
    documented = {k: int(v) for k, v in re.findall(r"([A-Z_]+) (-?\d+)", block)}
    keys = dict(re.findall(r"ACM_TUNE_([A-Z_]+) = (\d+)", text))
    removed = {"NEWTON_FAST", "LM_DEVICE"}
    assert set(documented) == set(keys) - removed, (set(documented) ^ (set(keys) - removed))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from apex_camera_models import _lib\n"
            "L = _lib.load()\n"
            "for k, d in %r:\n"
            "    print(k, L.acm_set_tuning(k, d))\n") % (
                os.path.join(ROOT, "apex-camera-models_amd"),
                sorted((int(keys[name]), d) for name, d in documented.items()))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         check=True, timeout=300).stdout
    got = {int(a): int(b) for a, b in (ln.split() for ln in out.splitlines())}
    for name, default in documented.items():
        assert got[int(keys[name])] == default, (name, got[int(keys[name])], default)


def test_newton_tolerance_threshold_is_exact():
    # camera_models.hpp kNewtonTol2: the RadTan Newton loop (rad_tan.rs:459,
    # :503) tests sqrt(s) < 1e-6; the kernel tests s < kNewtonTol2 instead.
    # Both must agree for every s >= 0 -- check the doubles around the cut.
    import numpy as np
    text = open(os.path.join(ROOT, "apex-camera-models_amd", "csrc", "camera_models.hpp")).read()
    t = float.fromhex(re.search(r"kNewtonTol2 = (0x[0-9a-fp.+-]+);", text).group(1))
    s = np.float64(t)
    for _ in range(64):
        s = np.nextafter(s, 0.0)
    for _ in range(128):
        assert (math.sqrt(float(s)) < 1e-6) == (float(s) < t)
        s = np.nextafter(s, np.inf)
    for v in (0.0, 1e-300, 1e-13, 1e-12, 1.0, math.inf):
        assert (math.sqrt(v) < 1e-6) == (v < t)


def _packed_r(A):
    import numpy as np
    R = np.linalg.qr(A, mode="r")
    R = R * np.sign(np.where(np.diag(R) == 0, 1.0, np.diag(R)))[:, None]
    M = R.shape[0]
    return np.array([R[r, c] for r in range(M) for c in range(r, M)])


@pytest.mark.parametrize("model,k", [(2, 4), (1, 3), (3, 1)])
def test_linear_system_r_merge_is_qr_of_stacked_rows(model, k):
    # the multi-GPU linear_estimation fold: merge(R(A1), R(A2)) = R([A1; A2])
    import numpy as np
    from apex_camera_models import _lib
    L = _lib.load()
    rng = np.random.default_rng(k)
    A1, A2 = rng.normal(size=(50, k + 1)), rng.normal(size=(37, k + 1))
    r1, r2 = _packed_r(A1), _packed_r(A2)
    a = (ctypes.c_double * len(r1))(*r1)
    b = (ctypes.c_double * len(r2))(*r2)
    assert L.acm_linear_system_r_merge(model, a, b) == 0
    np.testing.assert_allclose(np.array(a[:]), _packed_r(np.vstack([A1, A2])), rtol=1e-12,
                               atol=1e-12)
    assert L.acm_linear_system_r_merge(6, a, b) == _lib.ERR_NOT_SUPPORTED


def test_linear_estimation_solve_host_checks():
    from apex_camera_models import _lib
    L = _lib.load()
    _, cam = _init(2, [190.0, 190.0, 254.0, 256.0, 0.0, 0.0, 0.0, 0.0], 512, 512)
    r = (ctypes.c_double * 15)(*([0.0] * 15))
    assert L.acm_linear_estimation_solve(ctypes.byref(cam), 3, r, 0) == _lib.ERR_INVALID_PARAMS
    assert L.acm_linear_estimation_solve(ctypes.byref(cam), 10, r, 1) == _lib.ERR_NUMERICAL
