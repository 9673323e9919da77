"""Pins the CPU oracle (oracle/) before it is trusted as the parity checker.

1. The reference's own known answers (tests/golden/reference_kats.json,
   transcribed from /root/reference tests with file:line) pass on it.
2. Its f64 values agree with an independent 50-digit mpmath restatement of
   the model equations to a few ulps, and its analytic parameter Jacobians
   (apex-solver's, whose source is absent: "parity unpinned" against the
   crate) agree with 50-digit numerical derivatives.
3. It reproduces the committed golden vectors bit for bit (regression pin).
"""
import os

import numpy as np
import pytest

import kat_suite
import mp_models
import oracle as O
from _backends import OracleBackend, rel_err

SAMPLES = {
    0: ([461.629, 460.152, 362.680, 246.049], (752, 480)),
    1: ([461.629, 460.152, 362.680, 246.049, -0.28340811, 0.07395907, 0.00019359,
         1.76187114e-05, 0.0], (752, 480)),
    2: ([190.97847715128717, 190.9733070521226, 254.93170605935475, 256.8974428996504,
         0.0034823894022493434, 0.0007150348452162257, -0.0020532361418706202,
         0.00020293673591811182], (512, 512)),
    3: ([348.112754378549, 347.1109973814674, 365.8121721753254, 249.3555778487899,
         0.5657413673629862, -0.24425190195168348], (752, 480)),
    4: ([1313.83, 1313.27, 960.471, 546.981, 1.01674], (752, 480)),
    5: ([1313.83, 1313.27, 960.471, 546.981, 1.01674, 0.5], (752, 480)),
    6: ([379.045, 379.008, 505.512, 509.969, 0.9259487501905697], (752, 480)),
}


@pytest.mark.parametrize("case", kat_suite.ALL, ids=lambda f: f.__name__)
def test_reference_kats_on_oracle(case):
    case(OracleBackend())


def _rand_pts(n, seed):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(0.5, 4.0, n)], 1)


@pytest.mark.parametrize("model", range(7))
def test_oracle_project_matches_mpmath(model):
    params, (w, h) = SAMPLES[model]
    pts = _rand_pts(60, 100 + model)
    uv, st, _ = O.project(model, params, w, h, pts)
    n_ok = 0
    for i in range(len(pts)):
        if st[i] != 0:
            continue
        n_ok += 1
        ref = mp_models.project(model, params, pts[i])
        for a, b in zip(uv[i], ref):
            # f64 chain of ~20 roundings + libm atan2: a few ulps of the pixel scale
            assert abs(a - float(b)) <= 1e-12 * max(abs(float(b)), 1.0), (model, i, a, b)
    assert n_ok > 10


@pytest.mark.parametrize("model", range(7))
def test_oracle_jacobian_matches_mpmath(model):
    params, (w, h) = SAMPLES[model]
    pts = _rand_pts(12, 200 + model)
    _, st, J = O.project(model, params, w, h, pts, want_jac=True)
    checked = 0
    for i in range(len(pts)):
        if st[i] != 0:
            continue
        Ju, Jv = mp_models.jacobian(model, params, pts[i])
        scale = max(max(abs(float(t)) for t in Ju + Jv), 1.0)
        for k in range(len(params)):
            for a, b in ((J[k, i, 0], Ju[k]), (J[k, i, 1], Jv[k])):
                assert abs(a - float(b)) <= 1e-10 * max(abs(float(b)), 1e-6 * scale), \
                    (model, i, k, a, float(b))
        checked += 1
    assert checked >= 3


@pytest.mark.parametrize("model", range(7))
def test_oracle_unproject_matches_mpmath(model):
    params, (w, h) = SAMPLES[model]
    rng = np.random.default_rng(300 + model)
    uv = np.stack([rng.uniform(0, w, 80), rng.uniform(0, h, 80)], 1)
    ray, st = O.unproject(model, params, w, h, uv)
    n_ok = 0
    for i in range(len(uv)):
        if st[i] != 0:
            continue
        n_ok += 1
        ref = mp_models.unproject(model, params, uv[i])
        # Newton models stop at |delta| < 1e-6 (kannala_brandt.rs:510,
        # rad_tan.rs:459/503), so they are only that close to the exact root
        tol = 1e-6 if model in (1, 2) else 1e-12
        for a, b in zip(ray[i], ref):
            assert abs(a - float(b)) <= tol, (model, i, a, float(b))
    assert n_ok > 10


def test_oracle_sample_points_properties():
    # src/util/mod.rs:70-95 on samples/double_sphere.yaml, n = 100
    params, (w, h) = SAMPLES[3]
    uv, xyz, total = O.sample_points(3, params, w, h, 100)
    assert len(uv) > 0 and len(uv) == len(xyz)
    assert np.all(xyz[:, 2] > 0)
    assert total == 13 * 8  # round(sqrt(100*752/480)) x round(sqrt(100*480/752))


def test_oracle_radtan_linear_system():
    # tests/parameter_estimation.rs:8-63: 50 samples estimate nonzero k's;
    # 2 samples (< 3) is an InvalidParams error
    params, (w, h) = SAMPLES[1]
    uv, xyz, _ = O.sample_points(1, params, w, h, 50)
    p0 = params[:4] + [0.0] * 5
    A, b, k = O.linear_estimation_system(1, p0, xyz, uv)
    assert k == 3
    sol = np.linalg.lstsq(A, b, rcond=None)[0]
    assert np.any(np.abs(sol) > 1e-10)
    uv2, xyz2, _ = O.sample_points(1, params, w, h, 2)
    _, _, k2 = O.linear_estimation_system(1, p0, xyz2, uv2)
    assert k2 == -1


def test_oracle_reprojection_error_semantics():
    params, (w, h) = SAMPLES[3]
    pts = _rand_pts(101, 7)
    pts[3] = [0.1, 0.2, -1.0]  # fails -> skipped (error_metrics.rs:76)
    uv, st, _ = O.project(3, params, w, h, pts)
    obs = np.where(np.isnan(uv), 0.0, uv) + 0.5
    stats, m = O.reprojection_error(3, params, w, h, pts, obs)
    assert m == int((st == 0).sum())
    e = np.sqrt(2 * 0.25) * np.ones(m)
    assert stats["rmse"] == pytest.approx(np.sqrt(0.5), rel=1e-12)
    assert stats["median"] == pytest.approx(np.median(e), rel=1e-12)
    assert stats["stddev"] <= 1e-12


@pytest.mark.parametrize("model", range(7))
def test_oracle_reproduces_golden(model, golden_dir):
    path = os.path.join(golden_dir, f"golden_{model}.npz")
    g = np.load(path)
    params = g["params"].tolist()
    w, h = int(g["res"][0]), int(g["res"][1])
    uv, st, J = O.project(model, params, w, h, g["xyz"], want_jac=True)
    assert np.array_equal(st, g["proj_status"])
    assert np.array_equal(uv, g["uv"], equal_nan=True)
    assert np.array_equal(J, g["jac"], equal_nan=True)
    ray, st2 = O.unproject(model, params, w, h, g["uv_in"])
    assert np.array_equal(st2, g["unproj_status"])
    assert np.array_equal(ray, g["rays"], equal_nan=True)


@pytest.mark.parametrize("model", range(7))
def test_oracle_o3_build_is_bit_identical(model, golden_dir):
    """bench.py's cpu_baseline times liboracle_o3.so (-O3 -ffp-contract=off,
    BASELINE.md section 2): it must compute exactly what the -O2 checker does."""
    g = np.load(os.path.join(golden_dir, f"golden_{model}.npz"))
    params = g["params"].tolist()
    w, h = int(g["res"][0]), int(g["res"][1])
    L = O.lib("O3")
    xyz = np.ascontiguousarray(g["xyz"])
    n = xyz.shape[0]
    P = O.NUM_PARAMS[model]
    uv = np.empty((n, 2))
    st = np.empty(n, dtype=np.uint8)
    J = np.empty((P, n, 2))
    pa = np.ascontiguousarray(params, dtype=np.float64)
    L.oracle_project_batch(model, O._dp(pa), w, h, n, O._dp(xyz), O._dp(uv), O._u8p(st), O._dp(J))
    assert np.array_equal(st, g["proj_status"])
    assert np.array_equal(uv, g["uv"], equal_nan=True)
    assert np.array_equal(J, g["jac"], equal_nan=True)


def test_rel_err_helper():
    assert rel_err([1.0, np.nan], [1.0, np.nan]) == 0.0
    with pytest.raises(AssertionError):
        rel_err([1.0, 2.0], [1.0, np.nan])


def _py_fov_grid(params, xyz, uv):
    """fov.rs:176-229 in plain Python floats (same IEEE ops, same libm)."""
    import math
    fx, fy, cx, cy = params[:4]
    sums, cnts = [], []
    best_w, best = 1.0, math.inf
    for i in range(10, 300):
        wt = i / 100.0
        s, c = 0.0, 0
        for (x, y, z), (uo, vo) in zip(xyz.tolist(), uv.tolist()):
            r2 = x * x + y * y
            r = math.sqrt(r2)
            t = math.tan(wt / 2.0)
            a = math.atan2(2.0 * t * r, z)
            rd = 2.0 * t / wt if r2 < math.sqrt(2.220446049250313e-16) else a / (r * wt)
            du = (fx * (x * rd) + cx) - uo
            dv = (fy * (y * rd) + cy) - vo
            e = math.sqrt(du * du + dv * dv)
            if math.isfinite(e):
                s += e
                c += 1
        sums.append(s)
        cnts.append(c)
        if c > 0 and s / c < best:
            best, best_w = s / c, wt
    return best_w, np.array(sums), np.array(cnts, dtype=float)


def test_oracle_fov_grid_search_matches_python_restatement():
    params, (w, h) = SAMPLES[6]
    xyz = _rand_pts(60, 11)
    xyz[0] = [0.0, 0.0, 1.0]       # r2 < sqrt(EPS) branch
    xyz[1] = [0.3, 0.1, 0.0]       # z = 0
    uv, _, _ = O.project(6, params, w, h, xyz)
    uv = np.where(np.isnan(uv), np.inf, uv) + 0.3
    uv[5] = [np.nan, 1.0]          # non-finite error -> skipped
    bw, s, c = O.fov_grid_search(params[:4] + [1.0], xyz, uv)
    pw, ps, pc = _py_fov_grid(params, xyz, uv)
    assert bw == pw
    assert np.array_equal(s, ps) and np.array_equal(c, pc)
    assert c.max() <= 59


@pytest.mark.parametrize("w_true", [0.37, 0.93, 1.5, 2.41])
def test_oracle_fov_grid_recovers_on_grid_w(w_true):
    # data projected by FovModel::project (fov.rs:284-316, the same formula as
    # the search, :191-209) with an on-grid w has zero error exactly there
    params, (w, h) = SAMPLES[6]
    p = params[:4] + [w_true]
    xyz = _rand_pts(300, 5)
    uv, st, _ = O.project(6, p, w, h, xyz)
    ok = st == 0
    bw, s, c = O.fov_grid_search(p, xyz[ok], uv[ok])
    assert bw == w_true
    assert s[int(round(w_true * 100)) - 10] == 0.0


def test_oracle_fov_grid_needs_two_points():
    params, _ = SAMPLES[6]
    bw, _, _ = O.fov_grid_search(params, np.zeros((1, 3)), np.zeros((1, 2)))
    assert bw is None
