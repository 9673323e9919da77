"""Parity of the HIP kernels (through the C-ABI of libacm.so) against the CPU
oracle and the committed golden vectors.

Bar (BASELINE.json north_star): validity masks / status codes bit-exact;
f64 projections, rays, residuals and Jacobians within 1e-10 relative.
Relative error here is |gpu - ref| / max(|ref|, floor) with
  floor = 1.0 (one pixel / unit ray) for uv, rays and residuals, so values
          that cancel towards 0 are held to 1e-10 absolute, and
  floor = the point's largest |J| entry for Jacobians (per-point scale).
Models whose projection has no transcendental (Pinhole, RadTan, DS, UCM,
EUCM) are additionally required to be bit-exact: same operation order, no FMA
contraction, IEEE-correct div/sqrt on both sides.
"""
import os

import numpy as np
import pytest

import kat_suite
import oracle as O
from _backends import GpuBackend, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-10
NO_TRANSCENDENTAL_PROJECT = (0, 1, 3, 4, 5)
NO_TRANSCENDENTAL_UNPROJECT = (0, 1, 3, 4, 5)
# Models whose default unprojection returns the reference's rays bit for bit.
# RadTan's (and KB's) default Newton loop is the certified fast one
# (ACM_REFERENCE_NEWTON off): statuses exact, rays within a few ulp;
# test_newton_reference_loop_bit_exact pins the knob-off path bit for bit.
EXACT_RAYS_UNPROJECT = (0, 3, 4, 5)
ULP = 2.0 ** -52


def ulps_of_one(a, b):
    """max |a - b| in units of ulp(1) over finite entries (unit rays)"""
    fin = np.isfinite(b)
    assert np.array_equal(fin, np.isfinite(a)), "finite pattern differs"
    return float(np.abs(a[fin] - b[fin]).max() / ULP) if fin.any() else 0.0


@pytest.fixture(scope="module")
def be():
    return GpuBackend()


def _golden(golden_dir, model):
    g = np.load(os.path.join(golden_dir, f"golden_{model}.npz"))
    return g, g["params"].tolist(), int(g["res"][0]), int(g["res"][1])


def jac_err(a, b):
    """per-point scaled error of (P, N, 2) Jacobians; NaN patterns must match
    (a non-finite input point can project 'Ok' to NaN, as in the reference)"""
    assert np.array_equal(np.isnan(a), np.isnan(b)), "NaN pattern differs"
    a = np.where(np.isnan(b), 0.0, a)
    b = np.where(np.isnan(b), 0.0, b)
    fin = np.isfinite(b).all(axis=(0, 2))
    assert np.array_equal(a[:, ~fin], b[:, ~fin])
    a, b = a[:, fin], b[:, fin]
    if b.size == 0:
        return 0.0
    scale = np.maximum(np.abs(b).max(axis=(0, 2)), 1e-300)
    d = np.abs(a - b).max(axis=(0, 2))
    return float((d / scale).max())


def _finite_rows(g):
    """golden points whose projection is either a failure or finite (drops the
    inf/NaN edge inputs that the reference itself propagates as NaN)"""
    uv, st = g["uv"], g["proj_status"]
    keep = np.isfinite(g["xyz"]).all(1) & ((st != 0) | np.isfinite(uv).all(1))
    return keep


def bits_equal(a, b):
    import torch
    return torch.equal(a.contiguous().view(torch.int64), b.contiguous().view(torch.int64))


@pytest.mark.parametrize("layout", ["aos", "soa"])
@pytest.mark.parametrize("model", range(7))
def test_project_jacobian_vs_golden(be, golden_dir, model, layout):
    g, params, w, h = _golden(golden_dir, model)
    uv, st, J = be.project(model, params, w, h, g["xyz"], want_jac=True, layout=layout)
    assert np.array_equal(st, g["proj_status"]), np.nonzero(st != g["proj_status"])
    assert rel_err(uv, g["uv"], floor=1.0) <= TOL
    assert np.all(J[:, st != 0] == 0.0)
    assert jac_err(J, g["jac"]) <= TOL
    if model in NO_TRANSCENDENTAL_PROJECT:
        assert np.array_equal(uv, g["uv"], equal_nan=True)
        assert np.array_equal(J, g["jac"], equal_nan=True)


@pytest.mark.parametrize("layout", ["aos", "soa"])
@pytest.mark.parametrize("model", range(7))
def test_unproject_vs_golden(be, golden_dir, model, layout):
    g, params, w, h = _golden(golden_dir, model)
    rays, st = be.unproject(model, params, w, h, g["uv_in"], layout=layout)
    assert np.array_equal(st, g["unproj_status"]), np.nonzero(st != g["unproj_status"])
    assert rel_err(rays, g["rays"], floor=1.0) <= TOL
    if model in EXACT_RAYS_UNPROJECT:
        assert np.array_equal(rays, g["rays"], equal_nan=True)
    if model == 1:
        assert ulps_of_one(rays[st == 0], g["rays"][st == 0]) <= 8


@pytest.mark.parametrize("model", [1, 2])
def test_newton_reference_loop_bit_exact(be, golden_dir, model):
    """ACM_REFERENCE_NEWTON (per call) runs the reference's own Newton loop for
    every pixel: RadTan rays then equal the golden (oracle) rays bit for bit,
    in acm_unproject and in sample_points; KB's stay within 1e-10 (its sin /
    cos are polynomials either way).  Statuses are the same in both modes."""
    from apex_camera_models import util
    from test_oracle import SAMPLES
    g, params, w, h = _golden(golden_dir, model)
    rays, st = be.unproject(model, params, w, h, g["uv_in"], reference_newton=True)
    assert np.array_equal(st, g["unproj_status"])
    if model == 1:
        assert np.array_equal(rays, g["rays"], equal_nan=True)
    else:
        assert rel_err(rays, g["rays"], floor=1.0) <= TOL
    sp, (sw, sh) = SAMPLES[model]
    m = _model_obj(model, sp, sw, sh)
    uv0, xyz0, _ = O.sample_points(model, sp, sw, sh, 20_000)
    uv, xyz = util.sample_points(m, 20_000, reference_newton=True)
    assert np.array_equal(uv.cpu().numpy(), uv0)
    if model == 1:
        assert np.array_equal(xyz.cpu().numpy(), xyz0)


# strongly distorted cameras inside the fast loops' per-camera bounds (and one
# RadTan camera outside them), as in round 2's newton_fast probe (git history)
NEWTON_STRESS = [
    (2, [190.97847715128717, 190.9733070521226, 254.93170605935475, 256.8974428996504,
         0.5, -0.3, 0.1, -0.02], (512, 512)),
    (2, [190.97847715128717, 190.9733070521226, 254.93170605935475, 256.8974428996504,
         -0.2, 0.15, -0.05, 0.004], (512, 512)),
    (1, [461.629, 460.152, 362.680, 246.049, -0.45, 0.12, 0.003, -0.002, -0.005], (752, 480)),
    (1, [461.629, 460.152, 362.680, 246.049, 0.3, -0.05, 0.01, 0.01, 0.002], (752, 480)),
    (1, [461.629, 460.152, 362.680, 246.049, -0.6, 0.45, 0.003, -0.002, -0.1], (752, 480)),
]


@pytest.mark.parametrize("case", range(len(NEWTON_STRESS)))
def test_newton_fast_statuses_identical_under_stress(be, case):
    """The certified fast loops against the reference's loop on 1M pixels
    spread over the image and a 10-pixel margin of strongly distorted
    cameras, where Newton fails for up to 20% of the pixels and many deltas
    pass near the threshold: identical statuses (the certificate's claim),
    and rays within 32 ulp of 1 (KB's third stress camera reaches ~24: its
    Newton steps amplify rounding), against the oracle too."""
    model, params, (w, h) = NEWTON_STRESS[case]
    rng = np.random.default_rng(case)
    n = 1_000_000
    px = np.stack([rng.uniform(-10, w + 10, n), rng.uniform(-10, h + 10, n)], 1)
    rays1, st1 = be.unproject(model, params, w, h, px)
    rays0, st0 = be.unproject(model, params, w, h, px, reference_newton=True)
    assert np.array_equal(st1, st0), np.nonzero(st1 != st0)[0][:5]
    ok = st0 == 0
    assert ulps_of_one(rays1[ok], rays0[ok]) <= 32
    sub = slice(0, 50_000)
    r_o, s_o = O.unproject(model, params, w, h, px[sub])
    assert np.array_equal(st1[sub], s_o)
    if model == 1:
        assert np.array_equal(rays0[sub][s_o == 0], r_o[s_o == 0], equal_nan=True)


@pytest.mark.parametrize("case", kat_suite.ALL, ids=lambda f: f.__name__)
def test_reference_kats_on_gpu(be, case):
    case(be)


@pytest.mark.parametrize("n", [1, 63, 64, 255, 257, 1000, 65537])
def test_ragged_sizes_kb(be, n):
    params, (w, h) = kat_suite.KATS["yaml_values"]["kannala_brandt"]["params"], (512, 512)
    rng = np.random.default_rng(n)
    pts = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(-0.2, 4, n)], 1)
    uv, st, J = be.project(2, params, w, h, pts, want_jac=True)
    uv0, st0, J0 = O.project(2, params, w, h, pts, want_jac=True)
    assert np.array_equal(st, st0)
    assert rel_err(uv, uv0, 1.0) <= TOL and jac_err(J, J0) <= TOL


def _model_obj(model, params, w, h):
    return GpuBackend()._model(model, params, w, h)


@pytest.mark.parametrize("policy", [0, 1])
@pytest.mark.parametrize("model", range(7))
def test_residual_jacobian_vs_oracle(golden_dir, model, policy):
    import torch
    from apex_camera_models import factors
    g, params, w, h = _golden(golden_dir, model)
    keep = _finite_rows(g)
    xyz = g["xyz"][keep]
    obs = np.where(np.isnan(g["uv"][keep]), 3.0, g["uv"][keep]) + \
        np.linspace(-2, 2, len(xyz))[:, None]
    cls = [factors.PinholeCameraParamsFactor, factors.RadTanCameraParamsFactor,
           factors.KannalaBrandtCameraParamsFactor, factors.DoubleSphereCameraParamsFactor,
           factors.UcmCameraParamsFactor, factors.EucmCameraParamsFactor,
           factors.FovCameraParamsFactor][model]
    from apex_camera_models.camera import Resolution
    f = cls(torch.as_tensor(xyz), torch.as_tensor(obs), Resolution(w, h), invalid_policy=policy)
    r, J = f.linearize(params)
    r = r.cpu().numpy().reshape(-1, 2)
    Jn = J.t().contiguous().cpu().numpy().reshape(len(params), -1, 2)
    r0, J0, st0 = O.residual_jacobian(model, params, w, h, xyz, obs, policy)
    assert rel_err(r, r0, floor=1.0) <= TOL
    assert jac_err(Jn, J0) <= TOL
    assert J.shape == (2 * len(xyz), len(params)) and J.stride() == (1, 2 * len(xyz))


@pytest.mark.parametrize("policy", [0, 1])
@pytest.mark.parametrize("model", range(7))
def test_normal_equations_vs_oracle(golden_dir, model, policy):
    import torch
    from apex_camera_models import factors
    from apex_camera_models.camera import Resolution
    g, params, w, h = _golden(golden_dir, model)
    keep = _finite_rows(g)
    xyz = g["xyz"][keep]
    obs = np.where(np.isnan(g["uv"][keep]), 3.0, g["uv"][keep]) + 0.25
    f = factors.CameraParamsFactor.__subclasses__()[model](
        torch.as_tensor(xyz), torch.as_tensor(obs), Resolution(w, h), invalid_policy=policy)
    P = len(params)
    A0, b0, c0, nv0 = O.normal_equations(model, params, w, h, xyz, obs, policy)
    res = f.normal_equations(params)
    A, b, c, nv = [t.cpu().numpy() for t in f.unpack_normal_equations(res, P)]
    assert int(nv) == nv0
    # reduction order differs from the oracle's point order: hold the sums to
    # 1e-10 of the largest entry (f64 summation of ~2.5k terms)
    assert np.abs(A - A0).max() <= TOL * np.abs(A0).max()
    assert np.abs(b - b0).max() <= TOL * max(np.abs(b0).max(), 1.0)
    assert abs(c - c0) <= TOL * max(abs(c0), 1.0)
    # deterministic: a second evaluation is bit-identical
    res2 = f.normal_equations(params)
    assert torch.equal(res, res2)


@pytest.mark.parametrize("model", range(7))
def test_normal_equations_every_tuning_cell(model):
    """Every (waves, points-per-lane-step) cell of k_normal_eq on a ragged
    batch several grid strides long (exercises the unrolled tails) agrees
    with the oracle; the knobs only change the summation order."""
    import torch
    from apex_camera_models import _lib, factors, samples
    from apex_camera_models.camera import Resolution
    params, (w, h) = samples.SAMPLES[model]
    n = 1_234_567
    xyz = samples.synthetic_points(n)
    xyz = xyz[np.isfinite(xyz).all(1)]
    uv0, st0, _ = O.project(model, params, w, h, xyz)
    obs = np.where(np.isnan(uv0), 3.0, uv0) + 0.25
    A0, b0, c0, nv0 = O.normal_equations(model, params, w, h, xyz, obs, 0)
    f = factors.CameraParamsFactor.__subclasses__()[model](
        torch.as_tensor(xyz), torch.as_tensor(obs), Resolution(w, h))
    P = len(params)
    L = _lib.load()
    # (KB also: loads 3 and 4 steps ahead)
    cells = [(wv, un, ntl) for wv in (0, 1, 3, 4) for un in (0, 1, 2, 3) for ntl in (-1, 0)]
    if model == 2:
        cells += [(wv, un, -1) for wv in (1, 3) for un in (4, 5)]
    try:
        for cell in cells:
            wv, un, ntl = cell
            L.acm_set_tuning(_lib.TUNE_NE_WAVES, wv)
            L.acm_set_tuning(_lib.TUNE_NE_UNROLL, un)
            L.acm_set_tuning(_lib.TUNE_NT_LOADS, ntl)
            res = f.normal_equations(params)
            A, b, c, nv = [t.cpu().numpy() for t in f.unpack_normal_equations(res, P)]
            assert int(nv) == nv0, cell
            assert np.abs(A - A0).max() <= TOL * np.abs(A0).max(), cell
            assert np.abs(b - b0).max() <= TOL * max(np.abs(b0).max(), 1.0), cell
            assert abs(c - c0) <= TOL * max(abs(c0), 1.0), cell
    finally:
        L.acm_set_tuning(_lib.TUNE_NE_WAVES, 0)
        L.acm_set_tuning(_lib.TUNE_NE_UNROLL, 0)
        L.acm_set_tuning(_lib.TUNE_NT_LOADS, -1)


@pytest.mark.parametrize("model", range(7))
def test_reprojection_error_vs_oracle(golden_dir, model):
    import torch
    from apex_camera_models import util
    g, params, w, h = _golden(golden_dir, model)
    keep = _finite_rows(g)
    xyz = g["xyz"][keep]
    obs = np.where(np.isnan(g["uv"][keep]), 0.0, g["uv"][keep]) + \
        np.sin(np.arange(len(xyz)))[:, None]
    m = _model_obj(model, params, w, h)
    pe = util.compute_reprojection_error(m, torch.as_tensor(xyz), torch.as_tensor(obs))
    ref, nv = O.reprojection_error(model, params, w, h, xyz, obs)
    assert pe.n_valid == nv
    for k in ("rmse", "mean", "stddev"):
        assert abs(getattr(pe, k) - ref[k]) <= TOL * max(abs(ref[k]), 1.0), k
    for k in ("min", "max", "median"):  # order statistics of identical per-point errors
        assert abs(getattr(pe, k) - ref[k]) <= TOL * max(abs(ref[k]), 1.0), k
    if model in NO_TRANSCENDENTAL_PROJECT:
        assert pe.min == ref["min"] and pe.max == ref["max"] and pe.median == ref["median"]


@pytest.mark.parametrize("n", [1, 2, 63, 65, 1000, 300_001])
def test_reprojection_stddev_single_pass_no_cancellation(n):
    """The one-pass variance (per-lane shifted sums + Chan merges) against
    the oracle's two-pass sum((e - mean)^2) where E[e^2] - mean^2 would
    cancel: errors of ~424 px with a spread of ~1e-3 px (a sum-of-squares
    formula keeps ~4 digits here).  Ragged n, one point and all-equal cases."""
    import torch
    from apex_camera_models import samples, util
    params, (w, h) = samples.SAMPLES[0]
    rng = np.random.default_rng(n)
    xyz = np.stack([rng.uniform(-0.3, 0.3, n), rng.uniform(-0.3, 0.3, n),
                    rng.uniform(1.0, 2.0, n)], 1)
    uv0, st0, _ = O.project(0, params, w, h, xyz)
    m = _model_obj(0, params, w, h)
    for spread in (1e-3, 0.0):
        obs = uv0 + 300.0 + spread * np.sin(np.arange(n))[:, None]
        pe = util.compute_reprojection_error(m, torch.as_tensor(xyz), torch.as_tensor(obs))
        ref, nv = O.reprojection_error(0, params, w, h, xyz, obs)
        assert pe.n_valid == nv
        assert abs(pe.mean - ref["mean"]) <= TOL * ref["mean"]
        # stddev to 1e-9 of itself, or -- when the spread is 0 -- to the
        # rounding of the oracle's own sequential mean (n eps mean), which
        # then is all its two-pass stddev measures
        slack = 4.0 * n * np.finfo(float).eps * ref["mean"]
        assert abs(pe.stddev - ref["stddev"]) <= 1e-9 * ref["stddev"] + slack, \
            (spread, pe.stddev, ref["stddev"])


def test_reprojection_error_zero_points():
    import torch
    from apex_camera_models import util
    m = _model_obj(2, kat_suite.KATS["yaml_values"]["kannala_brandt"]["params"], 512, 512)
    with pytest.raises(util.ZeroProjectionPoints):
        util.compute_reprojection_error(m, torch.tensor([[0.1, 0.2, -1.0]]),
                                        torch.tensor([[1.0, 1.0]]))


@pytest.mark.parametrize("n", [1, 2, 1000, 2_000_003])
def test_reprojection_error_fused_matches_two_calls(n):
    """acm_reprojection_error (statistics + median, the median's first
    histogram counted by the statistics pass) against acm_reprojection_stats
    + acm_median_valid on the same inputs: the same errors and the same
    median bit for bit, the statistics to rounding (the two passes may run
    different workgroup counts).  Failed projections (z < 0) and NaN
    observations are in the input; errors both into the caller's buffer and
    into the workspace."""
    import ctypes
    import torch
    from apex_camera_models import _lib, samples, util
    L = _lib.load()
    params, (w, h) = samples.SAMPLES[3]
    rng = np.random.default_rng(n)
    xyz = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(-0.3, 2.0, n)], 1)
    obs = rng.uniform(0, w, (n, 2))
    obs[::7] = np.nan
    m = _model_obj(3, params, w, h)
    p3 = torch.as_tensor(xyz, device="cuda")
    p2 = torch.as_tensor(obs, device="cuda")
    e_sep = torch.empty((n,), dtype=torch.float64, device="cuda")
    st = util.reprojection_stats(m, p3, p2, e_sep)
    nv = int(st[5].item())
    med = util.reprojection_median(e_sep, nv) if nv else float("nan")
    cam = m.acm_camera()
    wsb = L.acm_reprojection_error_workspace_size(n)
    for own_errors in (True, False):
        ws = torch.empty(((wsb + 7) // 8,), dtype=torch.float64, device="cuda")
        res = torch.empty((9,), dtype=torch.float64, device="cuda")
        e = torch.full((n,), -1.0, dtype=torch.float64, device="cuda")
        _lib.check(L.acm_reprojection_error(ctypes.byref(cam), n, p3.data_ptr(), _lib.LAYOUT_AOS,
                                            p2.data_ptr(), res.data_ptr(),
                                            e.data_ptr() if own_errors else None, ws.data_ptr(),
                                            wsb, torch.cuda.current_stream().cuda_stream))
        r = res.cpu().numpy()
        s0 = st.cpu().numpy()
        assert r[5] == s0[5]
        if own_errors:
            assert torch.equal(torch.isnan(e), torch.isnan(e_sep))
            ok = ~torch.isnan(e)
            assert torch.equal(e[ok], e_sep[ok])
        if nv == 0:
            assert np.isnan(r[8])
            continue
        assert r[8] == med, (r[8], med)
        assert r[1] == s0[1] and r[2] == s0[2]  # min, max
        for k in (0, 3, 4, 6, 7):
            assert abs(r[k] - s0[k]) <= 1e-12 * max(abs(s0[k]), 1.0), (k, r[k], s0[k])


@pytest.mark.parametrize("n", [2, 100, 500, 20_000])
@pytest.mark.parametrize("model", range(7))
def test_sample_points_vs_oracle(model, n):
    from apex_camera_models import util
    from test_oracle import SAMPLES
    params, (w, h) = SAMPLES[model]
    m = _model_obj(model, params, w, h)
    uv, xyz = util.sample_points(m, n)
    uv0, xyz0, _ = O.sample_points(model, params, w, h, n)
    assert uv.shape[0] == uv0.shape[0]  # same kept set ...
    assert np.array_equal(uv.cpu().numpy(), uv0)  # ... in the same order, bit-exact pixels
    assert rel_err(xyz.cpu().numpy(), xyz0, floor=1.0) <= TOL
    if model in EXACT_RAYS_UNPROJECT:
        assert np.array_equal(xyz.cpu().numpy(), xyz0)


@pytest.mark.parametrize("model", range(7))
def test_sample_points_every_path_matches_oracle(model):
    """The single-pass look-back kernel at every tile size (2/4/8 x 256
    cells, ~500 tiles, a ragged last tile) and the two-pass path give the
    oracle's kept set in the oracle's order, bit for bit, and a row-range
    shard of the grid (odd cell offset) matches its slice of the full run."""
    import torch
    from apex_camera_models import _lib, util
    from apex_camera_models.distributed import gpu_sample_points_range, grid_row_range
    from test_oracle import SAMPLES
    params, (w, h) = SAMPLES[model]
    m = _model_obj(model, params, w, h)
    n = 500_000
    uv0, xyz0, _ = O.sample_points(model, params, w, h, n)
    L = _lib.load()
    ncx = int(round(np.sqrt(n * (w / h))))
    ncy = int(round(np.sqrt(n * (h / w))))
    try:
        for v in (-1, 0, 1, 2, 3, 4):
            L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, v)
            uv, xyz = util.sample_points(m, n)
            assert np.array_equal(uv.cpu().numpy(), uv0), v
            assert rel_err(xyz.cpu().numpy(), xyz0, floor=1.0) <= TOL, v
            if model in EXACT_RAYS_UNPROJECT:
                assert np.array_equal(xyz.cpu().numpy(), xyz0), v
            fn = gpu_sample_points_range(m, n)
            parts = [fn(*grid_row_range(ncx, ncy, r, 3)) for r in range(3)]
            assert torch.equal(torch.cat([p[0] for p in parts]), uv), v
            assert torch.equal(torch.cat([p[1] for p in parts]), xyz), v
    finally:
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, -1)


def test_sample_points_kb_clamped_angle():
    """KB with no distortion and a short focal length: every pixel with
    ru >= pi/2 clamps to theta = 1.5707963267948966 (kannala_brandt.rs:467)
    and Newton stays there, so Z = cos(theta) / |p| is +6.1e-17 / |p| -- kept
    (point_sampling.rs:91-94) -- while the next double up would be dropped.
    The keep decision at that exact angle, and the kept set around it, must
    match the oracle (glibc cos)."""
    from apex_camera_models import util
    params = [100.0, 100.0, 320.0, 240.0, 0.0, 0.0, 0.0, 0.0]
    w, h = 640, 480
    m = _model_obj(2, params, w, h)
    for n in (5000, 300_000):
        uv, xyz = util.sample_points(m, n)
        uv0, xyz0, _ = O.sample_points(2, params, w, h, n)
        assert np.array_equal(uv.cpu().numpy(), uv0)
        assert rel_err(xyz.cpu().numpy(), xyz0, floor=1.0) <= TOL
        # the clamped pixels are there (Z tiny but positive)
        assert (xyz0[:, 2] < 1e-15).sum() > 0


# cameras whose unprojection fails over whole regions of the image: the two
# distorted KB cameras above, and RadTan with a short focal length, whose
# radial map folds over inside the image (r_d peaks at r^2 = -1 / (3 k1):
# the corners have no preimage and Newton fails there)
SPEC_DROP_CAMS = NEWTON_STRESS[:2] + [
    (1, [200.0, 200.0, 376.0, 240.0, -0.45, 0.12, 0.003, -0.002, -0.005], (752, 480)),
    (1, [200.0, 200.0, 376.0, 240.0, -0.45, 0.0, 0.003, -0.002, 0.0], (752, 480)),
    (1, [300.0, 300.0, 370.0, 250.0, -0.6, 0.1, 0.001, 0.002, 0.0], (752, 480)),
]


@pytest.mark.parametrize("case", range(len(SPEC_DROP_CAMS)))
def test_sample_points_speculative_with_drops(case):
    """The speculative segment path (ACM_TUNE_SAMPLE_FUSED = 4, auto for
    RadTan) on the strongly distorted cameras, whose Newton fails over whole
    regions of the image: the repair pass must move every segment after the
    first drop, and the result equals the segment two-pass path, the
    round-1 two-pass path and the oracle bit for bit -- also per row-range
    shard, whose first drop comes at a different place."""
    import torch
    from apex_camera_models import _lib, util
    from apex_camera_models.distributed import gpu_sample_points_range, grid_row_range
    model, params, (w, h) = SPEC_DROP_CAMS[case]
    m = _model_obj(model, params, w, h)
    n = 400_000
    L = _lib.load()
    ncx = int(round(np.sqrt(n * (w / h))))
    ncy = int(round(np.sqrt(n * (h / w))))
    try:
        outs = {}
        for v in (4, 0, -1):
            L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, v)
            outs[v] = util.sample_points(m, n)
            if v == 4:
                fn = gpu_sample_points_range(m, n)
                parts = [fn(*grid_row_range(ncx, ncy, r, 3)) for r in range(3)]
        uv, xyz = outs[4]
        for v in (0, -1):
            assert torch_equal_bits(uv, outs[v][0]) and torch_equal_bits(xyz, outs[v][1]), v
        assert torch.equal(torch.cat([p[0] for p in parts]), uv)
        assert torch.equal(torch.cat([p[1] for p in parts]), xyz)
    finally:
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, -1)
    assert uv.shape[0] < ncx * ncy  # this camera drops cells
    uv0, xyz0, _ = O.sample_points(model, params, w, h, n)
    assert np.array_equal(uv.cpu().numpy(), uv0)
    assert rel_err(xyz.cpu().numpy(), xyz0, floor=1.0) <= TOL


@pytest.mark.parametrize("fused", [1, 2, 3])
@pytest.mark.parametrize("model", [1, 2, 4])
def test_sample_points_lookback_fallback(model, fused):
    """ACM_TUNE_SAMPLE_PATIENCE = 0: a tile whose predecessor has not yet
    published its count counts that predecessor's cells itself at once (the
    path that guarantees progress whatever the dispatch order), at every tile
    size.  Outputs stay bit-identical to the default run and the oracle."""
    from apex_camera_models import _lib, util
    from test_oracle import SAMPLES
    params, (w, h) = SAMPLES[model]
    m = _model_obj(model, params, w, h)
    n = 2_000_000
    L = _lib.load()
    uv_d, xyz_d = util.sample_points(m, n)
    try:
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, fused)
        L.acm_set_tuning(_lib.TUNE_SAMPLE_PATIENCE, 0)
        for _ in range(3):
            uv, xyz = util.sample_points(m, n)
            assert torch_equal_bits(uv, uv_d) and torch_equal_bits(xyz, xyz_d)
    finally:
        L.acm_set_tuning(_lib.TUNE_SAMPLE_PATIENCE, -1)
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, -1)
    uv0, xyz0, _ = O.sample_points(model, params, w, h, n)
    assert np.array_equal(uv.cpu().numpy(), uv0)


def torch_equal_bits(a, b):
    import torch
    return a.shape == b.shape and torch.equal(a.contiguous().view(torch.int64),
                                              b.contiguous().view(torch.int64))


def test_full_size_kb_properties():
    """BASELINE config 2 size (10M): properties that need no oracle run over the
    whole batch, plus an oracle check of a 200k-point strided subsample."""
    import torch
    from apex_camera_models import samples
    params, (w, h) = samples.SAMPLES[2]
    m = _model_obj(2, params, w, h)
    n = 10_000_000
    pts = samples.synthetic_points_device(n)
    uv, st, J = m.project_batch(pts, jacobian=True)
    uv2, st2, J2 = m.project_batch(pts, jacobian=True)
    assert torch.equal(st, st2) and bits_equal(J, J2) and bits_equal(uv, uv2)  # deterministic
    fin = torch.isfinite(pts).all(1)
    assert torch.equal(torch.isnan(uv[:, 0])[fin], (st != 0)[fin])
    ok = (st == 0) & fin
    assert int(ok.sum()) > 0.99 * n
    rays, rst = m.unproject_batch(uv[ok])
    p = pts[ok]
    pn = p / torch.linalg.norm(p, dim=1, keepdim=True)
    good = rst == 0
    dots = (pn[good] * rays[good]).sum(1)
    assert float(dots.min()) > 1.0 - 1e-9
    idx = torch.arange(0, n, 50, device="cuda")
    sub = pts[idx].cpu().numpy()
    uv0, st0, J0 = O.project(2, params, w, h, sub, want_jac=True)
    assert np.array_equal(st[idx].cpu().numpy(), st0)
    assert rel_err(uv[idx].cpu().numpy(), uv0, 1.0) <= TOL
    assert jac_err(J[:, idx].cpu().numpy(), J0) <= TOL


def test_empty_batch_is_noop():
    import torch
    params, (w, h) = kat_suite.KATS["yaml_values"]["kannala_brandt"]["params"], (512, 512)
    m = _model_obj(2, params, w, h)
    uv, st, J = m.project_batch(torch.empty((0, 3), dtype=torch.float64), jacobian=True)
    assert uv.shape == (0, 2) and st.shape == (0,) and J.shape == (8, 0, 2)


@pytest.mark.parametrize("model", range(7))
def test_f32_path_tracks_f64(golden_dir, model):
    """f32 evaluation of the same model code (config 5 sweep): masks may only
    differ where an f64 threshold test is within f32 rounding; values within
    f32 accuracy of the f64 oracle."""
    import torch
    g, params, w, h = _golden(golden_dir, model)
    keep = _finite_rows(g) & (np.abs(g["xyz"]) < 1e3).all(1)
    xyz = g["xyz"][keep]
    m = _model_obj(model, params, w, h)
    uv, st, J = m.project_batch(torch.as_tensor(xyz, dtype=torch.float32), jacobian=True)
    assert uv.dtype == torch.float32 and J.dtype == torch.float32
    st = st.cpu().numpy()
    st0 = g["proj_status"][keep]
    agree = (st == st0).mean()
    assert agree > 0.99, agree
    both = (st == 0) & (st0 == 0)
    u0 = g["uv"][keep][both]
    err = np.abs(uv.cpu().numpy()[both].astype(np.float64) - u0) / np.maximum(np.abs(u0), 1.0)
    assert np.nanmax(err) < 1e-4


@pytest.mark.parametrize("model", [2, 3])
def test_buffers_at_8_byte_offsets(golden_dir, model):
    """The C-ABI takes plain f64 pointers: a caller may hand sub-views that are
    only 8-byte aligned (e.g. a Matrix2xX slice starting at an odd column
    offset of a larger buffer).  Every 16-B vector store must still land
    correctly -- same results as 16-B-aligned buffers."""
    import ctypes

    import torch
    from apex_camera_models import _lib
    g = np.load(os.path.join(golden_dir, f"golden_{model}.npz"))
    params = g["params"].tolist()
    w, h = int(g["res"][0]), int(g["res"][1])
    pts = g["xyz"]
    n = len(pts)
    P = len(params)
    L = _lib.load()
    m = GpuBackend()._model(model, params, w, h)
    cam = m.acm_camera()
    base_p = torch.zeros(3 * n + 1, dtype=torch.float64, device="cuda")
    base_p[1:] = torch.as_tensor(pts.ravel(), device="cuda")
    uv = torch.full((2 * n + 1,), 7.0, dtype=torch.float64, device="cuda")
    st = torch.zeros(n + 1, dtype=torch.uint8, device="cuda")
    jac = torch.full((2 * n * P + 1,), 7.0, dtype=torch.float64, device="cuda")
    _lib.check(L.acm_project(ctypes.byref(cam), n, base_p.data_ptr() + 8, 0, uv.data_ptr() + 8,
                             st.data_ptr() + 1, jac.data_ptr() + 8, None))
    nu = len(g["uv_in"])
    uvin = torch.zeros(2 * nu + 1, dtype=torch.float64, device="cuda")
    uvin[1:] = torch.as_tensor(g["uv_in"].ravel(), device="cuda")
    rays = torch.full((3 * nu + 1,), 7.0, dtype=torch.float64, device="cuda")
    st2 = torch.zeros(nu + 1, dtype=torch.uint8, device="cuda")
    _lib.check(L.acm_unproject(ctypes.byref(cam), nu, uvin.data_ptr() + 8, rays.data_ptr() + 8,
                               0, st2.data_ptr() + 1, None))
    torch.cuda.synchronize()
    ref_uv, ref_st, ref_j = GpuBackend().project(model, params, w, h, pts)
    assert uv[0].item() == 7.0 and jac[0].item() == 7.0  # nothing written before the view
    assert np.array_equal(st[1:].cpu().numpy(), ref_st)
    assert np.array_equal(uv[1:].cpu().numpy().reshape(n, 2), ref_uv, equal_nan=True)
    assert np.array_equal(jac[1:].cpu().numpy().reshape(P, n, 2), ref_j, equal_nan=True)
    ref_r, ref_s2 = GpuBackend().unproject(model, params, w, h, g["uv_in"])
    assert np.array_equal(st2[1:].cpu().numpy(), ref_s2)
    assert np.array_equal(rays[1:].cpu().numpy().reshape(nu, 3), ref_r, equal_nan=True)


def _gpu_median(vals):
    import ctypes

    import torch
    from apex_camera_models import _lib
    L = _lib.load()
    v = torch.as_tensor(np.asarray(vals, dtype=np.float64), device="cuda")
    n = v.numel()
    m = int((~torch.isnan(v)).sum())
    ws_b = L.acm_median_workspace_size(n)
    ws = torch.empty(((ws_b + 7) // 8,), dtype=torch.float64, device="cuda")
    out = torch.empty((1,), dtype=torch.float64, device="cuda")
    _lib.check(L.acm_median_valid(n, v.data_ptr() if n else None, None, m, out.data_ptr(),
                                  ws.data_ptr(), ws_b, None))
    return float(out.item())


@pytest.mark.parametrize("case", ["odd", "even", "ties", "tie_pair", "nan_mix", "one", "all_nan",
                                  "denormal", "wide", "zeros", "big", "big_ties", "narrow"])
def test_median_radix_select_exact(case):
    """acm_median_valid (6-pass 11-bit radix select, both ranks at once) is
    the exact median of the non-NaN values, error_metrics.rs:103-111."""
    rng = np.random.default_rng(hash(case) % 2**32)
    v = {
        "odd": rng.uniform(0, 5, 1001),
        "even": rng.uniform(0, 5, 1000),
        "ties": np.repeat(rng.uniform(0, 1, 37), 5),
        "tie_pair": np.array([1.0, 2.0, 2.0, 3.0]),
        "nan_mix": np.where(rng.uniform(size=5000) < 0.3, np.nan, rng.exponential(1.0, 5000)),
        "one": np.array([0.125]),
        "all_nan": np.full(17, np.nan),
        "denormal": np.concatenate([np.full(10, 5e-324), np.full(11, 1e-310), [0.0] * 3]),
        "wide": 10.0 ** rng.uniform(-300, 300, 4097),
        "zeros": np.zeros(64),
        "big": rng.exponential(0.01, 3_000_001),
        # every value a candidate after two passes: overflows the per-workgroup
        # LDS stage of the compaction kernel
        "big_ties": np.concatenate([np.full(2_000_000, 0.25), rng.uniform(0, 1, 1001)]),
        # 5M values within a few ulps: candidates share 40+ leading bits
        "narrow": 1.0 + rng.integers(0, 64, 5_000_000) * np.finfo(np.float64).eps,
    }[case]
    got = _gpu_median(v)
    valid = v[~np.isnan(v)]
    if valid.size == 0:
        assert np.isnan(got)
    else:
        assert got == np.median(valid), (got, np.median(valid))


def test_status_on_thresholds_matches_oracle(be):
    """tests/boundary_probes.py: +-8 ulps around every threshold root; the
    kernels' statuses equal the oracle's (which test_boundaries.py pins to a
    binary64 emulation of the Rust conditions), values bit-exact for the
    models without a transcendental (RadTan's unprojection within 8 ulp: its
    default Newton loop is the certified fast one) and within 1e-10 for KB."""
    import boundary_probes as B
    for model, p, (w, h), kind, pts in B.probes():
        if kind == "project":
            uv, st, _ = be.project(model, p, w, h, pts, want_jac=False)
            uv0, st0, _ = O.project(model, p, w, h, pts)
        else:
            uv, st = be.unproject(model, p, w, h, pts)
            uv0, st0 = O.unproject(model, p, w, h, pts)
        assert np.array_equal(st, st0), (model, kind, np.nonzero(st != st0)[0][:5])
        ok = st0 == 0
        if model == 2:
            assert rel_err(uv[ok], uv0[ok], floor=1.0) <= TOL
        elif model == 1 and kind == "unproject":  # the certified fast Newton
            assert ulps_of_one(uv[ok], uv0[ok]) <= 8
        else:
            assert np.array_equal(uv[ok], uv0[ok], equal_nan=True), (model, kind)


@pytest.mark.parametrize("n", [1, 255, 257, 1000, 65537])
def test_unproject_every_store_form_identical(n):
    """ACM_TUNE_UNPROJECT_PPT: 1 or 2 pixels per lane, three 8-B stores per
    AoS ray or a wave's rays staged in LDS and written as 16-B pieces, on
    ragged sizes and with the ray buffer 16-B aligned or only 8-B aligned
    (staging then falls back): every form writes the same bytes."""
    import ctypes
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    rng = np.random.default_rng(n)
    for model in (0, 1, 2):
        params, (w, h) = samples.SAMPLES[model]
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), model,
                                     (ctypes.c_double * len(params))(*params), len(params), w, h))
        px = torch.as_tensor(np.stack([rng.uniform(-5, w + 5, n), rng.uniform(-5, h + 5, n)], 1),
                             device="cuda")
        outs = []
        try:
            for v in (-1, 1, 2, 3):
                L.acm_set_tuning(_lib.TUNE_UNPROJECT_PPT, v)
                for shift in (0, 1):  # rays at +0 or +8 bytes
                    buf = torch.full((3 * n + 2,), 7.0, dtype=torch.float64, device="cuda")
                    st = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
                    _lib.check(L.acm_unproject(ctypes.byref(cam), n, px.data_ptr(),
                                               buf[shift:].data_ptr(), 0, st.data_ptr(), None))
                    torch.cuda.synchronize()
                    b = buf.cpu().numpy()
                    assert b[0] == 7.0 or shift == 0
                    assert b[3 * n + shift:].tolist() == [7.0] * (2 - shift)  # nothing past the end
                    outs.append((b[shift:shift + 3 * n].view(np.int64), st.cpu().numpy()))
        finally:
            L.acm_set_tuning(_lib.TUNE_UNPROJECT_PPT, -1)
        for r, s in outs[1:]:
            assert np.array_equal(r, outs[0][0]) and np.array_equal(s, outs[0][1]), model


def test_newton_fast_random_cameras():
    """Randomised sweep of the certified fast Newton loops: 150 KB and 150
    RadTan cameras with random intrinsics and distortion (about a third of
    them beyond the fast loops' per-camera bounds, which must then take the
    reference loop), 40K pixels each spread over the image and a margin.
    Statuses with and without ACM_REFERENCE_NEWTON are identical for every
    pixel, rays within 64 ulp of 1."""
    import ctypes
    import torch
    from apex_camera_models import _lib
    L = _lib.load()
    rng = np.random.default_rng(2024)
    n = 40_000
    st_on = torch.empty((n,), dtype=torch.uint8, device="cuda")
    st_off = torch.empty_like(st_on)
    r_on = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    r_off = torch.empty_like(r_on)
    failures = 0
    covered = {1: [0, 0], 2: [0, 0]}  # [beyond the fast loop's bound, within]
    for model in (2, 1):
        for _ in range(150):
            w, h = int(rng.integers(320, 1400)), int(rng.integers(240, 1100))
            f = rng.uniform(0.3, 1.2) * w
            base = [f, f * rng.uniform(0.95, 1.05), w * rng.uniform(0.4, 0.6),
                    h * rng.uniform(0.4, 0.6)]
            if model == 2:
                dist = list(rng.normal(0, [0.2, 0.1, 0.1, 0.15]))
                bound = 4 * abs(dist[0]) + 16 * abs(dist[1]) + 64 * abs(dist[2]) + \
                    256 * abs(dist[3])
                covered[model][int(bound <= 63)] += 1
            else:  # k1 k2 p1 p2 k3
                dist = list(rng.normal(0, [0.3, 0.1, 0.005, 0.005, 0.02]))
                bound = 8 * abs(dist[0]) + 64 * abs(dist[1]) + 512 * abs(dist[4]) + \
                    16 * (abs(dist[2]) + abs(dist[3]))
                covered[model][int(bound <= 15)] += 1
            params = base + dist
            cam = _lib.AcmCamera()
            _lib.check(L.acm_camera_init(ctypes.byref(cam), model,
                                         (ctypes.c_double * len(params))(*params),
                                         len(params), w, h))
            px = torch.as_tensor(np.stack([rng.uniform(-20, w + 20, n),
                                           rng.uniform(-20, h + 20, n)], 1), device="cuda")
            for flag, st, r in ((0, st_on, r_on), (_lib.REFERENCE_NEWTON, st_off, r_off)):
                _lib.check(L.acm_unproject(ctypes.byref(cam), n, px.data_ptr(), r.data_ptr(),
                                           flag, st.data_ptr(), None))
            torch.cuda.synchronize()
            if not torch.equal(st_on, st_off):
                failures += 1
                continue
            ok = st_off == 0
            d = (r_on[ok] - r_off[ok]).abs()
            fin = torch.isfinite(r_off[ok]).all(1)
            assert torch.equal(fin, torch.isfinite(r_on[ok]).all(1)), (model, params)
            if fin.any():
                assert float(d[fin].max()) <= 64 * 2.0 ** -52, (model, params)
    assert failures == 0, failures
    for model in (1, 2):  # both paths of the per-camera switch were exercised
        assert min(covered[model]) >= 15, covered


@pytest.mark.parametrize("layout", [0, 1])
@pytest.mark.parametrize("n", [1, 257, 300_001])
@pytest.mark.parametrize("model", range(7))
def test_project_unproject_fused_matches_two_calls(model, n, layout):
    """acm_project_unproject (BASELINE config 4's round trip in one pass)
    writes exactly what acm_project followed by acm_unproject of its pixels
    writes: pixels (NaN positions included), both statuses and the rays, bit
    for bit, AoS and SoA, on the synthetic cloud with its edge points (z <= 0,
    the origin, non-finite coordinates)."""
    import ctypes
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    params, (w, h) = samples.SAMPLES[model]
    cam = _model_obj(model, params, w, h).acm_camera()
    pts = samples.synthetic_points_device(n)
    if layout == 1:
        pts = pts.t().contiguous()
    sh = torch.cuda.current_stream().cuda_stream

    def bufs():
        return (torch.full((n, 2), -1.0, dtype=torch.float64, device="cuda"),
                torch.full((n,), 77, dtype=torch.uint8, device="cuda"),
                torch.full((n, 3) if layout == 0 else (3, n), -1.0, dtype=torch.float64,
                           device="cuda"),
                torch.full((n,), 77, dtype=torch.uint8, device="cuda"))
    a, b = bufs(), bufs()
    _lib.check(L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), layout, a[0].data_ptr(),
                             a[1].data_ptr(), None, sh))
    _lib.check(L.acm_unproject(ctypes.byref(cam), n, a[0].data_ptr(), a[2].data_ptr(), layout,
                               a[3].data_ptr(), sh))
    _lib.check(L.acm_project_unproject(ctypes.byref(cam), n, pts.data_ptr(), layout,
                                       b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(),
                                       b[3].data_ptr(), sh))
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        xh, yh = x.cpu().numpy(), y.cpu().numpy()
        assert xh.tobytes() == yh.tobytes() or np.array_equal(xh, yh, equal_nan=True)


def check_round_trip_vs_oracle(model, params, w, h, xyz, uv, st, rays, st2):
    """acm_project_unproject's four outputs against the oracle's project of the
    same points followed by the oracle's unproject of the ORACLE's own pixels
    (NaN pixels of failed projections included), the per-point loop of
    tests/projection_accuracy.rs:49-73 over mod.rs:256 / :271.  Statuses of
    both steps bit-exact; uv and rays within 1e-10 (floor 1); bit-exact values
    for the models without a transcendental (pixels: Pinhole, RadTan, DS, UCM,
    EUCM; rays: Pinhole, DS, UCM, EUCM), RadTan rays within 8 ulp of 1."""
    uv0, s0, _ = O.project(model, params, w, h, xyz)
    assert np.array_equal(st, s0), np.nonzero(st != s0)[0][:5]
    assert rel_err(uv, uv0, floor=1.0) <= TOL
    if model in NO_TRANSCENDENTAL_PROJECT:
        assert np.array_equal(uv, uv0, equal_nan=True)
    r0, s20 = O.unproject(model, params, w, h, uv0)
    assert np.array_equal(st2, s20), np.nonzero(st2 != s20)[0][:5]
    assert rel_err(rays, r0, floor=1.0) <= TOL
    if model in EXACT_RAYS_UNPROJECT:
        assert np.array_equal(rays, r0, equal_nan=True)
    if model == 1:
        assert ulps_of_one(rays[s20 == 0], r0[s20 == 0]) <= 8


@pytest.mark.parametrize("layout", ["aos", "soa"])
@pytest.mark.parametrize("model", range(7))
def test_project_unproject_fused_vs_oracle_golden(be, golden_dir, model, layout):
    """acm_project_unproject on every golden point set (edge points on every
    decision boundary, z <= 0, the origin, non-finite coordinates), pinned to
    the oracle directly, not only to the two-call path;
    its pixels and statuses also equal the frozen golden ones."""
    g, params, w, h = _golden(golden_dir, model)
    uv, st, rays, st2 = be.round_trip(model, params, w, h, g["xyz"], layout=layout)
    assert np.array_equal(st, g["proj_status"])
    assert rel_err(uv, g["uv"], floor=1.0) <= TOL
    check_round_trip_vs_oracle(model, params, w, h, g["xyz"], uv, st, rays, st2)


@pytest.mark.parametrize("model", range(7))
def test_project_unproject_layout_knob_same_bits(model):
    """ACM_TUNE_ROUND_TRIP (points per lane 1 / 2 / 4, LDS-staged or direct
    AoS ray stores) selects among kernels with identical outputs: every
    setting writes the default's pixels, statuses and rays bit for bit,
    on a ragged size with the synthetic cloud's edge points."""
    import ctypes
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    params, (w, h) = samples.SAMPLES[model]
    cam = _model_obj(model, params, w, h).acm_camera()
    n = 300_001
    pts = samples.synthetic_points_device(n)
    sh = torch.cuda.current_stream().cuda_stream

    def run():
        out = (torch.empty((n, 2), dtype=torch.float64, device="cuda"),
               torch.empty((n,), dtype=torch.uint8, device="cuda"),
               torch.empty((n, 3), dtype=torch.float64, device="cuda"),
               torch.empty((n,), dtype=torch.uint8, device="cuda"))
        _lib.check(L.acm_project_unproject(ctypes.byref(cam), n, pts.data_ptr(), 0,
                                           out[0].data_ptr(), out[1].data_ptr(),
                                           out[2].data_ptr(), out[3].data_ptr(), sh))
        torch.cuda.synchronize()
        return [t.cpu().numpy().tobytes() for t in out]
    ref = run()
    try:
        for v in (1, 2, 4, 9, 10, 12, 17, 18, 20):
            L.acm_set_tuning(_lib.TUNE_ROUND_TRIP, v)
            assert run() == ref, v
    finally:
        L.acm_set_tuning(_lib.TUNE_ROUND_TRIP, -1)
