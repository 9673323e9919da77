"""linear_estimation (GPU TSQR) and the LM model conversion against CPU
references: numpy's SVD least squares on the oracle-assembled A, b (the
reference's nalgebra SVD solve), and scipy's bounded least_squares on the
oracle residual/Jacobian (apex-solver's LM source is absent: the conversion
is judged by the optimum it reaches, not by iterate-for-iterate parity)."""
import numpy as np
import pytest

import oracle as O
from test_oracle import SAMPLES

pytestmark = pytest.mark.gpu

KB, DS, UCM, EUCM, RADTAN = 2, 3, 4, 5, 1


def _model(mid, params, w, h):
    from _backends import GpuBackend
    return GpuBackend()._model(mid, params, w, h)


def _sampled(src, n):
    params, (w, h) = SAMPLES[src]
    uv, xyz, _ = O.sample_points(src, params, w, h, n)
    return uv, xyz, w, h


def _lstsq_ref(model, params, xyz, uv):
    A, b, k = O.linear_estimation_system(model, params, xyz, uv)
    assert k > 0
    # nalgebra svd.solve(b, eps): singular values <= eps dropped
    U, s, Vt = np.linalg.svd(A, full_matrices=False)
    eps = 2.220446049250313e-16 if model == KB else 1e-10
    coef = np.where(s > eps, (U.T @ b) / np.where(s > eps, s, 1.0), 0.0)
    return Vt.T @ coef


@pytest.mark.parametrize("target,src", [(DS, KB), (UCM, KB), (EUCM, KB), (KB, DS), (RADTAN, KB),
                                        (RADTAN, RADTAN), (KB, KB), (DS, UCM)])
def test_linear_estimation_matches_svd_reference(target, src):
    import torch
    uv, xyz, w, h = _sampled(src, 2000)
    sp, _ = SAMPLES[src]
    init = {KB: sp[:4] + [0.0] * 4, DS: sp[:4] + [0.5, 0.1], UCM: sp[:4] + [0.5],
            EUCM: sp[:4] + [0.5, 1.0], RADTAN: sp[:4] + [0.0] * 5}[target]
    m = _model(target, init, w, h)
    m.linear_estimation(torch.as_tensor(xyz), torch.as_tensor(uv))
    x = _lstsq_ref(target, init, xyz, uv)
    got = m.params()
    if target == KB:
        est = got[4:8]
    elif target == RADTAN:
        est = [got[4], got[5], got[8]]
        assert got[6] == 0.0 and got[7] == 0.0
    else:
        est = [got[4]]
        a = x[0]
        lo, hi = {DS: (0.0, 1.0), UCM: (0.0, np.inf), EUCM: (0.0, 2.0)}[target]
        x = [0.01 if a <= lo else (hi if a > hi else a)]  # the reference's clamps
        if target == DS:
            assert got[5] == 0.0
        if target == EUCM:
            assert got[5] == 1.0
    np.testing.assert_allclose(est, x, rtol=1e-8, atol=1e-12)


def test_linear_estimation_errors_like_reference():
    import torch
    from apex_camera_models.camera import InvalidParams
    # tests/parameter_estimation.rs:40-63: RadTan with 2 points -> error
    uv, xyz, w, h = _sampled(RADTAN, 2)
    assert len(uv) < 3
    m = _model(RADTAN, SAMPLES[RADTAN][0][:4] + [0.0] * 5, w, h)
    with pytest.raises(InvalidParams):
        m.linear_estimation(torch.as_tensor(xyz), torch.as_tensor(uv))
    # tests/parameter_estimation.rs:8-37: 50 samples -> nonzero distortion
    uv, xyz, w, h = _sampled(RADTAN, 50)
    m.linear_estimation(torch.as_tensor(xyz), torch.as_tensor(uv))
    assert any(abs(d) > 1e-10 for d in m.distortions)
    # mismatched counts (tests/parameter_estimation.rs:66-91)
    with pytest.raises(InvalidParams):
        m.linear_estimation(torch.as_tensor(xyz[:5]), torch.as_tensor(uv))
    # KB needs >= 4 points (kannala_brandt.rs:174-178)
    mk = _model(KB, SAMPLES[KB][0][:4] + [0.0] * 4, 512, 512)
    with pytest.raises(InvalidParams):
        mk.linear_estimation(torch.as_tensor(xyz[:3]), torch.as_tensor(uv[:3]))


def test_linear_estimation_deterministic_large():
    """TSQR over 1M correspondences: fixed reduction order -> bit-identical."""
    import torch
    from apex_camera_models import util
    params, (w, h) = SAMPLES[KB]
    src = _model(KB, params, w, h)
    uv, xyz = util.sample_points(src, 1_000_000)
    a = _model(DS, params[:4] + [0.5, 0.1], w, h)
    b = _model(DS, params[:4] + [0.5, 0.1], w, h)
    a.linear_estimation(xyz, uv)
    b.linear_estimation(xyz, uv)
    assert a.alpha == b.alpha
    ref = _lstsq_ref(DS, params[:4] + [0.5, 0.1], xyz.cpu().numpy(), uv.cpu().numpy())
    assert abs(a.alpha - ref[0]) <= 1e-9 * abs(ref[0])


def _scipy_reference(target, init, bounds, xyz, uv, w, h):
    from scipy.optimize import least_squares
    P = len(init)
    lo = np.array([bounds.get(i, (-np.inf, np.inf))[0] for i in range(P)])
    hi = np.array([bounds.get(i, (-np.inf, np.inf))[1] for i in range(P)])

    def fun(p):
        r, _, _ = O.residual_jacobian(target, p, w, h, xyz, uv, 0, want_jac=False)
        return r.ravel()

    def jac(p):
        _, J, _ = O.residual_jacobian(target, p, w, h, xyz, uv, 0)
        return J.reshape(P, -1).T

    x0 = np.clip(np.array(init), lo, hi)
    res = least_squares(fun, x0, jac=jac, bounds=(lo, hi), method="trf", xtol=1e-15,
                        ftol=1e-15, gtol=1e-15, max_nfev=2000)
    return res.x


@pytest.mark.parametrize("target", ["double_sphere", "ucm", "eucm", "kannala_brandt"])
def test_conversion_from_kb_reaches_reference_optimum(target):
    """camera_converter.rs on samples/kannala_brandt.yaml with the CLI default
    of 500 points: GPU pipeline (sample_points -> linear_estimation -> LM)
    vs scipy's bounded TRF on the oracle residuals from the same linear
    initialisation.  README.md:163-166 quotes mean errors of 0.008 px (DS),
    0.145 px (UCM), 0.314 px (EUCM) for this conversion."""
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, util
    from apex_camera_models.optimizer import CONVERTER_BOUNDS
    params, (w, h) = SAMPLES[KB]
    src = KannalaBrandtModel._from_params(params, Resolution(w, h))
    uv, xyz = util.sample_points(src, 500)
    met = conversion.convert(src, target, xyz, uv)
    assert met.convergence_status == "Converged", met.lm_termination
    got = met.final_reprojection_error.mean
    # scipy from the same linear-estimation start
    start = conversion._init_target(target, src)
    start.linear_estimation(xyz, uv)
    tid = start.MODEL_ID
    ref_p = _scipy_reference(tid, start.params(), CONVERTER_BOUNDS[target],
                             xyz.cpu().numpy(), uv.cpu().numpy(), w, h)
    ref_stats, _ = O.reprojection_error(tid, ref_p, w, h, xyz.cpu().numpy(), uv.cpu().numpy())
    print(target, "gpu LM mean err", got, "scipy", ref_stats["mean"], met.lm_iterations,
          met.lm_termination)
    assert got <= ref_stats["mean"] * 1.02 + 1e-9
    # README.md:163-166 (unspecified hardware/version): 0.008 / 0.145 / 0.314 px.
    # scipy and this LM agree on the optimum of THIS data to ~1e-7 relative
    # (DS 0.00893 px), so the README figures are held only as a sanity bound.
    readme = {"double_sphere": 0.008, "ucm": 0.145, "eucm": 0.314}.get(target)
    if readme is not None:
        assert got <= 2.0 * readme


def test_sample_points_range_concatenates_to_full():
    from apex_camera_models import KannalaBrandtModel, Resolution, util
    from apex_camera_models.distributed import gpu_sample_points_range, grid_row_range
    params, (w, h) = SAMPLES[KB]
    m = KannalaBrandtModel._from_params(params, Resolution(w, h))
    n = 200_000
    uv, xyz = util.sample_points(m, n)
    ncx = int(round(np.sqrt(n * (w / h))))
    ncy = int(round(np.sqrt(n * (h / w))))
    fn = gpu_sample_points_range(m, n)
    parts = [fn(*grid_row_range(ncx, ncy, r, 3)) for r in range(3)]
    import torch
    assert torch.equal(torch.cat([p[0] for p in parts]), uv)
    assert torch.equal(torch.cat([p[1] for p in parts]), xyz)


def test_lm_rccl_allreduce_single_rank():
    """The LM all-reduce hook through RCCL (world 1: sum == identity, so the
    optimum is bit-identical to the un-reduced run)."""
    import socket

    import torch.distributed as dist
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, util
    from apex_camera_models.distributed import rccl_allreduce
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        params, (w, h) = SAMPLES[KB]
        src = KannalaBrandtModel._from_params(params, Resolution(w, h))
        uv, xyz = util.sample_points(src, 500)
        a = conversion.convert(src, "double_sphere", xyz, uv)
        b = conversion.convert(src, "double_sphere", xyz, uv, allreduce=rccl_allreduce())
        assert a.model.params() == b.model.params()
        assert a.lm_iterations == b.lm_iterations
    finally:
        dist.destroy_process_group()
