"""The reference's integration tests (/root/reference/tests/projection_accuracy.rs,
model_conversions.rs, parameter_estimation.rs) and in-file unit tests,
restated against the Python mirror of the API -- every projection runs in
libacm.so's HIP kernels.  Test names follow the Rust ones."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SAMPLES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "samples")


def load(cls_name, fname):
    import apex_camera_models as acm
    return getattr(acm, cls_name).load_from_yaml(os.path.join(SAMPLES_DIR, fname))


def normalize(p):
    p = np.asarray(p, dtype=np.float64)
    return p / np.linalg.norm(p)


def pinhole_640():
    import apex_camera_models as acm
    m = acm.PinholeModel.new([500.0, 500.0, 320.0, 240.0])
    m.resolution.width, m.resolution.height = 640, 480
    return m


# ---------------------------------------------------- projection_accuracy.rs
def test_projection_behind_camera():
    from apex_camera_models import CameraModelError
    m = load("DoubleSphereModel", "double_sphere.yaml")
    with pytest.raises(CameraModelError):
        m.project([0.1, 0.2, -1.0])


def test_projection_at_center():
    from apex_camera_models import CameraModelError
    m = load("DoubleSphereModel", "double_sphere.yaml")
    with pytest.raises(CameraModelError):
        m.project([0.0, 0.0, 0.0])


def test_unprojection_validates_bounds():
    from apex_camera_models import CameraModelError
    m = pinhole_640()
    for p in ([-100.0, 100.0], [1000.0, 1000.0]):
        with pytest.raises(CameraModelError):
            m.unproject(p)


def test_projection_unprojection_consistency():
    m = pinhole_640()
    for p in ([0.0, 0.0, 1.0], [0.2, 0.1, 1.5], [-0.1, -0.2, 2.0]):
        ray = m.unproject(m.project(p))
        assert abs(float(np.dot(normalize(p), ray)) - 1.0) < 1e-6


def test_boundary_projections():
    from apex_camera_models.camera import ProjectionOutSideImage
    m = load("DoubleSphereModel", "double_sphere.yaml")
    for p in ([0.5, 0.0, 2.0], [-0.5, 0.0, 2.0], [0.0, 0.5, 2.0], [0.0, -0.5, 2.0]):
        try:
            u, v = m.project(p)
            assert 0 <= u < m.resolution.width and 0 <= v < m.resolution.height
        except ProjectionOutSideImage:
            pass


# ------------------------------------------------------ model_conversions.rs
FIVE = [[0.1, 0.1, 1.0], [0.3, 0.0, 1.5], [-0.2, 0.3, 2.0], [-0.3, -0.2, 1.8],
        [0.15, -0.25, 2.5]]


@pytest.mark.parametrize("cls_name,fname,min_dot", [
    ("DoubleSphereModel", "double_sphere.yaml", 0.99),
    ("KannalaBrandtModel", "kannala_brandt.yaml", 0.99),
    ("RadTanModel", "rad_tan.yaml", 0.99)])
def test_basic_operations(cls_name, fname, min_dot):
    from apex_camera_models import CameraModelError
    m = load(cls_name, fname)
    ok = 0
    for p in FIVE:
        try:
            uv = m.project(p)
        except CameraModelError:
            continue
        assert 0 <= uv[0] < m.resolution.width and 0 <= uv[1] < m.resolution.height
        try:
            ray = m.unproject(uv)
        except CameraModelError:
            continue
        assert float(np.dot(normalize(p), ray)) > min_dot
        ok += 1
    assert ok > 0


@pytest.mark.parametrize("cls_name,fname", [("UcmModel", "ucm.yaml"), ("EucmModel", "eucm.yaml")])
def test_ucm_eucm_basic_operations(cls_name, fname):
    from apex_camera_models import CameraModelError
    m = load(cls_name, fname)
    total = 0
    for p in FIVE:
        try:
            uv = m.project(p)
        except CameraModelError:
            continue
        total += 1
        if 0 <= uv[0] < m.resolution.width and 0 <= uv[1] < m.resolution.height:
            ray = m.unproject(uv)
            assert float(np.dot(normalize(p), ray)) > 0.99
    assert total > 0


def test_pinhole_basic_operations():
    from apex_camera_models import CameraModelError
    m = pinhole_640()
    ok = 0
    for p in FIVE:
        try:
            uv = m.project(p)
        except CameraModelError:
            continue
        ray = m.unproject(uv)
        assert float(np.dot(normalize(p), ray)) > 0.9999
        ok += 1
    assert ok > 0


# ---------------------------------------------------- parameter_estimation.rs
def _radtan_zero(model):
    import apex_camera_models as acm
    m = acm.RadTanModel.new(model.params()[:4] + [0.0] * 5)
    m.resolution = model.get_resolution()
    return m


def test_rad_tan_linear_estimation():
    from apex_camera_models import util
    model = load("RadTanModel", "rad_tan.yaml")
    p2, p3 = util.sample_points(model, 50)
    est = _radtan_zero(model)
    est.linear_estimation(p3, p2)
    assert any(abs(d) > 1e-10 for d in est.distortions)


def test_linear_estimation_with_insufficient_points():
    from apex_camera_models import util
    from apex_camera_models.camera import InvalidParams
    model = load("RadTanModel", "rad_tan.yaml")
    p2, p3 = util.sample_points(model, 2)
    with pytest.raises(InvalidParams):
        _radtan_zero(model).linear_estimation(p3, p2)


def test_linear_estimation_with_mismatched_points():
    from apex_camera_models import util
    from apex_camera_models.camera import InvalidParams
    model = load("RadTanModel", "rad_tan.yaml")
    p2, p3 = util.sample_points(model, 10)
    with pytest.raises(InvalidParams):
        _radtan_zero(model).linear_estimation(p3[:5], p2)


# ------------------------------------------------------------ in-file tests
def test_pinhole_doc_example():  # pinhole.rs:153-163
    u, v = pinhole_640().project([0.1, 0.2, 1.0])
    assert abs(u - 370.0) < 1e-6 and abs(v - 340.0) < 1e-6


def test_kb_project_unproject_identity():  # kannala_brandt.rs:897-944
    import apex_camera_models as acm
    m = acm.KannalaBrandtModel.new([461.58688085556616, 460.2811732644195, 366.28603126815506,
                                    249.08026891791644, -0.012523386218579752,
                                    0.057836801948828065, -0.08495347810986263,
                                    0.04362766880887814])
    m.resolution.width, m.resolution.height = 752, 480
    uv = m.project([0.1, 0.2, 1.0])
    ray = m.unproject(uv)
    np.testing.assert_allclose(ray, normalize([0.1, 0.2, 1.0]), atol=1e-5)


def test_kb_errors():  # kannala_brandt.rs:946-974
    import apex_camera_models as acm
    from apex_camera_models.camera import PointAtCameraCenter, PointIsOutSideImage
    m = load("KannalaBrandtModel", "kannala_brandt.yaml")
    with pytest.raises(PointAtCameraCenter):
        m.project([0.0, 0.0, 0.0])
    with pytest.raises(PointIsOutSideImage):
        m.project([0.1, 0.2, -1.0])
    with pytest.raises(PointIsOutSideImage):
        m.unproject([m.resolution.width + 10.0, m.resolution.height + 10.0])


def test_sample_points():  # util/mod.rs:65-95
    from apex_camera_models import util
    m = load("DoubleSphereModel", "double_sphere.yaml")
    p2, p3 = util.sample_points(m, 100)
    assert p2.shape[0] > 0 and p2.shape[0] == p3.shape[0]
    assert bool((p3[:, 2] > 0).all())


def test_compute_reprojection_error_zero_on_own_samples():
    from apex_camera_models import util
    m = load("DoubleSphereModel", "double_sphere.yaml")
    p2, p3 = util.sample_points(m, 500)
    pe = util.compute_reprojection_error(m, p3, p2)
    assert pe.rmse < 1e-9 and pe.max < 1e-9 and pe.n_valid == p2.shape[0]
