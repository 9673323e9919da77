"""YAML load/save of the cam0 format, mirroring /root/reference/tests/
yaml_serialization.rs and the in-file load tests (double_sphere.rs:677-692,
kannala_brandt.rs:864-895, rad_tan.rs:806-860), on the reference's own
fixture files (tests/golden/samples/*.yaml, copied from samples/).  Host-side
only: no GPU needed."""
import math
import os

import pytest

SAMPLES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "samples")


def path(name):
    return os.path.join(SAMPLES_DIR, name)


def test_double_sphere_load_values():  # double_sphere.rs:677-692
    from apex_camera_models import DoubleSphereModel
    m = DoubleSphereModel.load_from_yaml(path("double_sphere.yaml"))
    assert m.intrinsics.fx == 348.112754378549
    assert m.intrinsics.fy == 347.1109973814674
    assert m.intrinsics.cx == 365.8121721753254
    assert m.intrinsics.cy == 249.3555778487899
    assert m.alpha == 0.5657413673629862
    assert m.xi == -0.24425190195168348
    assert (m.resolution.width, m.resolution.height) == (752, 480)


def test_kannala_brandt_load_values():  # kannala_brandt.rs:864-884
    from apex_camera_models import KannalaBrandtModel
    m = KannalaBrandtModel.load_from_yaml(path("kannala_brandt.yaml"))
    assert abs(m.intrinsics.fx - 190.97847715128717) < 1e-9
    assert abs(m.intrinsics.cy - 256.8974428996504) < 1e-9
    assert (m.resolution.width, m.resolution.height) == (512, 512)
    assert abs(m.distortions[0] - 0.0034823894022493434) < 1e-9
    assert abs(m.distortions[3] - 0.00020293673591811182) < 1e-9
    assert m.get_model_name() == "kannala_brandt"


def test_rad_tan_load_values():  # rad_tan.rs:806-825
    from apex_camera_models import RadTanModel
    m = RadTanModel.load_from_yaml(path("rad_tan.yaml"))
    assert m.intrinsics.fx == 461.629 and m.intrinsics.cy == 246.049
    assert m.distortions == [-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05, 0.0]


def test_load_missing_file_is_io_error():  # kannala_brandt.rs:886-895
    from apex_camera_models import KannalaBrandtModel
    from apex_camera_models.camera import IOError_
    with pytest.raises(IOError_):
        KannalaBrandtModel.load_from_yaml(path("non_existent_file.yaml"))


@pytest.mark.parametrize("cls_name,fname", [
    ("DoubleSphereModel", "double_sphere.yaml"), ("RadTanModel", "rad_tan.yaml"),
    ("UcmModel", "ucm.yaml"), ("EucmModel", "eucm.yaml"), ("KannalaBrandtModel",
                                                          "kannala_brandt.yaml"),
    ("PinholeModel", "pinhole.yaml"), ("FovModel", "fov.yaml")])
def test_yaml_round_trip(tmp_path, cls_name, fname):  # tests/yaml_serialization.rs
    import apex_camera_models as acm
    cls = getattr(acm, cls_name)
    m = cls.load_from_yaml(path(fname))
    out = str(tmp_path / "out" / fname)
    m.save_to_yaml(out)
    r = cls.load_from_yaml(out)
    assert r.params() == m.params()
    assert (r.resolution.width, r.resolution.height) == (m.resolution.width, m.resolution.height)
    assert r.get_distortion() == m.get_distortion()


def test_new_param_count_and_validation():  # tests/model_conversions.rs:162-186
    import apex_camera_models as acm
    from apex_camera_models.camera import (FocalLengthMustBePositive, InvalidParams,
                                           PrincipalPointMustBeFinite)
    for cls, n in [(acm.DoubleSphereModel, 2), (acm.KannalaBrandtModel, 1),
                   (acm.RadTanModel, 2), (acm.UcmModel, 1), (acm.EucmModel, 1),
                   (acm.PinholeModel, 1)]:
        with pytest.raises(InvalidParams):
            cls.new([500.0] * n)
    with pytest.raises(FocalLengthMustBePositive):
        acm.PinholeModel.new([-500.0, 500.0, 320.0, 240.0])
    with pytest.raises(FocalLengthMustBePositive):
        acm.PinholeModel.new([0.0, 500.0, 320.0, 240.0])
    with pytest.raises(PrincipalPointMustBeFinite):
        acm.PinholeModel.new([500.0, 500.0, math.inf, 240.0])
    with pytest.raises(PrincipalPointMustBeFinite):
        acm.PinholeModel.new([500.0, 500.0, 320.0, math.nan])


def test_validate_params_ds():  # double_sphere.rs:811-854
    import apex_camera_models as acm
    from apex_camera_models.camera import FocalLengthMustBePositive, InvalidParams
    m = acm.DoubleSphereModel.load_from_yaml(path("double_sphere.yaml"))
    m.validate_params()
    m.alpha = 0.0
    with pytest.raises(InvalidParams, match=r"alpha must be in \(0, 1\]"):
        m.validate_params()
    m.alpha = 1.1
    with pytest.raises(InvalidParams):
        m.validate_params()
    m.alpha = 0.5
    m.xi = math.nan
    with pytest.raises(InvalidParams, match="xi must be finite"):
        m.validate_params()
    m.xi = 0.1
    m.intrinsics.fx = 0.0
    with pytest.raises(FocalLengthMustBePositive):
        m.validate_params()


def test_model_names_and_getters():  # mod.rs:583-620, kannala_brandt.rs:976-997
    import apex_camera_models as acm
    assert acm.DoubleSphereModel.new([350.0, 350.0, 320.0, 240.0, 0.58, -0.18]).get_model_name() \
        == "double_sphere"
    assert acm.EucmModel.new([350.0, 350.0, 320.0, 240.0, 1.0, 0.5]).get_model_name() == "eucm"
    assert acm.FovModel.new([379.045, 379.008, 505.512, 509.969, 0.92]).get_model_name() == "fov"
    assert acm.KannalaBrandtModel.new([460.0, 460.0, 320.0, 240.0, -0.01, 0.05, -0.08, 0.04]) \
        .get_model_name() == "kannala_brandt"
    assert acm.PinholeModel.new([460.0, 460.0, 320.0, 240.0]).get_model_name() == "pinhole"
    assert acm.RadTanModel.new([460.0, 460.0, 320.0, 240.0, -0.28, 0.07, 0.0002, 0.00002, 0.0]) \
        .get_model_name() == "rad_tan"
    assert acm.UcmModel.new([350.0, 350.0, 320.0, 240.0, 0.8]).get_model_name() == "ucm"
    ds = acm.DoubleSphereModel.new([350.0, 350.0, 320.0, 240.0, 0.58, -0.18])
    assert ds.get_distortion() == [0.58, -0.18]  # [alpha, xi] (double_sphere.rs:636-638)


def test_fov_reference_kats():
    """fov.rs:524-537 (samples/fov.yaml values), :668-714 (validate_params),
    :750-756 (parameter count) -- tests/golden/reference_kats.json."""
    import apex_camera_models as acm
    import kat_suite
    from _backends import parse_params
    from apex_camera_models.camera import FocalLengthMustBePositive, InvalidParams
    y = kat_suite.KATS["yaml_values"]["fov"]
    m = acm.FovModel.load_from_yaml(path("fov.yaml"))
    assert m.params() == y["params"]
    assert (m.resolution.width, m.resolution.height) == tuple(y["res"])
    errs = {"Valid": None, "InvalidParams": InvalidParams,
            "FocalLengthMustBePositive": FocalLengthMustBePositive}
    for k in kat_suite.KATS["validate_params"]:
        if k["model"] != "fov":
            continue
        mm = acm.FovModel.new(parse_params(k["params"]))
        if errs[k["error"]] is None:
            mm.validate_params()
        else:
            with pytest.raises(errs[k["error"]]):
                mm.validate_params()
    with pytest.raises(InvalidParams):
        acm.FovModel.new([379.045, 379.008, 505.512, 509.969])
