"""Writes tests/golden/reference_kats.json: the known answers the reference's
own tests assert, transcribed as data with their source (file:line in
/root/reference, amin-abouee/apex-camera-models v0.4.1).

The reference is Rust and cannot be compiled or run in this image (no
rustc/cargo), so these assertions -- plus tests/golden/samples/*.yaml, the
reference's own fixture files -- are what pins the oracle (oracle/).
Run: python tests/golden/make_reference_kats.py
"""
import json
import os

PINHOLE_500 = [500.0, 500.0, 320.0, 240.0]
KB_SAMPLE = [461.58688085556616, 460.2811732644195, 366.28603126815506, 249.08026891791644,
             -0.012523386218579752, 0.057836801948828065, -0.08495347810986263,
             0.04362766880887814]
KB_YAML = [190.97847715128717, 190.9733070521226, 254.93170605935475, 256.8974428996504,
           0.0034823894022493434, 0.0007150348452162257, -0.0020532361418706202,
           0.00020293673591811182]
DS_YAML = [348.112754378549, 347.1109973814674, 365.8121721753254, 249.3555778487899,
           0.5657413673629862, -0.24425190195168348]
UCM_SAMPLE = [1313.83, 1313.27, 960.471, 546.981, 1.01674]
EUCM_SAMPLE = [1313.83, 1313.27, 960.471, 546.981, 1.01674, 0.5]
RADTAN_YAML = [461.629, 460.152, 362.680, 246.049, -0.28340811, 0.07395907, 0.00019359,
               1.76187114e-05, 0.0]
FOV_YAML = [379.045, 379.008, 505.512, 509.969, 0.9259487501905697]  # fov.rs:508-522, samples/fov.yaml
FIVE_POINTS = [[0.1, 0.1, 1.0], [0.3, 0.0, 1.5], [-0.2, 0.3, 2.0], [-0.3, -0.2, 1.8],
               [0.15, -0.25, 2.5]]  # tests/model_conversions.rs:9-17

KATS = {
    "project_value": [
        {"model": "pinhole", "params": PINHOLE_500, "res": [640, 480], "point": [0.1, 0.2, 1.0],
         "expect": [370.0, 340.0], "tol": 1e-6, "src": "src/camera/pinhole.rs:153-163"},
    ],
    "project_status": [
        {"model": "kannala_brandt", "params": KB_SAMPLE, "res": [752, 480],
         "point": [0.0, 0.0, 0.0], "status": "PointAtCameraCenter",
         "src": "src/camera/kannala_brandt.rs:947-953"},
        {"model": "kannala_brandt", "params": KB_SAMPLE, "res": [752, 480],
         "point": [0.1, 0.2, -1.0], "status": "PointIsOutSideImage",
         "src": "src/camera/kannala_brandt.rs:956-962"},
        {"model": "double_sphere", "params": DS_YAML, "res": [752, 480],
         "point": [0.0, 0.0, 0.0], "status": "PointIsOutSideImage",
         "src": "src/camera/double_sphere.rs:762-801; tests/projection_accuracy.rs:20-29"},
        {"model": "double_sphere", "params": DS_YAML, "res": [752, 480],
         "point": [0.1, 0.2, -1.0], "status": "PointIsOutSideImage",
         "src": "src/camera/double_sphere.rs:804-810; tests/projection_accuracy.rs:9-18"},
        {"model": "ucm", "params": UCM_SAMPLE, "res": [752, 480], "point": [0.0, 0.0, 0.0],
         "status": "PointIsOutSideImage", "src": "src/camera/ucm.rs:646-674"},
        {"model": "ucm", "params": UCM_SAMPLE, "res": [752, 480], "point": [0.1, 0.2, -1.0],
         "status": "PointIsOutSideImage", "src": "src/camera/ucm.rs:677-684"},
        {"model": "eucm", "params": EUCM_SAMPLE, "res": [752, 480], "point": [0.0, 0.0, 0.0],
         "status": "PointIsOutSideImage", "src": "src/camera/eucm.rs:634-662"},
        {"model": "eucm", "params": EUCM_SAMPLE, "res": [752, 480], "point": [0.1, 0.2, -1.0],
         "status": "PointIsOutSideImage", "src": "src/camera/eucm.rs:665-672"},
        {"model": "fov", "params": FOV_YAML, "res": [752, 480], "point": [0.0, 0.0, 0.0],
         "status": "PointAtCameraCenter", "src": "src/camera/fov.rs:647-655"},
        {"model": "fov", "params": FOV_YAML, "res": [752, 480], "point": [0.1, 0.2, -1.0],
         "status": "PointAtCameraCenter", "src": "src/camera/fov.rs:658-666"},
    ],
    # `if let Ok(p) = model.project(..)`: any error is accepted, an Ok result
    # must land within tol of the principal point
    "project_near_center_if_ok": [
        {"model": "fov", "params": FOV_YAML, "res": [752, 480], "point": [0.0, 0.0, 0.1],
         "tol": 1e-3, "src": "src/camera/fov.rs:638-645"},
    ],
    # DS/UCM/EUCM near-origin point: either PointIsOutSideImage or ~(cx, cy) +-1e-3
    "project_near_center": [
        {"model": m, "params": p, "res": [752, 480], "point": [0.0, 0.0, 1e-9], "tol": 1e-3,
         "src": s}
        for m, p, s in [("double_sphere", DS_YAML, "src/camera/double_sphere.rs:741-760"),
                        ("ucm", UCM_SAMPLE, "src/camera/ucm.rs:646-660"),
                        ("eucm", EUCM_SAMPLE, "src/camera/eucm.rs:634-648")]
    ],
    "unproject_status": [
        {"model": "kannala_brandt", "params": KB_SAMPLE, "res": [752, 480],
         "point": [762.0, 490.0], "status": "PointIsOutSideImage",
         "src": "src/camera/kannala_brandt.rs:965-974"},
        {"model": "pinhole", "params": PINHOLE_500, "res": [640, 480], "point": [-100.0, 100.0],
         "status": "PointIsOutSideImage", "src": "tests/projection_accuracy.rs:31-46"},
        {"model": "pinhole", "params": PINHOLE_500, "res": [640, 480],
         "point": [1000.0, 1000.0], "status": "PointIsOutSideImage",
         "src": "tests/projection_accuracy.rs:31-46"},
    ],
    # project -> unproject must return the normalised input within `tol` per component
    "round_trip": [
        {"model": "kannala_brandt", "params": KB_SAMPLE, "res": [752, 480],
         "point": [0.1, 0.2, 1.0], "tol": 1e-5, "in_bounds": True,
         "src": "src/camera/kannala_brandt.rs:897-944"},
        {"model": "double_sphere", "params": DS_YAML, "res": [752, 480],
         "point": [0.5, -0.3, 2.0], "tol": 1e-6, "in_bounds": True,
         "src": "src/camera/double_sphere.rs:734-758"},
        {"model": "rad_tan", "params": RADTAN_YAML, "res": [752, 480],
         "point": [0.5, -0.3, 2.0], "tol": 1e-6, "in_bounds": True,
         "src": "src/camera/rad_tan.rs:866-890"},
        {"model": "ucm", "params": UCM_SAMPLE, "res": [752, 480], "point": [0.1, 0.1, 3.0],
         "tol": 1e-4, "in_bounds": False, "src": "src/camera/ucm.rs:588-617"},
        {"model": "ucm", "params": UCM_SAMPLE, "res": [752, 480], "point": [0.0, 0.0, 1.0],
         "tol": 1e-6, "in_bounds": False, "center_tol": 1.0, "src": "src/camera/ucm.rs:620-642"},
        {"model": "eucm", "params": EUCM_SAMPLE, "res": [752, 480], "point": [0.1, 0.1, 3.0],
         "tol": 1e-4, "in_bounds": False, "src": "src/camera/eucm.rs:576-605"},
        {"model": "eucm", "params": EUCM_SAMPLE, "res": [752, 480], "point": [0.0, 0.0, 1.0],
         "tol": 1e-6, "in_bounds": False, "center_tol": 1.0, "src": "src/camera/eucm.rs:608-630"},
        {"model": "fov", "params": FOV_YAML, "res": [752, 480], "point": [0.1, 0.1, 3.0],
         "tol": 1e-4, "in_bounds": False, "finite": True, "src": "src/camera/fov.rs:576-606"},
        {"model": "fov", "params": FOV_YAML, "res": [752, 480], "point": [0.0, 0.0, 1.0],
         "tol": 1e-6, "in_bounds": False, "center_tol": 1.0, "src": "src/camera/fov.rs:609-631"},
    ],
    # dot(normalize(p), unproject(project(p))) >= min_dot for successful projections
    "round_trip_dot": [
        {"model": "pinhole", "params": PINHOLE_500, "res": [640, 480],
         "points": [[0.0, 0.0, 1.0], [0.2, 0.1, 1.5], [-0.1, -0.2, 2.0]], "min_dot": 1.0 - 1e-6,
         "src": "tests/projection_accuracy.rs:49-73"},
        {"model": "pinhole", "params": PINHOLE_500, "res": [640, 480], "points": FIVE_POINTS,
         "min_dot": 0.9999, "src": "tests/model_conversions.rs:142-159"},
        {"model": "double_sphere", "params": DS_YAML, "res": [752, 480], "points": FIVE_POINTS,
         "min_dot": 0.99, "src": "tests/model_conversions.rs:20-38"},
        {"model": "kannala_brandt", "params": KB_YAML, "res": [512, 512], "points": FIVE_POINTS,
         "min_dot": 0.99, "src": "tests/model_conversions.rs:41-59"},
        {"model": "rad_tan", "params": RADTAN_YAML, "res": [752, 480], "points": FIVE_POINTS,
         "min_dot": 0.99, "src": "tests/model_conversions.rs:62-80"},
    ],
    "validate_params": [
        {"model": "pinhole", "params": [-500.0, 500.0, 320.0, 240.0],
         "error": "FocalLengthMustBePositive", "src": "tests/model_conversions.rs:172-176"},
        {"model": "pinhole", "params": [0.0, 500.0, 320.0, 240.0],
         "error": "FocalLengthMustBePositive", "src": "tests/model_conversions.rs:178-179"},
        {"model": "pinhole", "params": [500.0, 500.0, "inf", 240.0],
         "error": "PrincipalPointMustBeFinite", "src": "tests/model_conversions.rs:181-182"},
        {"model": "pinhole", "params": [500.0, 500.0, 320.0, "nan"],
         "error": "PrincipalPointMustBeFinite", "src": "tests/model_conversions.rs:184-185"},
        {"model": "fov", "params": FOV_YAML, "error": "Valid", "src": "src/camera/fov.rs:668-673"},
    ] + [
        {"model": "fov", "params": FOV_YAML[:4] + [w], "error": "InvalidParams",
         "src": "src/camera/fov.rs:677-703"} for w in (0.0, -0.5, 3.5, "nan")
    ] + [
        {"model": "fov", "params": [0.0] + FOV_YAML[1:], "error": "FocalLengthMustBePositive",
         "src": "src/camera/fov.rs:705-714"},
    ],
    "param_count_errors": [
        {"model": "double_sphere", "n": 2}, {"model": "kannala_brandt", "n": 1},
        {"model": "rad_tan", "n": 2}, {"model": "ucm", "n": 1}, {"model": "eucm", "n": 1},
        {"model": "pinhole", "n": 1},
        {"model": "fov", "n": 4, "src": "src/camera/fov.rs:750-756"},
    ],
    "param_count_errors_src": "tests/model_conversions.rs:162-169",
    "yaml_values": {
        "kannala_brandt": {"params": KB_YAML, "res": [512, 512],
                           "src": "src/camera/kannala_brandt.rs:864-884"},
        "double_sphere": {"params": DS_YAML, "res": [752, 480],
                          "src": "src/camera/double_sphere.rs:677-692"},
        "rad_tan": {"params": RADTAN_YAML, "res": [752, 480], "src": "src/camera/rad_tan.rs:806-825"},
        "fov": {"params": FOV_YAML, "res": [752, 480], "src": "src/camera/fov.rs:524-537"},
    },
    "sample_points": {"model": "double_sphere", "params": DS_YAML, "res": [752, 480], "n": 100,
                      "src": "src/util/mod.rs:70-95"},
    "radtan_linear_estimation": {"params": RADTAN_YAML, "res": [752, 480], "n_ok": 50,
                                 "n_too_few": 2, "src": "tests/parameter_estimation.rs:8-63"},
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(out, "w") as f:
        json.dump(KATS, f, indent=1)
    print("wrote", out)
