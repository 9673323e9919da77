"""cam0 YAML load/save (src/camera/mod.rs:412-578 `yaml_io`, plus the
KB / RadTan custom loaders kannala_brandt.rs:593-696, rad_tan.rs:~560-620).

Host-side configuration only (not on the hot path).  Uses yaml.safe_load.
"""
from __future__ import annotations

import os

import yaml


def _err(kind, msg):
    from . import camera
    return getattr(camera, kind)(msg)


def _floats(seq, what):
    out = []
    for k, x in enumerate(seq):
        if isinstance(x, bool) or not isinstance(x, float):
            # yaml-rust `as_f64` only accepts real (float) scalars
            raise _err("InvalidParams", f"Invalid {what}[{k}]: not a float")
        out.append(float(x))
    return out


def load_camera_yaml(cls, path):
    from . import camera
    try:
        with open(path, "r") as f:
            text = f.read()
    except OSError as e:
        raise camera.IOError_(str(e)) from None
    try:
        doc = yaml.safe_load(text)
    except yaml.YAMLError as e:
        raise camera.YamlError(str(e)) from None
    if not doc:
        raise camera.InvalidParams("Empty YAML document")
    cam = doc.get("cam0") if isinstance(doc, dict) else None
    if not isinstance(cam, dict):
        raise camera.InvalidParams("Missing 'cam0' node in YAML")
    intr = cam.get("intrinsics")
    if not isinstance(intr, list):
        raise camera.InvalidParams("YAML missing 'intrinsics' array under 'cam0'")
    res = cam.get("resolution")
    if not isinstance(res, list) or len(res) < 2:
        raise camera.InvalidParams("Resolution array must have at least 2 elements")
    if not all(isinstance(r, int) and not isinstance(r, bool) for r in res[:2]):
        raise camera.InvalidParams("Invalid width/height: not an integer")
    resolution = camera.Resolution(int(res[0]) & 0xFFFFFFFF, int(res[1]) & 0xFFFFFFFF)
    if cls in (camera.KannalaBrandtModel, camera.RadTanModel):
        need = 4 if cls is camera.KannalaBrandtModel else 5
        if len(intr) < 4:
            raise camera.InvalidParams("Intrinsics array in YAML must have at least 4 elements")
        dist = cam.get("distortion")
        if not isinstance(dist, list) or len(dist) < need:
            raise camera.InvalidParams("Missing or invalid 'distortion' array in YAML")
        p = _floats(intr[:4], "intrinsics") + _floats(dist[:need], "distortion")
    else:
        if len(intr) < cls.NUM_PARAMS:
            raise camera.InvalidParams(
                f"Intrinsics array must have at least {cls.NUM_PARAMS} elements, got {len(intr)}")
        p = _floats(intr, "intrinsics")
        if len(p) != cls.NUM_PARAMS:
            raise camera.InvalidParams(
                f"Expected {cls.NUM_PARAMS} intrinsics values, got {len(p)}")
    model = cls._from_params(p, resolution)
    model.validate_params()
    return model


def save_camera_yaml(model, path):
    from . import camera
    parent = os.path.dirname(path)
    if parent:
        os.makedirs(parent, exist_ok=True)
    i = model.intrinsics
    cam0 = {"camera_model": model.get_model_name()}
    if isinstance(model, (camera.KannalaBrandtModel, camera.RadTanModel)):
        # the loaders read `distortion` (the KB saver's `distortion_coeffs`
        # key mismatch is a reference bug acknowledged in
        # tests/yaml_serialization.rs:35-36; we write the key the loader reads)
        cam0["intrinsics"] = [i.fx, i.fy, i.cx, i.cy]
        cam0["distortion"] = model.get_distortion()
    else:
        cam0["intrinsics"] = [i.fx, i.fy, i.cx, i.cy] + model.get_distortion()
    cam0["resolution"] = [int(model.resolution.width), int(model.resolution.height)]
    try:
        with open(path, "w") as f:
            yaml.safe_dump({"cam0": cam0}, f, default_flow_style=None, sort_keys=False)
    except OSError as e:
        raise camera.IOError_(str(e)) from None
