import ctypes, sys, os
sys.path.insert(0, "apex-camera-models_amd"); sys.path.insert(0, ".")
import torch
from apex_camera_models import _lib, samples, util
from apex_camera_models.camera import MODEL_CLASSES, Resolution
L = _lib.load()
names = ["pinhole", "rad_tan", "kannala_brandt", "double_sphere", "ucm", "eucm", "fov"]
for mid in (3, 2, 0):
    params, (w, h) = samples.SAMPLES[mid]
    m = MODEL_CLASSES[names[mid]]._from_params([float(p) for p in params], Resolution(w, h))
    for fused in (0, 2):
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, fused)
        for _ in range(4):
            r = util.sample_points(m, 100_000_000)
            torch.cuda.synchronize()
            del r
L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, -1)
print("ok")
