"""Why is DS project+J slower on config-3 (KB-sampled) data than on the
synthetic cloud?  Matrix: points (synthetic / sampled) x DS params (sample
yaml / linear-estimation) x buffer (as returned / fresh clone), nt stores.

  python tools/diag_data.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from apex_camera_models import (KannalaBrandtModel, Resolution, _lib, conversion, samples,
                                    util)
    L = _lib.load()
    kp, (kw, kh) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(kw, kh))
    obs_s, pts_s = util.sample_points(src, 10_000_000)
    n = pts_s.shape[0]
    model = conversion._init_target("double_sphere", src)
    model.linear_estimation(pts_s, obs_s)
    cam_le = model.acm_camera()
    dsp, (w, h) = samples.SAMPLES[3]
    cam_y = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam_y), 3, (ctypes.c_double * 6)(*dsp), 6, w, h))
    pts_y = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((6, n, 2), dtype=torch.float64, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    L.acm_set_tuning(_lib.TUNE_PROJECT_VARIANT, 1)

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    bufs = {"synthetic": pts_y, "sampled": pts_s, "sampled_clone": pts_s.clone(),
            "sampled_shuffled": pts_s[torch.randperm(n, device="cuda")].contiguous(),
            "sampled_plus_synth_z": torch.stack([pts_s[:, 0], pts_s[:, 1], pts_y[:, 2]], 1)
            .contiguous()}
    cams = {"yaml": cam_y, "linest": cam_le}
    out = {}
    for rep in range(3):
        for bn, b in bufs.items():
            for cn, c in cams.items():
                def f():
                    L.acm_project(ctypes.byref(c), n, b.data_ptr(), 0, uv.data_ptr(),
                                  st.data_ptr(), jac.data_ptr(), sh)
                ms = timed(f)
                k = f"{bn}/{cn}"
                out[k] = min(out.get(k, 1e9), ms)
                if rep == 0:
                    out[k + "/valid"] = int((st == 0).sum())
    L.acm_set_tuning(_lib.TUNE_PROJECT_VARIANT, -1)
    print(json.dumps({"what": "DS project+J nt, data matrix", "points": n,
                      "params_linest": list(cam_le.params)[:6], "cells": out}))


if __name__ == "__main__":
    main()
