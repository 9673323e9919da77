"""Non-temporal-load A/B for the read-heavy maps: project without J
(24 B read / 17 B written per point) and unproject (16 / 25), every model,
10M points, interleaved in one process.

  python tools/diag_ntl.py
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
    from apex_camera_models import _lib, samples
    L = _lib.load()
    n = 10_000_000
    pts = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    rays = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream

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

    out = {}
    for mid in range(7):
        params, (w, h) = samples.SAMPLES[mid]
        P = len(params)
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * P)(*params), P,
                                     w, h))
        L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(), st.data_ptr(),
                      None, sh)
        uvin = torch.nan_to_num(uv, nan=1.0).contiguous()
        cells = {}
        for _ in range(3):
            for var in (1, 5):  # nt stores, + nt loads
                L.acm_set_tuning(_lib.TUNE_PROJECT_VARIANT, var)
                k = f"project_v{var}"
                cells[k] = min(cells.get(k, 1e9), timed(lambda: L.acm_project(
                    ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(), st.data_ptr(), None,
                    sh)))
            L.acm_set_tuning(_lib.TUNE_PROJECT_VARIANT, -1)
            for ntl in (0, 1):
                L.acm_set_tuning(_lib.TUNE_NT_LOADS_UNPROJECT, ntl)
                k = f"unproject_ntl{ntl}"
                cells[k] = min(cells.get(k, 1e9), timed(lambda: L.acm_unproject(
                    ctypes.byref(cam), n, uvin.data_ptr(), rays.data_ptr(), 0, st.data_ptr(),
                    sh)))
            L.acm_set_tuning(_lib.TUNE_NT_LOADS_UNPROJECT, -1)
        out[mid] = {k: {"ms": round(v, 4),
                        "GBps": round((41 if k.startswith("project") else 41) * n / v / 1e6, 1)}
                    for k, v in cells.items()}
    print(json.dumps({"what": "nt-load A/B (project no J, unproject)", "points": n,
                      "cells": out}))


if __name__ == "__main__":
    main()
