"""Store-policy diagnostic: DS project+J vs DS residual+J, plain vs
non-temporal stores, interleaved in one process on the same 10M points.

  python tools/diag_store.py [--points N] [--reps R]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--model", type=int, default=3)
    ap.add_argument("--sampled", action="store_true",
                    help="config-3 data: KB sample_points grid, DS params from linear_estimation")
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    mid = a.model
    params, (w, h) = samples.SAMPLES[mid]
    P = len(params)
    n = a.points
    cam = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * P)(*params), P, w, h))
    pts = samples.synthetic_points_device(n)
    obs_in = None
    if a.sampled:
        from apex_camera_models import KannalaBrandtModel, Resolution, conversion, util
        kp, (kw, kh) = samples.SAMPLES[2]
        src = KannalaBrandtModel._from_params(kp, Resolution(kw, kh))
        obs_in, pts = util.sample_points(src, n)
        n = pts.shape[0]
        model = conversion._init_target("double_sphere", src)
        model.linear_estimation(pts, obs_in)
        cam = model.acm_camera()
        mid, P = 3, 6
        pts, obs_in = pts.contiguous(), obs_in.contiguous()
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((P, n, 2), dtype=torch.float64, device="cuda")
    res = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    jac2 = torch.empty((P, n, 2), dtype=torch.float64, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(), st.data_ptr(),
                  jac.data_ptr(), sh)
    obs = (torch.nan_to_num(uv, nan=1.0) + 0.25).contiguous() if obs_in is None else obs_in
    valid = int((st == 0).sum())

    def proj():
        L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(), st.data_ptr(),
                      jac.data_ptr(), sh)

    def resid(with_status):
        def f():
            L.acm_residual_jacobian(ctypes.byref(cam), n, pts.data_ptr(), 0, obs.data_ptr(), 0,
                                    res.data_ptr(), jac2.data_ptr(),
                                    st.data_ptr() if with_status else None, sh)
        return f

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

    cells = {}
    for _ in range(a.reps):
        for al in (0, 1):
            L.acm_set_tuning(_lib.TUNE_ALIGN_J, al)
            for pv in (0, 1):
                L.acm_set_tuning(_lib.TUNE_PROJECT_VARIANT, pv)
                k = f"project_J_{'nt' if pv else 'plain'}{'_aligned' if al else ''}"
                cells.setdefault(k, []).append(timed(proj))
            L.acm_set_tuning(_lib.TUNE_PROJECT_VARIANT, -1)
            for rv in (0, 1):
                L.acm_set_tuning(_lib.TUNE_RESIDUAL_NT, rv)
                for ws in (False, True):
                    k = (f"residual_J_{'nt' if rv else 'plain'}{'_status' if ws else ''}"
                         f"{'_aligned' if al else ''}")
                    cells.setdefault(k, []).append(timed(resid(ws)))
            L.acm_set_tuning(_lib.TUNE_RESIDUAL_NT, 0)
        L.acm_set_tuning(_lib.TUNE_ALIGN_J, -1)
    bpp_p = 24 + 16 + 1 + 16 * P
    bpp_r = 40 + 16 + 16 * P
    out = {}
    for k, v in cells.items():
        ms = min(v)
        b = bpp_p if k.startswith("project") else bpp_r + (1 if "status" in k else 0)
        out[k] = {"ms": round(ms, 4), "GBps": round(b * n / ms / 1e6, 1)}
    print(json.dumps({"what": "store policy A/B", "model": mid, "points": n, "valid": valid,
                      "sampled": a.sampled, "cells": out}))


if __name__ == "__main__":
    main()
