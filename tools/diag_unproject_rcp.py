"""Unprojection A/B for ACM_TUNE_UNPROJECT_RCP: (u - cx) / fx, (v - cy) / fy
as two IEEE divisions (0) or through the host's RN(1 / fx), RN(1 / fy) plus
one FMA correction (1, div_by_f in camera_models.hpp).  Every model:
acm_unproject over 10M pixels (the projections of the bench cloud) and
sample_points on the config-5 grid (1e8 requested cells), interleaved in one
process.  The outputs of both settings must be bit-identical.

  python tools/diag_unproject_rcp.py [--cells N]
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
    ap.add_argument("--cells", type=int, default=100_000_000)
    ap.add_argument("--points", type=int, default=10_000_000)
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples, util
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    names = ["pinhole", "rad_tan", "kannala_brandt", "double_sphere", "ucm", "eucm", "fov"]
    L = _lib.load()
    n = a.points
    pts = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    rays = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream

    def timed(fn, reps):
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
        m = MODEL_CLASSES[names[mid]]._from_params([float(p) for p in params], Resolution(w, h))

        def unp():
            L.acm_unproject(ctypes.byref(cam), n, uvin.data_ptr(), rays.data_ptr(), 0,
                            st.data_ptr(), sh)

        same = True
        ref = None
        for v in (0, 1):
            L.acm_set_tuning(_lib.TUNE_UNPROJECT_RCP, v)
            unp()
            s = util.sample_points(m, a.cells)
            got = (rays.view(torch.int64).clone(), st.clone(), s[0].clone(), s[1].clone())
            if ref is None:
                ref = got
            else:
                same = same and all(torch.equal(x, y) for x, y in zip(ref, got))
            del s
        del ref, got
        cells = {}
        for _ in range(3):
            for v in (0, 1):
                L.acm_set_tuning(_lib.TUNE_UNPROJECT_RCP, v)
                k = f"unproject_rcp{v}"
                cells[k] = min(cells.get(k, 1e9), timed(unp, 20))
                k = f"sample_rcp{v}"
                cells[k] = min(cells.get(k, 1e9), timed(lambda: util.sample_points(m, a.cells), 3))
        L.acm_set_tuning(_lib.TUNE_UNPROJECT_RCP, -1)
        out[mid] = {"identical": same,
                    **{k: {"ms": round(t, 4),
                           **({"GBps": round(41 * n / t / 1e6, 1)} if k.startswith("unp") else {})}
                       for k, t in cells.items()}}
        print(json.dumps({"model": names[mid], **out[mid]}), flush=True)
    print(json.dumps({"what": "unproject rcp A/B", "points": n, "cells": a.cells,
                      "models": out}))


if __name__ == "__main__":
    main()
