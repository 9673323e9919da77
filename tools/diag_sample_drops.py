"""sample_points paths on RadTan cameras that drop cells: auto (-1, the
speculative segment path for RadTan), the speculative path itself (4) and
the single pass (2) at 1e8 requested cells, C-ABI calls on preallocated
buffers, fastest of three blocks; the outputs must be identical.  (A host
probe that sent cameras with drops in their first rows to the single pass
was measured here and dropped: the speculative path won even then.)

  python tools/diag_sample_drops.py [--cells N]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)

CAMS = {
    "sample": None,  # samples.SAMPLES[1]
    "fold_corners": [200.0, 200.0, 376.0, 240.0, -0.45, 0.12, 0.003, -0.002, -0.005],
    "fold_wide": [300.0, 300.0, 370.0, 250.0, -0.6, 0.1, 0.001, 0.002, 0.0],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=100_000_000)
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    L = _lib.load()
    sh = torch.cuda.current_stream().cuda_stream
    for name, params in CAMS.items():
        p0, (w, h) = samples.SAMPLES[1]
        params = list(p0) if params is None else params
        m = MODEL_CLASSES["rad_tan"]._from_params([float(x) for x in params], Resolution(w, h))
        cam = m.acm_camera()
        ncx, ncy = ctypes.c_uint32(), ctypes.c_uint32()
        L.acm_sample_points_grid(cam.width, cam.height, a.cells, ctypes.byref(ncx),
                                 ctypes.byref(ncy))
        cap = ncx.value * ncy.value
        uv = torch.empty((cap, 2), dtype=torch.float64, device="cuda")
        xyz = torch.empty((cap, 3), dtype=torch.float64, device="cuda")
        cnt = torch.zeros((2,), dtype=torch.int64, device="cuda")
        wsb = L.acm_sample_points_workspace_size(ctypes.byref(cam), a.cells)
        ws = torch.empty(((wsb + 7) // 8,), dtype=torch.float64, device="cuda")

        def call(mode):
            L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, mode)
            _lib.check(L.acm_sample_points(ctypes.byref(cam), a.cells, uv.data_ptr(),
                                           xyz.data_ptr(), cnt.data_ptr(), ws.data_ptr(), wsb, sh))
        ref = None
        res = {}
        for mode in (-1, 4, 2):
            call(mode)
            torch.cuda.synchronize()
            k = int(cnt[0].item())
            out = (uv[:k].clone(), xyz[:k].clone())
            if ref is None:
                ref = out
            same = torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
            best = 1e9
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    call(mode)
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 3)
            res[str(mode)] = {"ms": round(best, 4), "identical": same}
            del out
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, -1)
        print(json.dumps({"camera": name, "cells": cap, "kept": int(ref[0].shape[0]), **res}),
              flush=True)
        del uv, xyz, ws, ref


if __name__ == "__main__":
    main()
