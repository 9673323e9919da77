"""sample_points A/B of every path (ACM_TUNE_SAMPLE_FUSED): the segment
two-pass default ("seg"; "seg_nocert" = ACM_TUNE_SAMPLE_CERT 0, every
segment counted cell by cell; "seg_w1".."seg_w4" = ACM_TUNE_SAMPLE_WRITE),
the round-1 two-pass count / scan / write path ("two_pass") and the single
pass with a decoupled look-back ("fused_r2" / "_r4" / "_r8"), the
speculative segment path ("spec": write in place, repair after a drop), every
model on the config-5 grid (1e8 requested cells), interleaved in one
process.  The outputs must be bit-identical.

  python tools/diag_sample.py [--cells N]
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
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples, util
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    names = ["pinhole", "rad_tan", "kannala_brandt", "double_sphere", "ucm", "eucm", "fov"]
    L = _lib.load()
    out = {}
    for mid in [int(x) for x in os.environ.get("MODELS", "0,1,2,3,4,5,6").split(",")]:
        params, (w, h) = samples.SAMPLES[mid]
        m = MODEL_CLASSES[names[mid]]._from_params([float(p) for p in params], Resolution(w, h))

        # variant names: seg (default), seg_nocert, seg_w1..seg_w4
        # (ACM_TUNE_SAMPLE_WRITE), two_pass, fused_r2 / r4 / r8
        def run_knobs(v):
            fused = {"two_pass": 0, "fused_r2": 1, "fused_r4": 2, "fused_r8": 3,
                     "spec": 4}.get(v, -1)
            L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, fused)
            L.acm_set_tuning(_lib.TUNE_SAMPLE_CERT, 0 if v == "seg_nocert" else -1)
            L.acm_set_tuning(_lib.TUNE_SAMPLE_WRITE, int(v[-1]) if v.startswith("seg_w") else -1)

        def run(v):
            run_knobs(v)
            return util.sample_points(m, a.cells)

        VS = os.environ.get("VARIANTS", "seg,seg_nocert,two_pass,fused_r4").split(",")
        res = {v: run(v) for v in VS}
        same = all(torch.equal(res[VS[0]][k], res[v][k]) for k in (0, 1) for v in VS)
        kept = int(res[VS[0]][0].shape[0])
        del res
        # timing: the C-ABI call on preallocated buffers (no per-call 4 GB
        # allocation, no host read-back of the count between launches)
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
        sh = torch.cuda.current_stream().cuda_stream

        def call(v):
            run_knobs(v)
            _lib.check(L.acm_sample_points(ctypes.byref(cam), a.cells, uv.data_ptr(),
                                           xyz.data_ptr(), cnt.data_ptr(), ws.data_ptr(), wsb,
                                           sh))
        cells = {}
        for _ in range(int(os.environ.get("REPS", "3"))):
            for v in VS:
                call(v)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    call(v)
                e1.record()
                torch.cuda.synchronize()
                cells[v] = min(cells.get(v, 1e9), e0.elapsed_time(e1) / 3)
        del uv, xyz, ws
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, -1)
        L.acm_set_tuning(_lib.TUNE_SAMPLE_CERT, -1)
        L.acm_set_tuning(_lib.TUNE_SAMPLE_WRITE, -1)
        out[mid] = {"kept": kept, "identical": same,
                    **{k: {"ms": round(v, 4), "Gcells_s": round(a.cells / v / 1e6, 1),
                           "out_TBps": round(40 * kept / v / 1e9, 2)}
                       for k, v in cells.items()}}
        print(json.dumps({"model": mid, **out[mid]}), flush=True)
    print(json.dumps({"what": "sample_points paths", "cells": a.cells,
                      "models": out}))


if __name__ == "__main__":
    main()
