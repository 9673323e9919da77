"""Column-alignment sensitivity of the 2N x P column-major Jacobian stores:
column c starts at byte c * 16N, so unless 16N is a multiple of 128 B (the
cache line), a wave's 1 KiB column chunk straddles partial lines.  Times the
zero-compute mimic (tools/hbm_probe.hip) and the real KB k_project at
several N, plain and nt stores.

  python tools/diag_align.py
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    Pr = ctypes.CDLL(os.path.join(HERE, "build", "libhbmprobe.so"))
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    Pr.acm_probe_mimic.argtypes = [sz, vp, vp, vp, vp, ci, ci, ci, vp]
    sh = torch.cuda.current_stream().cuda_stream
    params, (w, h) = samples.SAMPLES[2]
    cam = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam), 2, (ctypes.c_double * 8)(*params), 8, w, h))
    nmax = 10_000_008
    pts = samples.synthetic_points_device(nmax)
    uv = torch.empty((nmax, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((nmax,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((8 * nmax * 2,), dtype=torch.float64, device="cuda")

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
    for rep in range(2):
        for n in (10_000_000, 10_000_001, 10_000_002, 10_000_004, 9_291_849):
            for nt in (0, 1):
                def mim():
                    Pr.acm_probe_mimic(n, pts.data_ptr(), uv.data_ptr(), st.data_ptr(),
                                       jac.data_ptr(), 8, nt, 0, sh)
                L.acm_set_tuning(_lib.TUNE_PROJECT_VARIANT, nt)

                def real(al):
                    def f():
                        L.acm_set_tuning(_lib.TUNE_ALIGN_J, al)
                        L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(),
                                      st.data_ptr(), jac.data_ptr(), sh)
                    return f
                for k, f in (("mimic", mim), ("kb", real(0)), ("kbaligned", real(1))):
                    key = f"{k}_n{n}_{'nt' if nt else 'plain'}"
                    ms = timed(f)
                    out[key] = min(out.get(key, 1e9), ms)
    L.acm_set_tuning(_lib.TUNE_PROJECT_VARIANT, -1)
    L.acm_set_tuning(_lib.TUNE_ALIGN_J, -1)
    cells = {k: {"ms": round(v, 4), "GBps": round(169 * int(k.split("_n")[1].split("_")[0]) / v / 1e6, 1),
                 "col_misalign_B": (16 * int(k.split("_n")[1].split("_")[0])) % 128}
             for k, v in out.items()}
    print(json.dumps({"what": "J column alignment", "cells": cells}))


if __name__ == "__main__":
    main()
