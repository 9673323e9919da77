"""Interleaved A/B sweep of acm_project kernel variants in ONE process
(methodology rule: variants x rounds, report median/min; results must be
bit-identical across variants).

  python tools/sweep_project.py [--points 10000000] [--rounds 10] [--model kb]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))

MODELS = {"pinhole": 0, "radtan": 1, "kb": 2, "ds": 3, "ucm": 4, "eucm": 5, "fov": 6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--models", default="kb")
    ap.add_argument("--variants", default="0,1,2,3,4,5")
    ap.add_argument("--layouts", default="aos,soa")
    ap.add_argument("--jac", default="1")
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    n = a.points
    results = []
    for mname in a.models.split(","):
        mid = MODELS[mname]
        params, (w, h) = samples.SAMPLES[mid]
        P = len(params)
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * P)(*params), P,
                                     w, h))
        for lay in a.layouts.split(","):
            pts = samples.synthetic_points_device(n, layout=lay)
            layc = _lib.LAYOUT_SOA if lay == "soa" else _lib.LAYOUT_AOS
            for wj in [int(x) for x in a.jac.split(",")]:
                uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
                st = torch.empty((n,), dtype=torch.uint8, device="cuda")
                jac = torch.empty((P, n, 2), dtype=torch.float64, device="cuda") if wj else None
                sh = torch.cuda.current_stream().cuda_stream
                variants = [int(v) for v in a.variants.split(",")]
                times = {v: [] for v in variants}
                ref = None
                for r in range(a.rounds):
                    for v in variants:
                        L.acm_set_tuning(0, v)
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        _lib.check(L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), layc,
                                                 uv.data_ptr(), st.data_ptr(),
                                                 jac.data_ptr() if wj else None, sh))
                        e0.record()
                        for _ in range(a.reps):
                            L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), layc,
                                          uv.data_ptr(), st.data_ptr(),
                                          jac.data_ptr() if wj else None, sh)
                        e1.record()
                        torch.cuda.synchronize()
                        times[v].append(e0.elapsed_time(e1) / a.reps)
                        if r == 0:
                            sig = (uv.view(torch.int64).sum().item(), st.sum().item(),
                                   jac.view(torch.int64).sum().item() if wj else 0)
                            if ref is None:
                                ref = sig
                            assert sig == ref, f"variant {v} changed the results"
                L.acm_set_tuning(0, -1)
                bpp = 24 + 16 + 1 + (16 * P if wj else 0)
                for v in variants:
                    t = sorted(times[v])
                    med = t[len(t) // 2]
                    row = {"model": mname, "layout": lay, "jac": wj, "variant": v,
                           "median_ms": round(med, 5), "min_ms": round(t[0], 5),
                           "GBps": round(bpp * n / (med / 1e3) / 1e9, 1),
                           "Gpts": round(n / (med / 1e3) / 1e9, 3)}
                    results.append(row)
                    print(json.dumps(row), flush=True)
                del uv, st, jac
            del pts
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
