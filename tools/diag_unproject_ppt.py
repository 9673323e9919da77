"""acm_unproject pixels-per-lane / AoS ray-store A/B (ACM_TUNE_UNPROJECT_PPT:
1 and 2 pixels per lane with three 8-B stores per ray, 3 = 1 pixel per lane
with LDS-staged 16-B pieces, -1 = auto = 2 pixels per lane, staged),
interleaved in one process, every model, 10M pixels (the bench cloud's
projections), AoS and SoA rays.  Outputs must be bit-identical for every
setting.

  python tools/diag_unproject_ppt.py [--points N] [--reps R]
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
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    n = a.points
    sh = torch.cuda.current_stream().cuda_stream
    pts = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    rays = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = {}
    for mid in range(7):
        params, (w, h) = samples.SAMPLES[mid]
        P = len(params)
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * P)(*params), P,
                                     w, h))
        L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(), st.data_ptr(),
                      None, sh)
        px = torch.nan_to_num(uv, nan=1.0).contiguous()
        for layout in (0, 1):
            def unp():
                _lib.check(L.acm_unproject(ctypes.byref(cam), n, px.data_ptr(), rays.data_ptr(),
                                           layout, st.data_ptr(), sh))
            ref, times = {}, {1: [], 2: [], 3: [], -1: []}
            for k in times:
                L.acm_set_tuning(_lib.TUNE_UNPROJECT_PPT, k)
                unp()
                torch.cuda.synchronize()
                ref[k] = (rays.view(torch.int64).clone(), st.clone())
            for _ in range(a.reps):
                for k in times:
                    L.acm_set_tuning(_lib.TUNE_UNPROJECT_PPT, k)
                    unp()
                    e0.record()
                    for _ in range(5):
                        unp()
                    e1.record()
                    torch.cuda.synchronize()
                    times[k].append(e0.elapsed_time(e1) / 5)
            L.acm_set_tuning(_lib.TUNE_UNPROJECT_PPT, -1)
            same = all(torch.equal(ref[1][0], r[0]) and torch.equal(ref[1][1], r[1])
                       for r in ref.values())
            res = {"identical": same,
                   "ms": {f"ppt{k}": round(min(v), 4) for k, v in times.items()},
                   "TBps": {f"ppt{k}": round(n * 41 / min(v) / 1e9, 2) for k, v in times.items()}}
            key = f"{mid}/{'aos' if layout == 0 else 'soa'}"
            out[key] = res
            print(key, json.dumps(res), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
