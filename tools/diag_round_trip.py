"""Config-4 round trip (acm_project_unproject) A/B over ACM_TUNE_ROUND_TRIP
settings (points per lane, LDS-staged or direct ray stores): every model at
the bench leg's 50M points on one GPU, settings interleaved, HIP-event time
per call (best of --rounds blocks of --reps calls).

  python tools/diag_round_trip.py [--points N] [--settings -1,2,10,18,4,12,20]
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
    ap.add_argument("--points", type=int, default=50_000_000)
    ap.add_argument("--settings", default="-1,1,2,4,9,10,12,17,18,20")
    ap.add_argument("--models", default="0,1,2,3,4,5")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
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
    st2 = torch.empty((n,), dtype=torch.uint8, device="cuda")
    settings = [int(v) for v in a.settings.split(",")]
    for mid in (int(m) for m in a.models.split(",")):
        params, (w, h) = samples.SAMPLES[mid]
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * len(params))(
            *params), len(params), w, h))

        def call():
            _lib.check(L.acm_project_unproject(ctypes.byref(cam), n, pts.data_ptr(), 0,
                                               uv.data_ptr(), st.data_ptr(), rays.data_ptr(),
                                               st2.data_ptr(), sh))
        best = {}
        for _ in range(a.rounds):
            for v in settings:
                L.acm_set_tuning(_lib.TUNE_ROUND_TRIP, v)
                for _ in range(3):
                    call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                best[v] = min(best.get(v, 1e9), ms)
        L.acm_set_tuning(_lib.TUNE_ROUND_TRIP, -1)
        print(json.dumps({"model": mid, "points": n,
                          "ms": {str(k): round(v, 4) for k, v in best.items()},
                          "TBps_66B": {str(k): round(66 * n / v / 1e9, 2) for k, v in best.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
