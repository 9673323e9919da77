"""FOV grid-search kernels A/B on KB-sampled correspondences (the a18' row's
workload): acm_fov_grid_errors timed per ACM_TUNE_FOV_UNROLL value (HIP
events, >= 50 ms warm-up, fastest of 3 blocks), with every form's counts
checked equal to the record form's and its sums within 1e-12.

  python tools/diag_fov.py [--points N] [--forms -1,0,1]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--forms", default="0,-1")
    a = ap.parse_args()
    import numpy as np
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, conversion, samples, util
    L = _lib.load()
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz = util.sample_points(src, a.points)
    n = xyz.shape[0]
    fov = conversion._init_target("fov", src)
    cam = fov.acm_camera()
    wsb = L.acm_fov_grid_workspace_size(n)
    ws = torch.empty(((wsb + 7) // 8,), dtype=torch.float64, device="cuda")
    out = torch.empty((2 * _lib.FOV_GRID_SIZE,), dtype=torch.float64, device="cuda")

    def call():
        _lib.check(L.acm_fov_grid_errors(ctypes.byref(cam), n, xyz.data_ptr(), _lib.LAYOUT_AOS,
                                         uv.data_ptr(), out.data_ptr(), ws.data_ptr(), wsb, None))

    def gpu_ms(reps=5, blocks=3):
        torch.cuda.synchronize()
        t0, k = time.perf_counter(), 0
        while k < 3 or time.perf_counter() - t0 < 0.05:
            call()
            torch.cuda.synchronize()
            k += 1
        best = float("inf")
        for _ in range(blocks):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / reps)
        return best

    forms = [int(v) for v in a.forms.split(",")]
    res, ms = {}, {}
    try:
        for rep in range(2):  # interleaved
            for f in forms:
                L.acm_set_tuning(_lib.TUNE_FOV_UNROLL, f)
                t = gpu_ms()
                ms[f] = min(ms.get(f, t), t)
                res[f] = out.cpu().numpy().copy()
    finally:
        L.acm_set_tuning(_lib.TUNE_FOV_UNROLL, -1)
    G = _lib.FOV_GRID_SIZE
    ref = res[forms[0]]
    for f in forms:
        s, c = res[f][:G], res[f][G:]
        rel = float(np.max(np.abs(s - ref[:G]) / np.abs(ref[:G])))
        avg = s / np.maximum(c, 1)
        print(json.dumps({"form": f, "points": n, "ms": round(ms[f], 4),
                          "G_evals_per_s": round(G * n / ms[f] / 1e6, 1),
                          "counts_equal": bool(np.array_equal(c, ref[G:])),
                          "max_rel_sum_diff": rel, "best_w": (int(np.argmin(avg)) + 10) / 100}),
              flush=True)


if __name__ == "__main__":
    main()
