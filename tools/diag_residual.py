"""Factor linearisation (row a5) beside the projection it is built on:
acm_residual_jacobian (40 B read, 16 B residual + 16P B J written per point)
and acm_project (24 B read, 16 B uv + 16P B J + 1 B status written) for DS
and KB, and the residual alone (k_residual: 40 B read, 16 B written), at an N that keeps every J column on the 128-B grid (10M) and at the
rows tool's KB-sampled count (9,291,849: columns 16-B-shifted, LDS path).
Every library in --libs is timed, alternating (HIP events, best of --rounds
blocks of --reps calls).

  python tools/diag_residual.py [--libs a.so,b.so]
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
    ap.add_argument("--libs", default="apex-camera-models_amd/lib/libacm.so")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples  # data generation only
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    libs = []
    for path in a.libs.split(","):
        L = ctypes.CDLL(os.path.join(ROOT, path) if not os.path.isabs(path) else path)
        L.acm_camera_init.argtypes = [vp, ci, vp, ci, ctypes.c_uint32, ctypes.c_uint32]
        L.acm_project.argtypes = [vp, sz, vp, ci, vp, vp, vp, vp]
        L.acm_residual_jacobian.argtypes = [vp, sz, vp, ci, vp, ci, vp, vp, vp, vp]
        libs.append((os.path.basename(path), L))
    sh = torch.cuda.current_stream().cuda_stream
    nmax = 10_000_000
    pts = samples.synthetic_points_device(nmax)
    uv = torch.empty((nmax, 2), dtype=torch.float64, device="cuda")
    obs = torch.empty((nmax, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((nmax,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((8 * nmax * 2,), dtype=torch.float64, device="cuda")

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    for mid in (3, 2):
        params, (w, h) = samples.SAMPLES[mid]
        P = len(params)
        cams = {}
        for tag, L in libs:
            c = _lib.AcmCamera()
            assert L.acm_camera_init(ctypes.byref(c), mid, (ctypes.c_double * P)(*params), P, w, h) == 0
            cams[tag] = c
        L0 = libs[0][1]
        L0.acm_project(ctypes.byref(cams[libs[0][0]]), nmax, pts.data_ptr(), 0, obs.data_ptr(),
                       None, None, sh)
        obs.add_(0.25)
        for n in (10_000_000, 9_291_849):
            calls = {}
            for tag, L in libs:
                c = cams[tag]
                calls[f"residual_noj_{tag}"] = (56, lambda L=L, c=c, n=n: L.acm_residual_jacobian(
                    ctypes.byref(c), n, pts.data_ptr(), 0, obs.data_ptr(), 0, uv.data_ptr(),
                    None, None, sh))
                calls[f"project_{tag}"] = (16 * P + 41, lambda L=L, c=c, n=n: L.acm_project(
                    ctypes.byref(c), n, pts.data_ptr(), 0, uv.data_ptr(), st.data_ptr(),
                    jac.data_ptr(), sh))
                calls[f"residual_{tag}"] = (16 * P + 56, lambda L=L, c=c, n=n: L.acm_residual_jacobian(
                    ctypes.byref(c), n, pts.data_ptr(), 0, obs.data_ptr(), 0, uv.data_ptr(),
                    jac.data_ptr(), None, sh))
                calls[f"residual_status_{tag}"] = (16 * P + 57, lambda L=L, c=c, n=n: L.acm_residual_jacobian(
                    ctypes.byref(c), n, pts.data_ptr(), 0, obs.data_ptr(), 0, uv.data_ptr(),
                    jac.data_ptr(), st.data_ptr(), sh))
            best = {}
            items = list(calls.items())
            for rnd in range(a.rounds):
                for k, (_, fn) in (items if rnd % 2 == 0 else items[::-1]):
                    best[k] = min(best.get(k, 1e9), timed(fn))
            torch.cuda.synchronize()
            print(json.dumps({"model": mid, "n": n,
                              "ms": {k: round(v, 4) for k, v in best.items()},
                              "TBps": {k: round(calls[k][0] * n / v / 1e9, 2) for k, v in best.items()}}),
                  flush=True)


if __name__ == "__main__":
    main()
