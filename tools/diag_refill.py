"""RadTan acm_unproject A/B in one process: several builds of libacm.so
(e.g. lib/libacm_refill1.so, the ACM_DIAG_REFILL lane-refill kernel) timed
interleaved on the same pixels (the bench cloud projected with the RadTan
sample camera, as tools/bench_rows.py row a14), outputs compared bit for bit
with the first library.

  python tools/diag_refill.py lib/libacm.so lib/libacm_refill1.so ...
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))


def main():
    import torch
    from apex_camera_models import _lib, samples
    libs = []
    for p in sys.argv[1:]:
        L = ctypes.CDLL(os.path.join(ROOT, "apex-camera-models_amd", p))
        L.acm_unproject.argtypes = [ctypes.POINTER(_lib.AcmCamera), ctypes.c_size_t,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.acm_unproject.restype = ctypes.c_int
        L.acm_project.argtypes = [ctypes.POINTER(_lib.AcmCamera), ctypes.c_size_t,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        libs.append((p, L))
    n = int(os.environ.get("POINTS", "10000000"))
    params, (w, h) = samples.SAMPLES[1]
    cam = _lib.AcmCamera()
    P = len(params)
    _lib.check(_lib.load().acm_camera_init(ctypes.byref(cam), 1, (ctypes.c_double * P)(*params),
                                           P, w, h))
    pts = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    assert libs[0][1].acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(),
                                  st.data_ptr(), None, sh) == 0
    uv = torch.nan_to_num(uv, nan=1.0).contiguous()
    outs = {}
    for p, L in libs:
        rays = torch.full((n, 3), 7.0, dtype=torch.float64, device="cuda")
        s = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
        assert L.acm_unproject(ctypes.byref(cam), n, uv.data_ptr(), rays.data_ptr(), 0,
                               s.data_ptr(), sh) == 0
        torch.cuda.synchronize()
        outs[p] = (rays, s)
    r0, s0 = outs[libs[0][0]]
    res = {}
    for p, _ in libs:
        r, s = outs[p]
        res[p] = {"identical": bool(torch.equal(s, s0) and torch.equal(
            torch.nan_to_num(r, nan=123.0).view(torch.int64),
            torch.nan_to_num(r0, nan=123.0).view(torch.int64))), "ms": []}
    rays = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    s = torch.empty((n,), dtype=torch.uint8, device="cuda")
    for _ in range(5):
        for p, L in libs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                L.acm_unproject(ctypes.byref(cam), n, uv.data_ptr(), rays.data_ptr(), 0,
                                s.data_ptr(), sh)
            e1.record()
            torch.cuda.synchronize()
            res[p]["ms"].append(e0.elapsed_time(e1) / 10)
    for p in res:
        m = sorted(res[p]["ms"])
        res[p] = {"identical": res[p]["identical"], "ms_median": round(m[len(m) // 2], 4),
                  "GBps": round(41 * n / (m[len(m) // 2] * 1e-3) / 1e9, 1)}
    print(json.dumps({"what": "RadTan unproject A/B", "points": n, "libs": res}))


if __name__ == "__main__":
    main()
