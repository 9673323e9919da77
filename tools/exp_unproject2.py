"""KB unprojection: one pixel per lane (the production form) vs two pixels
per lane with merged Newton loops (tools/exp_unproject2.hip), 10M pixels of
the bench cloud projected with the KB sample camera; outputs compared bit
for bit, kernels timed interleaved with HIP events.

  make -C tools build/libexp_u2.so && python tools/exp_unproject2.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))


class ExpCam(ctypes.Structure):
    _fields_ = [("p", ctypes.c_double * 9), ("width", ctypes.c_uint32),
                ("height", ctypes.c_uint32), ("ifx", ctypes.c_double), ("ify", ctypes.c_double)]


def main():
    import torch
    from apex_camera_models import KannalaBrandtModel, samples
    E = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libexp_u2.so"))
    E.exp_unproject.argtypes = [ctypes.c_int, ctypes.POINTER(ExpCam), ctypes.c_size_t,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    E.exp_unproject.restype = ctypes.c_int
    n = int(os.environ.get("POINTS", "10000000"))
    params, (w, h) = samples.SAMPLES[2]
    m = KannalaBrandtModel.new(params)
    m.resolution.width, m.resolution.height = w, h
    pts = samples.synthetic_points_device(n)
    uv, _, _ = m.project_batch(pts)
    uv = torch.nan_to_num(uv, nan=1.0).contiguous()
    cam = ExpCam()
    for i, v in enumerate(params):
        cam.p[i] = v
    cam.width, cam.height = w, h
    cam.ifx, cam.ify = 1.0 / params[0], 1.0 / params[1]
    sh = torch.cuda.current_stream().cuda_stream
    out = {}
    for var in (1, 2):
        rays = torch.full((n, 3), 5.0, dtype=torch.float64, device="cuda")
        st = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
        assert E.exp_unproject(var, ctypes.byref(cam), n, uv.data_ptr(), rays.data_ptr(),
                               st.data_ptr(), sh) == 0
        torch.cuda.synchronize()
        out[var] = (rays, st)
    same = torch.equal(out[1][1], out[2][1]) and torch.equal(
        torch.nan_to_num(out[1][0], nan=9.0).view(torch.int64),
        torch.nan_to_num(out[2][0], nan=9.0).view(torch.int64))
    rays, st = out[1]
    ms = {1: [], 2: []}
    for _ in range(5):
        for var in (1, 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                E.exp_unproject(var, ctypes.byref(cam), n, uv.data_ptr(), rays.data_ptr(),
                                st.data_ptr(), sh)
            e1.record()
            torch.cuda.synchronize()
            ms[var].append(e0.elapsed_time(e1) / 10)
    med = {v: sorted(x)[len(x) // 2] for v, x in ms.items()}
    print(json.dumps({"what": "KB unproject, 1 vs 2 pixels per lane (merged Newton)",
                      "points": n, "identical": bool(same),
                      "one_per_lane_ms": round(med[1], 4), "two_per_lane_ms": round(med[2], 4),
                      "valid": int((out[1][1] == 0).sum())}))


if __name__ == "__main__":
    main()
