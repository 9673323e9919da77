"""KB sample_points at 1e8 cells with both outputs carved from ONE
allocation, the ray buffer placed `delta` bytes after the end of the pixel
buffer, for a set of deltas (tools/diag_sample_state.py found the call 0.70
vs 0.84 ms depending only on where the allocator put the outputs).  Timed
as tools/bench_rows.py times its a17 row."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))


def main():
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, samples
    L = _lib.load()
    sh = torch.cuda.current_stream().cuda_stream
    kp, (kw, kh) = samples.SAMPLES[2]
    cam = KannalaBrandtModel._from_params(kp, Resolution(kw, kh)).acm_camera()
    cells = 100_000_000
    gx, gy = ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(L.acm_sample_points_grid(cam.width, cam.height, cells, ctypes.byref(gx),
                                        ctypes.byref(gy)))
    cap = gx.value * gy.value
    cnt = torch.zeros((2,), dtype=torch.int64, device="cuda")
    wsb = L.acm_sample_points_workspace_size(ctypes.byref(cam), cells)
    sws = torch.empty(((wsb + 7) // 8,), dtype=torch.float64, device="cuda")
    MB = 1 << 20
    deltas = [int(x) for x in os.environ.get(
        "DELTAS", "0,256,4096,65536,1048576,2097152,2101248,4194304,8388608,33554432").split(",")]
    big = torch.empty((cap * 5 + (max(deltas) + 64 * MB) // 8,), dtype=torch.float64,
                      device="cuda")
    base = big.data_ptr()

    def gpu_ms(fn, reps=5, blocks=3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        k = 0
        while k < 3 or time.perf_counter() - t0 < 0.05:
            fn()
            torch.cuda.synchronize()
            k += 1
        best = float("inf")
        for _ in range(blocks):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / reps)
        return best

    out = {}
    for rep in range(2):
        for d in deltas:
            uvp = base
            xyzp = base + cap * 16 + d

            def sp():
                _lib.check(L.acm_sample_points(ctypes.byref(cam), cells, uvp, xyzp,
                                               cnt.data_ptr(), sws.data_ptr(), wsb, sh))
            ms = gpu_ms(sp)
            out.setdefault(str(d), []).append(round(ms, 4))
    print(json.dumps({"what": "KB sample_points ms by ray-buffer placement (bytes after the "
                      "pixel buffer), two rounds", "uv_base_mod_2MB": base % (2 * MB),
                      "by_delta": out}), flush=True)


if __name__ == "__main__":
    main()
