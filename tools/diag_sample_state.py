"""KB sample_points at 1e8 cells timed the way tools/bench_rows.py times its
a17 row (>= 50 ms of synchronised warm-up calls, then the fastest of three
blocks of five calls), in three process states: fresh; after the rows
tool's projection-row buffers (10M points, a 9-column Jacobian) were
allocated, used and freed; and with them still held.  Looks for the cause
of the rows tool's slower a17 figure (profiles/r04z3_kb_sample_points_harness.log)."""
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
    src = KannalaBrandtModel._from_params(kp, Resolution(kw, kh))
    cells = 100_000_000
    cam = src.acm_camera()

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

    def a17():
        gx, gy = ctypes.c_uint32(), ctypes.c_uint32()
        _lib.check(L.acm_sample_points_grid(cam.width, cam.height, cells, ctypes.byref(gx),
                                            ctypes.byref(gy)))
        cap = gx.value * gy.value
        su2 = torch.empty((cap, 2), dtype=torch.float64, device="cuda")
        sx3 = torch.empty((cap, 3), dtype=torch.float64, device="cuda")
        cnt = torch.zeros((2,), dtype=torch.int64, device="cuda")
        wsb = L.acm_sample_points_workspace_size(ctypes.byref(cam), cells)
        sws = torch.empty(((wsb + 7) // 8,), dtype=torch.float64, device="cuda")

        def sp():
            _lib.check(L.acm_sample_points(ctypes.byref(cam), cells, su2.data_ptr(),
                                           sx3.data_ptr(), cnt.data_ptr(), sws.data_ptr(), wsb,
                                           sh))
        ms = gpu_ms(sp)
        del su2, sx3, sws
        return round(ms, 4)

    mode = os.environ.get("MODE", "")
    if mode == "dummy":  # a 2 GB block allocated first and held
        hold = torch.empty((2 << 30) // 8, dtype=torch.float64, device="cuda")  # noqa: F841
    out = {"fresh": a17()}
    n = 10_000_000
    pts = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((9 * n * 2,), dtype=torch.float64, device="cuda")
    _lib.check(L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(),
                             st.data_ptr(), jac.data_ptr(), sh))
    torch.cuda.synchronize()
    out["others_held"] = a17()
    del pts, uv, st, jac
    out["others_freed"] = a17()
    torch.cuda.empty_cache()
    out["cache_emptied"] = a17()
    out["again"] = a17()
    print(json.dumps({"what": "KB sample_points a17 timing by process state (ms)", **out}),
          flush=True)


if __name__ == "__main__":
    main()
