"""Every SURVEY.md §8(a) row on the GPU (libacm.so kernels, HIP events) next
to the reference's CPU path (the oracle: the C restatement of the per-point
Rust loop, 1 thread) on a bounded sample of the same workload.  One JSON line
per row, then a markdown table on stderr.

  python tools/bench_rows.py [--points N] [--cpu-points M]

GPU: 10M points (maps, residual, normal equations, statistics), the 1e8-cell
KB grid (sample_points), 9.3M KB-sampled correspondences (linear estimation,
FOV grid).  CPU: the oracle on --cpu-points points (FOV grid: 1/10 of that),
rate = points / wall time.  Both in Mpoints/s of the row's own unit.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

NAMES = {0: "Pinhole", 1: "RadTan", 2: "KB", 3: "DS", 4: "UCM", 5: "EUCM", 6: "FOV"}
ROW_PROJ = {0: "a11", 1: "a13", 2: "a1", 3: "a4", 4: "a7", 5: "a9", 6: "f3"}
ROW_UNPROJ = {0: "a12", 1: "a14", 2: "a3", 3: "a6", 4: "a8", 5: "a10", 6: "f3"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--cpu-points", type=int, default=400_000)
    a = ap.parse_args()
    import torch

    import oracle as O
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, conversion, factors
    from apex_camera_models import samples, util
    L = _lib.load()
    sh = torch.cuda.current_stream().cuda_stream
    n, m = a.points, a.cpu_points
    rows = []

    def gpu_ms(fn, reps=10, blocks=3):
        # warm for >= 50 ms of GPU work first: each row follows seconds of
        # CPU-only oracle timing, and the GPU's clocks ramp back up over
        # milliseconds (r03: a 2-call warm-up timed KB sample_points at 1.02
        # ms against 0.80 ms in the kernel trace); then the fastest of
        # `blocks` blocks of `reps` back-to-back calls (steady state)
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

    def cpu_s(fn, min_s=0.5):
        fn()  # warm (page in, first-touch)
        t_all, k = 0.0, 0
        while t_all < min_s or k < 2:
            t0 = time.perf_counter()
            fn()
            t_all += time.perf_counter() - t0
            k += 1
        return t_all / k

    def emit(row, what, gpu_points, g_ms, bytes_pp, cpu_points, c_s):
        d = {"row": row, "what": what, "gpu_points": gpu_points, "gpu_ms": round(g_ms, 4),
             "gpu_Mpts_s": round(gpu_points / g_ms / 1e3, 1),
             "gpu_GBps": round(bytes_pp * gpu_points / g_ms / 1e6, 1) if bytes_pp else None,
             "cpu_points": cpu_points, "cpu_Mpts_s": round(cpu_points / c_s / 1e6, 2),
             "cpu_threads": 1}
        d["gpu_over_cpu"] = round(d["gpu_Mpts_s"] / d["cpu_Mpts_s"], 1)
        rows.append(d)
        print(json.dumps(d), flush=True)

    pts = samples.synthetic_points_device(n)
    pts_cpu = samples.synthetic_points(m)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((9 * n * 2,), dtype=torch.float64, device="cuda")
    rays = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    for mid in range(7):
        params, (w, h) = samples.SAMPLES[mid]
        P = len(params)
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * P)(*params), P,
                                     w, h))
        g = gpu_ms(lambda: L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(),
                                         st.data_ptr(), jac.data_ptr(), sh))
        c = cpu_s(lambda: O.project(mid, params, w, h, pts_cpu, want_jac=True))
        emit(ROW_PROJ[mid] + ("/a2" if mid == 2 else "/a15"), f"{NAMES[mid]} project + 2x{P} J",
             n, g, 41 + 16 * P, m, c)
        uvin = torch.nan_to_num(uv, nan=1.0).contiguous()
        uv_cpu = np.nan_to_num(O.project(mid, params, w, h, pts_cpu)[0], nan=1.0)
        g = gpu_ms(lambda: L.acm_unproject(ctypes.byref(cam), n, uvin.data_ptr(),
                                           rays.data_ptr(), 0, st.data_ptr(), sh))
        c = cpu_s(lambda: O.unproject(mid, params, w, h, uv_cpu))
        emit(ROW_UNPROJ[mid], f"{NAMES[mid]} unproject", n, g, 41, m, c)

    # DS residual + J and fused normal equations (a5) on KB-sampled data
    kp, (kw, kh) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(kw, kh))
    suv, sxyz = util.sample_points(src, n)
    ns = sxyz.shape[0]
    ds = conversion._init_target("double_sphere", src)
    ds.linear_estimation(sxyz, suv)
    dsp = ds.params()
    sel = np.random.default_rng(1).choice(ns, size=min(m, ns), replace=False)
    sxyz_c, suv_c = sxyz[sel].cpu().numpy(), suv[sel].cpu().numpy()
    dcam = ds.acm_camera()
    res = torch.empty((ns, 2), dtype=torch.float64, device="cuda")
    g = gpu_ms(lambda: L.acm_residual_jacobian(ctypes.byref(dcam), ns, sxyz.data_ptr(), 0,
                                               suv.data_ptr(), 0, res.data_ptr(), jac.data_ptr(),
                                               None, sh))
    c = cpu_s(lambda: O.residual_jacobian(3, dsp, kw, kh, sxyz_c, suv_c))
    emit("a5", "DS residual + 2Nx6 J (factor linearisation)", ns, g, 152, len(sel), c)
    f = factors.DoubleSphereCameraParamsFactor(sxyz, suv, Resolution(kw, kh))
    out = torch.empty((44,), dtype=torch.float64, device="cuda")
    g = gpu_ms(lambda: f.normal_equations(dsp, out))
    c = cpu_s(lambda: O.normal_equations(3, dsp, kw, kh, sxyz_c, suv_c))
    emit("a5", "DS fused normal equations (JtJ, Jtr, cost)", ns, g, 40, len(sel), c)

    # reprojection error with median (a16)
    errs = torch.empty((ns,), dtype=torch.float64, device="cuda")
    g = gpu_ms(lambda: util.compute_reprojection_error(ds, sxyz, suv))
    c = cpu_s(lambda: O.reprojection_error(3, dsp, kw, kh, sxyz_c, suv_c))
    emit("a16", "compute_reprojection_error (rmse/mean/std/min/max/median)", ns, g, None,
         len(sel), c)
    del errs

    # sample_points (a17): GPU on the 1e8-cell KB grid, CPU on 1e6 cells.
    # The C-ABI call on preallocated outputs / workspace, as a caller that
    # samples repeatedly would make it: util.sample_points also allocates
    # 4 GB of outputs and reads the kept count back (a host sync) per call,
    # which put ~0.3 ms of host time between the launches (r02's 1.28-1.44
    # ms figures against 1.08 ms of kernel time).
    from apex_camera_models.camera import _stream_handle
    cells = 100_000_000
    cam = src.acm_camera()
    # outputs sized to the grid acm_sample_points actually uses (ncx * ncy
    # may exceed the requested count; include/acm.h)
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
        _lib.check(L.acm_sample_points(ctypes.byref(cam), cells, su2.data_ptr(), sx3.data_ptr(),
                                       cnt.data_ptr(), sws.data_ptr(), wsb, _stream_handle()))
    g = gpu_ms(sp, reps=5)
    kept = int(cnt[0].item())
    c = cpu_s(lambda: O.sample_points(2, kp, kw, kh, 1_000_000))
    emit("a17", "sample_points (KB, cells; output 40 B per kept point)", cells, g,
         40 * kept / cells, 1_000_000, c)
    del su2, sx3, sws

    # linear estimation (a18): GPU TSQR + solve vs oracle A/b + numpy SVD lstsq
    g = gpu_ms(lambda: ds.linear_estimation(sxyz, suv), reps=5)

    def cpu_le():
        A, b, k = O.linear_estimation_system(3, dsp, sxyz_c, suv_c)
        np.linalg.lstsq(A, b, rcond=None)
    c = cpu_s(cpu_le)
    emit("a18", "DS linear_estimation (A, b and least squares)", ns, g, 40, len(sel), c)

    # FOV grid search (a18')
    fov = conversion._init_target("fov", src)
    g = gpu_ms(lambda: fov.linear_estimation(sxyz, suv), reps=3)
    mf = max(len(sel) // 10, 1000)
    c = cpu_s(lambda: O.fov_grid_search(fov.params(), sxyz_c[:mf], suv_c[:mf]))
    emit("a18'", "FOV linear_estimation (290-value grid search)", ns, g, None, mf, c)

    print("| row | what | GPU Mpts/s | GPU GB/s | CPU Mpts/s (1 thread) | GPU/CPU |",
          file=sys.stderr)
    print("|---|---|---|---|---|---|", file=sys.stderr)
    for d in rows:
        print(f"| {d['row']} | {d['what']} | {d['gpu_Mpts_s']} | {d['gpu_GBps'] or '—'} | "
              f"{d['cpu_Mpts_s']} | {d['gpu_over_cpu']} |", file=sys.stderr)


if __name__ == "__main__":
    main()
