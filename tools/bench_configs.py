"""Secondary measurements for BASELINE.json configs 1, 3, 4 and 5 (config 2 is
bench.py, the headline).  One JSON line per measurement; not the driver's
bench contract.

  python tools/bench_configs.py [--configs 1,3,4,5] [--scale 1.0]
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


def emit(d):
    print(json.dumps(d), flush=True)


def timed(fn, reps=20, warm=3, blocks=3):
    """GPU time per call: the fastest of `blocks` blocks of `reps` back-to-back
    calls, each block bracketed by one event pair (so the host-side
    ctypes/Python cost of each call overlaps the previous call's kernels
    instead of being counted as GPU time; the fastest block is the steady
    state, free of clock ramps and other processes' interference)."""
    import time

    import torch
    # at least `warm` calls and >= 50 ms of them: the clocks ramp over
    # milliseconds (a few calls of a 0.08 ms kernel timed it ~10% slow)
    torch.cuda.synchronize()
    t0, k = time.perf_counter(), 0
    while k < warm or time.perf_counter() - t0 < 0.05:
        fn()
        torch.cuda.synchronize()
        k += 1
    best = float("inf")
    for _ in range(blocks):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / reps)
    return best


def config1():
    """Pinhole project/unproject, 1k points, CPU reference path (oracle)
    500/500/320/240 @ 640x480 (tests/projection_accuracy.rs:50-53)."""
    import oracle as O
    p = [500.0, 500.0, 320.0, 240.0]
    rng = np.random.default_rng(1)
    pts = np.stack([rng.uniform(-0.3, 0.3, 1000), rng.uniform(-0.2, 0.2, 1000),
                    rng.uniform(0.5, 4.0, 1000)], 1)
    t0 = time.perf_counter()
    for _ in range(100):
        uv, st, _ = O.project(0, p, 640, 480, pts)
        ray, st2 = O.unproject(0, p, 640, 480, uv[st == 0])
    dt = (time.perf_counter() - t0) / 100
    pn = pts[st == 0] / np.linalg.norm(pts[st == 0], axis=1, keepdims=True)
    dots = (pn * ray).sum(1)
    emit({"config": 1, "what": "pinhole project+unproject 1k pts, CPU oracle (1 thread)",
          "ms": round(dt * 1e3, 4), "Mpoints_per_s": round(1000 / dt / 1e6, 2),
          "valid": int((st == 0).sum()), "min_round_trip_dot": float(dots.min())})


def lm_wall(src, xyz, uv, target, reps=5):
    """The bounded LM alone (camera_converter.rs:381-420), from the linear
    estimate: wall time of LevenbergMarquardt.optimize (every evaluation's
    fused normal equations, the host solve and the host <-> device round
    trip), the fastest of `reps` runs after one warm-up run."""
    import torch
    from apex_camera_models import conversion
    from apex_camera_models.optimizer import CONVERTER_BOUNDS, LevenbergMarquardt
    init = conversion._init_target(target, src)
    init.linear_estimation(xyz, uv)
    p0 = init.params()
    best, res = float("inf"), None
    for _ in range(reps + 1):
        m = conversion._init_target(target, src)
        m._set_params(list(p0))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = LevenbergMarquardt().optimize(m, xyz, uv, bounds=CONVERTER_BOUNDS[target])
        best = min(best, time.perf_counter() - t0)
    return {"what": f"bounded LM alone ({target}, from the linear estimate), wall",
            "points": int(xyz.shape[0]), "lm_ms": round(best * 1e3, 3),
            "iterations": res.iterations, "evaluations": res.evaluations,
            "ms_per_evaluation": round(best * 1e3 / res.evaluations, 4),
            "termination": res.termination}


def warm_convert(src, xyz, uv, reps=3, cells=None):
    """conversion.convert to double_sphere (camera_converter.rs:355-488),
    wall: one untimed call first (the caching allocator's first multi-GB
    workspaces and the first launches), then the fastest of `reps`.
    cells (r06): the util.CellSample of uv -- the cell form bench.py's
    config-5 leg runs (same results)."""
    import torch
    from apex_camera_models import conversion
    kw = {"cells": cells} if cells is not None else {}
    conversion.convert(src, "double_sphere", xyz, uv, **kw)
    best, met = float("inf"), None
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        met = conversion.convert(src, "double_sphere", xyz, uv, **kw)
        best = min(best, time.perf_counter() - t0)
    return met, best


def config3(n_target):
    """DS residual+J and fused normal equations over ~10M KB-sampled
    correspondences, inside the bounded LM of camera_converter.rs:355-488."""
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, conversion, factors
    from apex_camera_models import samples, util
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    t0 = time.perf_counter()
    uv, xyz = util.sample_points(src, n_target)
    torch.cuda.synchronize()
    t_sample = time.perf_counter() - t0
    n = xyz.shape[0]
    model = conversion._init_target("double_sphere", src)
    model.linear_estimation(xyz, uv)
    f = factors.DoubleSphereCameraParamsFactor(xyz, uv, Resolution(w, h))
    p = model.params()
    res = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    jac = torch.empty((6, n, 2), dtype=torch.float64, device="cuda")
    cam = model.acm_camera()
    L = _lib.load()
    sh = torch.cuda.current_stream().cuda_stream

    def rj():
        L.acm_residual_jacobian(ctypes.byref(cam), n, xyz.data_ptr(), 0, uv.data_ptr(), 0,
                                res.data_ptr(), jac.data_ptr(), None, sh)

    old = L.acm_set_tuning(1, 0)
    ms_rj_plain = timed(rj)
    L.acm_set_tuning(1, 1)
    ms_rj_nt = timed(rj)
    L.acm_set_tuning(1, old)
    emit({"config": 3, "what": "residual+J store policy A/B", "plain_ms": round(ms_rj_plain, 4),
          "nt_ms": round(ms_rj_nt, 4)})
    ms_rj = timed(rj)
    out = torch.empty((6 * 6 + 6 + 2,), dtype=torch.float64, device="cuda")
    ms_ne = timed(lambda: f.normal_equations(p, out))
    torch.cuda.synchronize()
    met, t_conv = warm_convert(src, xyz, uv)
    emit({"config": 3, **lm_wall(src, xyz, uv, "double_sphere")})
    emit({"config": 3, "what": "DS residual+J (2N x 6) kernel", "points": n,
          "ms": round(ms_rj, 4), "Mpoints_per_s": round(n / ms_rj / 1e3, 1),
          "GBps": round(153 * n / ms_rj / 1e6, 1)})
    emit({"config": 3, "what": "DS fused normal equations (JtJ, Jtr, cost)", "points": n,
          "ms": round(ms_ne, 4), "Mpoints_per_s": round(n / ms_ne / 1e3, 1),
          "GBps": round(40 * n / ms_ne / 1e6, 1)})
    emit({"config": 3,
          "what": "KB->DS conversion: linear estimation + bounded LM (wall, warm, best of 3)",
          "points": n, "sample_points_s": round(t_sample, 4), "convert_s": round(t_conv, 4),
          "lm_iterations": met.lm_iterations, "termination": met.lm_termination,
          "final_mean_px": met.final_reprojection_error.mean,
          "initial_mean_px": met.initial_reprojection_error.mean})


def config3_ne_all(n):
    """Fused normal equations for every model on the same synthetic batch."""
    import torch
    from apex_camera_models import _lib, factors, samples
    from apex_camera_models.camera import Resolution
    pts = samples.synthetic_points_device(n)
    pts = pts[torch.isfinite(pts).all(1)].contiguous()
    n = pts.shape[0]
    facs = [factors.PinholeCameraParamsFactor, factors.RadTanCameraParamsFactor,
            factors.KannalaBrandtCameraParamsFactor, factors.DoubleSphereCameraParamsFactor,
            factors.UcmCameraParamsFactor, factors.EucmCameraParamsFactor,
            factors.FovCameraParamsFactor]
    only = os.environ.get("NE_MODELS")  # e.g. "2": restrict the sweep
    for mid, fcls in enumerate(facs):
        if only and str(mid) not in only.split(","):
            continue
        params, (w, h) = samples.SAMPLES[mid]
        m = fcls.MODEL._from_params(list(params), Resolution(w, h))
        uv, _, _ = m.project_batch(pts)
        obs = torch.nan_to_num(uv, nan=0.0) + 0.25
        f = fcls(pts, obs, Resolution(w, h))
        P = len(params)
        out = torch.empty((P * P + P + 2,), dtype=torch.float64, device="cuda")
        L = _lib.load()
        res = {}
        # nt loads measured 5-11% faster in every cell (profiles/r01_ne_sweep.log);
        # unroll 3 = one point per step, loads two steps ahead
        combos = [(0, 0, -1)] + [(wv, un, 1) for wv in (1, 3, 4) for un in (1, 2, 3)]
        if mid == 2:  # KB: loads 3 and 4 steps ahead too
            combos += [(wv, un, 1) for wv in (1, 3) for un in (4, 5)]
        for rep in range(2):  # interleaved A/B: register target x lane step x nt loads
            for wv, un, nl in combos:
                L.acm_set_tuning(_lib.TUNE_NE_WAVES, wv)
                L.acm_set_tuning(_lib.TUNE_NE_UNROLL, un)
                L.acm_set_tuning(_lib.TUNE_NT_LOADS, nl)
                res.setdefault((wv, un, nl), []).append(
                    timed(lambda: f.normal_equations(params, out)))
                if rep == 0 and (wv, un, nl) == combos[0]:
                    ref = out.clone()
                elif rep == 0:  # grid size / lane order -> summation order
                    assert torch.allclose(out, ref, rtol=1e-12, atol=0.0), (wv, un, nl)
        L.acm_set_tuning(_lib.TUNE_NE_WAVES, 0)
        L.acm_set_tuning(_lib.TUNE_NE_UNROLL, 0)
        L.acm_set_tuning(_lib.TUNE_NT_LOADS, -1)
        ms = {k: min(v) for k, v in res.items()}
        best = min(ms, key=ms.get)
        emit({"config": 3, "what": "fused normal equations", "model": fcls.MODEL.__name__,
              "points": n, "ms_by_waves_unroll_ntl": {
                  f"w{k[0]}u{k[1]}n{k[2]}": round(v, 4) for k, v in ms.items()},
              "best": f"w{best[0]}u{best[1]}n{best[2]}",
              "Mpoints_per_s": round(n / ms[best] / 1e3, 1),
              "GBps": round(40 * n / ms[best] / 1e6, 1)})


def config_fov(n_target):
    """FOV linear_estimation (fov.rs:153-251 grid search, 290 x N evaluations)
    on KB-sampled correspondences, then the full KB->FOV conversion."""
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, samples, util
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz = util.sample_points(src, n_target)
    n = xyz.shape[0]
    m = conversion._init_target("fov", src)
    from apex_camera_models import _lib
    L = _lib.load()
    by = {}
    # interleaved A/B: -1 = point-lane form (r03), 0 = LDS records read one
    # point ahead (r03), 1 / 2 / 4 = the round-2 LDS kernel
    US = (-1, 0, 1, 2, 4)
    for rep in range(2):
        for u in US:
            L.acm_set_tuning(_lib.TUNE_FOV_UNROLL, u)
            m.w = 1.0
            by.setdefault(u, []).append(timed(lambda: m.linear_estimation(xyz, uv), reps=3,
                                              warm=1))
            by.setdefault(("w", u), []).append(m.w)
    L.acm_set_tuning(_lib.TUNE_FOV_UNROLL, -1)
    assert len({v[0] for k, v in by.items() if isinstance(k, tuple)}) == 1
    ms = min(by[-1])
    emit({"config": "fov", "what": "FOV grid kernel A/B",
          "ms_by_unroll": {str(u): round(min(by[u]), 3) for u in US}})
    met = conversion.convert(src, "fov", xyz, uv)
    emit({"config": "fov", "what": "FOV grid-search linear estimation", "points": n,
          "ms": round(ms, 3), "evaluations_per_s": round(290 * n / ms / 1e3, 1), "w": m.w,
          "convert_ms": round(met.optimization_time_ms, 2), "lm_iterations": met.lm_iterations,
          "termination": met.lm_termination,
          "final_mean_px": met.final_reprojection_error.mean})


def config4(n_per_model):
    """Every model: project -> unproject round trip (two launches, uv
    intermediate in HBM), plus the round-trip error sum (RCCL all-reduce on
    >1 rank)."""
    import torch
    from apex_camera_models import _lib, samples
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    names = {0: "pinhole", 1: "rad_tan", 2: "kannala_brandt", 3: "double_sphere", 4: "ucm",
             5: "eucm"}
    pts = samples.synthetic_points_device(n_per_model)
    L = _lib.load()
    for mid, name in names.items():
        params, (w, h) = samples.SAMPLES[mid]
        m = MODEL_CLASSES[name]._from_params(params, Resolution(w, h))
        cam = m.acm_camera()
        uv = torch.empty((n_per_model, 2), dtype=torch.float64, device="cuda")
        st = torch.empty((n_per_model,), dtype=torch.uint8, device="cuda")
        ray = torch.empty((n_per_model, 3), dtype=torch.float64, device="cuda")
        st2 = torch.empty((n_per_model,), dtype=torch.uint8, device="cuda")
        sh = torch.cuda.current_stream().cuda_stream

        def rt():
            L.acm_project(ctypes.byref(cam), n_per_model, pts.data_ptr(), 0, uv.data_ptr(),
                          st.data_ptr(), None, sh)
            L.acm_unproject(ctypes.byref(cam), n_per_model, uv.data_ptr(), ray.data_ptr(), 0,
                            st2.data_ptr(), sh)

        ms_f = timed(lambda: L.acm_project_unproject(ctypes.byref(cam), n_per_model,
                                                     pts.data_ptr(), 0, uv.data_ptr(),
                                                     st.data_ptr(), ray.data_ptr(),
                                                     st2.data_ptr(), sh))
        ms = timed(rt)
        ms_u = timed(lambda: L.acm_unproject(ctypes.byref(cam), n_per_model, uv.data_ptr(),
                                             ray.data_ptr(), 0, st2.data_ptr(), sh))
        ok = (st == 0) & (st2 == 0) & torch.isfinite(pts).all(1)
        pn = pts[ok] / torch.linalg.norm(pts[ok], dim=1, keepdim=True)
        err = torch.linalg.norm(ray[ok] - pn, dim=1)
        emit({"config": 4, "model": name, "points": n_per_model,
              "round_trip_ms": round(ms, 4), "round_trip_Mpoints_per_s": round(
                  n_per_model / ms / 1e3, 1),
              "round_trip_GBps": round(82 * n_per_model / ms / 1e6, 1),
              "fused_round_trip_ms": round(ms_f, 4),
              "fused_round_trip_GBps": round(66 * n_per_model / ms_f / 1e6, 1),
              "unproject_ms": round(ms_u, 4),
              "unproject_GBps": round(41 * n_per_model / ms_u / 1e6, 1),
              "round_trip_ok": int(ok.sum()), "max_round_trip_err": float(err.max()),
              "sum_sq_err": float((err * err).sum())})
        del uv, st, ray, st2
    torch.cuda.empty_cache()


def config5(n_cells):
    """KB -> DS on ~1e8 sampled correspondences (10000 x 10000 grid) + the
    f32-vs-f64 sweep of the DS projection at the optimum."""
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, samples, util
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz = util.sample_points(src, n_cells)  # warm-up: the allocator's first
    del uv, xyz                                 # multi-GB hipMalloc is not the kernel
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    uv, xyz = util.sample_points(src, n_cells)
    torch.cuda.synchronize()
    t_s = time.perf_counter() - t0
    n = xyz.shape[0]
    met, t_c = warm_convert(src, xyz, uv)
    emit({"config": 5, **lm_wall(src, xyz, uv, "double_sphere", reps=2)})
    emit({"config": 5, "what": "KB->DS conversion (sample_points; convert() wall, warm, best of 3)",
          "requested": n_cells, "correspondences": n, "sample_points_s": round(t_s, 4),
          "convert_s": round(t_c, 4), "lm_iterations": met.lm_iterations,
          "termination": met.lm_termination,
          "final_mean_px": met.final_reprojection_error.mean,
          "final_rmse_px": met.final_reprojection_error.rmse})
    del uv, xyz
    torch.cuda.empty_cache()
    uv, xyz, cs = util.sample_points(src, n_cells, cells=True)
    met_c, t_cc = warm_convert(src, xyz, uv, cells=cs)
    emit({"config": 5, "what": "KB->DS conversion on the cell form (convert(cells=...), as "
                               "bench.py's config5; wall, warm, best of 3)",
          "correspondences": int(xyz.shape[0]), "convert_s": round(t_cc, 4),
          "lm_iterations": met_c.lm_iterations,
          "same_params_as_pixels": met_c.model.params() == met.model.params()})
    del cs
    ds = met.model
    uv64, st64, _ = ds.project_batch(xyz)
    uv32, st32, _ = ds.project_batch(xyz.to(torch.float32))
    both = (st64 == 0) & (st32 == 0)
    d = ((uv32.double() - uv64).abs() / uv64.abs().clamp(min=1.0)).max(dim=1).values
    d = torch.where(both, d, torch.zeros_like(d))
    i = int(d.argmax())
    q = torch.quantile(d[both][:: max(1, int(both.sum()) // 1_000_000)], 0.9999)
    emit({"config": 5, "what": "f32 vs f64 DS projection sweep at the optimum",
          "points": n, "mask_disagreements": int((st64 != st32).sum()),
          "max_rel_err_f32": float(d[i]), "p9999_rel_err_f32": float(q),
          "worst": {"xyz": xyz[i].tolist(), "uv64": uv64[i].tolist(),
                    "uv32": uv32[i].tolist()}, "ds_params": ds.params()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,3,4,5")
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    cs = a.configs.split(",")
    if "1" in cs:
        config1()
    if "3" in cs:
        config3(int(10_000_000 * a.scale))
    if "fov" in cs:
        config_fov(int(10_000_000 * a.scale))
    if "3ne" in cs:
        config3_ne_all(int(10_000_000 * a.scale))
    if "4" in cs:
        config4(int(6_250_000 * a.scale))
    if "5" in cs:
        config5(int(100_000_000 * a.scale))


if __name__ == "__main__":
    main()
