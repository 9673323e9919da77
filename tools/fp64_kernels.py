"""Driver for the counter passes of the kernels DESIGN.md calls FP64-VALU
bound: RadTan and KB unproject (10M pixels), KB fused
normal equations (10M points), the FOV grid search (9.3M KB-sampled
correspondences) and sample_points (1e8-cell KB grid, the default segment path).  Each runs
`--reps` times after one warm-up; the HIP-event time per call is printed as
one JSON line per kernel, so the same command under `rocprofv3 --pmc ...`
yields per-dispatch counters and the event times side by side.

  python tools/fp64_kernels.py [--only radtan_unproject,kb_unproject,...] [--reps 5]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)

ALL = ("radtan_unproject", "kb_unproject", "kb_normal_eq", "fov_grid", "sample_kb")
# also selectable with --only: "ds_ne9" / "ds_ne93", the DS fused normal
# equations on the config-3 (9.29M) / config-5 (92.9M) KB-sampled
# correspondences at the DS linear estimate (the LM's inner loop);
# "ds_reproj9" / "ds_reproj93", compute_reprojection_error on the same data;
# "ds_prologue9" / "ds_prologue93", the initial error + linear estimation;
# "ds_ne93c" / "ds_reproj93c" / "ds_prologue93c" (r06): the same three at
# 92.9M on the cell form config 5 now runs (4-B cells instead of 16-B pixels)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=",".join(ALL))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--cells", type=int, default=100_000_000)
    ap.add_argument("--rt-points", type=int, default=50_000_000,
                    help="points of the rt_* (config-4 round trip) kernels")
    ap.add_argument("--sample-fused", type=int, default=None,
                    help="ACM_TUNE_SAMPLE_FUSED for sample_kb (-1 auto = segment path, 0 two-pass, 1/2/3 = single pass R 2/4/8)")
    ap.add_argument("--lib", default=None, help="load this libacm build instead (A/B builds, "
                    "e.g. make -C apex-camera-models_amd ieee)")
    a = ap.parse_args()
    want = set(a.only.split(","))
    if a.lib:
        os.environ["ACM_LIB_PATH"] = os.path.abspath(a.lib)
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, conversion, factors
    from apex_camera_models import samples, util
    L = _lib.load()
    assert os.path.samefile(_lib.LIB_PATH, a.lib or _lib.LIB_PATH)
    sh = torch.cuda.current_stream().cuda_stream
    n = a.points

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    def emit(name, units, ms, bytes_per_unit, **kw):
        d = {"kernel": name, "units": units, "ms": round(ms, 4),
             "GBps": round(bytes_per_unit * units / ms / 1e6, 1) if bytes_per_unit else None, **kw}
        print(json.dumps(d), flush=True)

    pts = samples.synthetic_points_device(n)
    for mid, name in ((1, "radtan_unproject"), (2, "kb_unproject")):
        if name not in want:
            continue
        params, (w, h) = samples.SAMPLES[mid]
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * len(params))(
            *params), len(params), w, h))
        uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
        st = torch.empty((n,), dtype=torch.uint8, device="cuda")
        L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(), st.data_ptr(),
                      None, sh)
        uv = torch.nan_to_num(uv, nan=1.0).contiguous()
        rays = torch.empty((n, 3), dtype=torch.float64, device="cuda")
        ms = timed(lambda: L.acm_unproject(ctypes.byref(cam), n, uv.data_ptr(), rays.data_ptr(),
                                           0, st.data_ptr(), sh))
        emit(name, n, ms, 41)
        del uv, rays, st
    # config 4's fused round trip (acm_project_unproject) at the bench leg's
    # 50M points on one GPU: rt_pinhole, rt_radtan, rt_kb, rt_ds, rt_ucm, rt_eucm
    rt = [(mid, nm) for mid, nm in ((0, "rt_pinhole"), (1, "rt_radtan"), (2, "rt_kb"),
                                    (3, "rt_ds"), (4, "rt_ucm"), (5, "rt_eucm")) if nm in want]
    if rt:
        del pts
        m = a.rt_points
        p50 = samples.synthetic_points_device(m)
        uv = torch.empty((m, 2), dtype=torch.float64, device="cuda")
        st = torch.empty((m,), dtype=torch.uint8, device="cuda")
        rays = torch.empty((m, 3), dtype=torch.float64, device="cuda")
        st2 = torch.empty((m,), dtype=torch.uint8, device="cuda")
        for mid, name in rt:
            params, (w, h) = samples.SAMPLES[mid]
            cam = _lib.AcmCamera()
            _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * len(params))(
                *params), len(params), w, h))
            ms = timed(lambda: _lib.check(L.acm_project_unproject(
                ctypes.byref(cam), m, p50.data_ptr(), 0, uv.data_ptr(), st.data_ptr(),
                rays.data_ptr(), st2.data_ptr(), sh)))
            emit(name, m, ms, 66)
        del p50, uv, st, rays, st2
        pts = samples.synthetic_points_device(n)
    if "kb_normal_eq" in want:
        p2 = pts[torch.isfinite(pts).all(1)].contiguous()
        params, (w, h) = samples.SAMPLES[2]
        m = KannalaBrandtModel._from_params(list(params), Resolution(w, h))
        uv, _, _ = m.project_batch(p2)
        obs = torch.nan_to_num(uv, nan=0.0) + 0.25
        f = factors.KannalaBrandtCameraParamsFactor(p2, obs, Resolution(w, h))
        out = torch.empty((8 * 8 + 8 + 2,), dtype=torch.float64, device="cuda")
        ms = timed(lambda: f.normal_equations(params, out))
        emit("kb_normal_eq", p2.shape[0], ms, 40)
        del p2, uv, obs, f
    del pts
    kp, (kw, kh) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(kw, kh))
    if "fov_grid" in want:
        suv, sxyz = util.sample_points(src, n)
        fov = conversion._init_target("fov", src)
        ms = timed(lambda: fov.linear_estimation(sxyz, suv))
        emit("fov_grid", sxyz.shape[0], ms, 40, evaluations=290 * sxyz.shape[0])
        del suv, sxyz
    for tag, rtag, ptag, cells in (("ds_ne9", "ds_reproj9", "ds_prologue9", 10_000_000),
                                   ("ds_ne93", "ds_reproj93", "ds_prologue93", 100_000_000)):
        if tag not in want and rtag not in want and ptag not in want:
            continue
        suv, sxyz = util.sample_points(src, cells)
        if ptag in want:  # initial error + linear estimation, one pass (48 B per point)
            ms = timed(lambda: util.initial_error_and_linear_estimation(
                conversion._init_target("double_sphere", src), sxyz, suv))
            emit(ptag, sxyz.shape[0], ms, 48)
        ds = conversion._init_target("double_sphere", src)
        ds.linear_estimation(sxyz, suv)
        if tag in want:
            f = factors.DoubleSphereCameraParamsFactor(sxyz, suv, Resolution(kw, kh))
            out = torch.empty((6 * 6 + 6 + 2,), dtype=torch.float64, device="cuda")
            p = ds.params()
            ms = timed(lambda: f.normal_equations(p, out))
            emit(tag, sxyz.shape[0], ms, 40)
            del f
        if rtag in want:  # compute_reprojection_error (reads 40 B, writes 8 B per point)
            ms = timed(lambda: util.compute_reprojection_error(ds, sxyz, suv))
            emit(rtag, sxyz.shape[0], ms, 48)
        del suv, sxyz
    if want & {"ds_ne93c", "ds_reproj93c", "ds_prologue93c"}:
        suv, sxyz, cs = util.sample_points(src, 100_000_000, cells=True)
        n = sxyz.shape[0]
        if "ds_prologue93c" in want:  # reads 28 B, writes 8 B per point
            ms = timed(lambda: util.initial_error_and_linear_estimation(
                conversion._init_target("double_sphere", src), sxyz, suv, cells=cs))
            emit("ds_prologue93c", n, ms, 36)
        ds = conversion._init_target("double_sphere", src)
        ds.linear_estimation(sxyz, suv)
        if "ds_ne93c" in want:  # reads 28 B per point
            cam = ds.acm_camera()
            wsb = L.acm_normal_equations_workspace_size(3, n)
            ws = torch.empty((wsb // 8 + 1,), dtype=torch.float64, device="cuda")
            out = torch.empty((6 * 6 + 6 + 2,), dtype=torch.float64, device="cuda")
            sh = torch.cuda.current_stream().cuda_stream
            ms = timed(lambda: L.acm_normal_equations_cells(
                ctypes.byref(cam), n, sxyz.data_ptr(), 0, cs.cells.data_ptr(),
                ctypes.byref(cs.grid), 0, out.data_ptr(), ws.data_ptr(), wsb, sh))
            emit("ds_ne93c", n, ms, 28)
            del ws
        if "ds_reproj93c" in want:  # reads 28 B, writes 8 B per point
            ms = timed(lambda: util.compute_reprojection_error(ds, sxyz, suv, cells=cs))
            emit("ds_reproj93c", n, ms, 36)
        del suv, sxyz, cs
    if "sample_kb" in want:
        if a.sample_fused is not None:
            L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, a.sample_fused)
        kept = util.sample_points(src, a.cells)[0].shape[0]
        ms = timed(lambda: util.sample_points(src, a.cells))
        emit("sample_kb", a.cells, ms, None, kept=kept,
             kept_GBps=round(40 * kept / ms / 1e6, 1))


if __name__ == "__main__":
    main()
