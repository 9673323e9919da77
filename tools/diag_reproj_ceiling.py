"""Config-5's streaming passes at 92.9M KB-sampled correspondences beside
zero-compute probes of their exact traffic:

  real  reproj_stats    acm_reprojection_stats (k_reproj_pass1: 40 B read,
                        8 B error written per point) at the DS linear estimate
  real  reproj_error    acm_reprojection_error (the same pass + the median's
                        first histogram, then the radix-select median)
  real  normal_eq       acm_normal_equations (40 B read per point)
  real  opening         acm_linear_estimation_with_error (initial error +
                        TSQR in one read, the median, the host solve)
  real  tsqr            acm_linear_system_qr (TSQR of [A | b] alone, 40 B read)
  probe round_trip      acm_probe_round_trip: config 4's round-trip traffic (66 B per
                        point at --rt-points, one point per lane) with no model,
                        beside acm_project_unproject for Pinhole on the same points
  probe reproj_A{2,4,6}_{none,nt,plain}_g{grid}
                        tools/hbm_probe.hip acm_probe_reproj: the same loads in
                        the same static-slot pipeline, one 8-B store per point
                        (or none), no camera model

HIP events, best of --rounds blocks of --reps calls; every library in --libs
(A/B builds) is timed on the real calls, alternating.

  python tools/diag_reproj_ceiling.py [--libs a.so,b.so] [--only real,probe]
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
    ap.add_argument("--cells", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--libs", default="apex-camera-models_amd/lib/libacm.so")
    ap.add_argument("--only", default="real,probe")
    ap.add_argument("--grids", default="1024,2048")
    ap.add_argument("--rt-points", type=int, default=50_000_000)
    a = ap.parse_args()
    only = set(a.only.split(","))
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, conversion, samples, util
    sh = torch.cuda.current_stream().cuda_stream
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz = util.sample_points(src, a.cells)
    n = xyz.shape[0]
    ds = conversion._init_target("double_sphere", src)
    ds.linear_estimation(xyz, uv)
    dsp = list(ds.params())
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int

    def timed(fn):
        for _ in range(3):
            fn()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    def emit(name, ms, bytes_per_point, **kw):
        print(json.dumps({"call": name, "points": n, "ms": {k: round(v, 4) for k, v in ms.items()},
                          "TBps": {k: round(bytes_per_point * n / v / 1e9, 2) for k, v in ms.items()},
                          **kw}), flush=True)

    if "real" in only:
        libs = []
        for path in a.libs.split(","):
            L = ctypes.CDLL(os.path.join(ROOT, path) if not os.path.isabs(path) else path)
            L.acm_camera_init.argtypes = [vp, ci, vp, ci, ctypes.c_uint32, ctypes.c_uint32]
            L.acm_reprojection_stats_workspace_size.argtypes = [sz]
            L.acm_reprojection_stats_workspace_size.restype = sz
            L.acm_reprojection_error_workspace_size.argtypes = [sz]
            L.acm_reprojection_error_workspace_size.restype = sz
            L.acm_normal_equations_workspace_size.argtypes = [ci, sz]
            L.acm_normal_equations_workspace_size.restype = sz
            L.acm_linear_estimation_with_error_workspace_size.argtypes = [ci, sz]
            L.acm_linear_estimation_with_error_workspace_size.restype = sz
            L.acm_reprojection_stats.argtypes = [vp, sz, vp, ci, vp, vp, vp, vp, sz, vp]
            L.acm_reprojection_error.argtypes = [vp, sz, vp, ci, vp, vp, vp, vp, sz, vp]
            L.acm_normal_equations.argtypes = [vp, sz, vp, ci, vp, ci, vp, vp, sz, vp]
            L.acm_linear_estimation_with_error.argtypes = [vp, sz, vp, ci, vp, vp, vp, sz, vp]
            L.acm_linear_system_qr_workspace_size.argtypes = [ci, sz]
            L.acm_linear_system_qr_workspace_size.restype = sz
            L.acm_linear_system_qr.argtypes = [vp, sz, vp, ci, vp, vp, vp, vp, sz, vp]
            libs.append((os.path.relpath(os.path.abspath(path), ROOT), L))

        def cam(L, params):
            c = _lib.AcmCamera()
            rc = L.acm_camera_init(ctypes.byref(c), 3, (ctypes.c_double * len(params))(*params),
                                   len(params), w, h)
            assert rc == 0, rc
            return c

        errs = torch.empty((n,), dtype=torch.float64, device="cuda")
        res = torch.empty((80,), dtype=torch.float64, device="cuda")
        wsb = max(max(L.acm_reprojection_error_workspace_size(n),
                      L.acm_normal_equations_workspace_size(3, n),
                      L.acm_linear_estimation_with_error_workspace_size(3, n),
                      L.acm_linear_system_qr_workspace_size(3, n)) for _, L in libs)
        eflag = torch.zeros((4,), dtype=torch.int32, device="cuda")
        ws = torch.empty(((wsb + 7) // 8,), dtype=torch.float64, device="cuda")
        init = [240.0, 240.0, 256.0, 256.0, 0.5, 0.1]  # _init_target's DS start

        def calls(L):
            c = cam(L, dsp)
            c0 = cam(L, init)
            cw = _lib.AcmCamera()

            def opening():
                ctypes.memmove(ctypes.byref(cw), ctypes.byref(c0), ctypes.sizeof(cw))
                L.acm_linear_estimation_with_error(ctypes.byref(cw), n, xyz.data_ptr(), 0,
                                                   uv.data_ptr(), res.data_ptr(), ws.data_ptr(),
                                                   wsb, sh)
            return {
                "reproj_stats": (48, lambda: L.acm_reprojection_stats(
                    ctypes.byref(c), n, xyz.data_ptr(), 0, uv.data_ptr(), res.data_ptr(),
                    errs.data_ptr(), ws.data_ptr(), wsb, sh)),
                "reproj_error": (48, lambda: L.acm_reprojection_error(
                    ctypes.byref(c), n, xyz.data_ptr(), 0, uv.data_ptr(), res.data_ptr(),
                    errs.data_ptr(), ws.data_ptr(), wsb, sh)),
                "normal_eq": (40, lambda: L.acm_normal_equations(
                    ctypes.byref(c), n, xyz.data_ptr(), 0, uv.data_ptr(), 0, res.data_ptr(),
                    ws.data_ptr(), wsb, sh)),
                "opening": (48, opening),
                "tsqr": (40, lambda: L.acm_linear_system_qr(
                    ctypes.byref(c0), n, xyz.data_ptr(), 0, uv.data_ptr(), res.data_ptr(),
                    eflag.data_ptr(), ws.data_ptr(), wsb, sh)),
            }
        per_lib = [(tag, calls(L)) for tag, L in libs]
        for name in ("reproj_stats", "reproj_error", "normal_eq", "opening", "tsqr"):
            best = {}
            for rnd in range(a.rounds):
                for tag, cs in (per_lib if rnd % 2 == 0 else per_lib[::-1]):
                    best[tag] = min(best.get(tag, 1e9), timed(cs[name][1]))
            emit(name, best, per_lib[0][1][name][0])
        del errs, ws
    if "rt" in only:
        del uv, xyz
        P = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libhbmprobe.so"))
        P.acm_probe_round_trip.argtypes = [sz, vp, vp, vp, vp, vp, vp]
        L = _lib.load()
        m = a.rt_points
        pts = samples.synthetic_points_device(m)
        uv2 = torch.empty((m, 2), dtype=torch.float64, device="cuda")
        st = torch.empty((m,), dtype=torch.uint8, device="cuda")
        rays = torch.empty((m, 3), dtype=torch.float64, device="cuda")
        st2 = torch.empty((m,), dtype=torch.uint8, device="cuda")
        params, (pw, ph) = samples.SAMPLES[0]
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), 0, (ctypes.c_double * len(params))(
            *params), len(params), pw, ph))
        calls = {"probe": lambda: P.acm_probe_round_trip(m, pts.data_ptr(), uv2.data_ptr(),
                                                         st.data_ptr(), rays.data_ptr(),
                                                         st2.data_ptr(), sh),
                 "pinhole": lambda: L.acm_project_unproject(ctypes.byref(cam), m, pts.data_ptr(), 0,
                                                            uv2.data_ptr(), st.data_ptr(),
                                                            rays.data_ptr(), st2.data_ptr(), sh)}
        best = {}
        for rnd in range(a.rounds):
            for k, fn in (list(calls.items()) if rnd % 2 == 0 else list(calls.items())[::-1]):
                best[k] = min(best.get(k, 1e9), timed(fn))
        print(json.dumps({"call": "round_trip_traffic", "points": m,
                          "ms": {k: round(v, 4) for k, v in best.items()},
                          "TBps": {k: round(66 * m / v / 1e9, 2) for k, v in best.items()}}),
              flush=True)
        return
    if "probe" in only:
        P = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libhbmprobe.so"))
        P.acm_probe_reproj.argtypes = [sz, vp, vp, vp, vp, ci, ci, ci, vp]
        err = torch.empty((n,), dtype=torch.float64, device="cuda")
        acc = torch.zeros((8192 * 4,), dtype=torch.float64, device="cuda")
        for g in (int(x) for x in a.grids.split(",")):
            for slots in (2, 4, 6):
                for store, sname in ((0, "none"), (1, "nt"), (2, "plain")):
                    ms = min(timed(lambda: P.acm_probe_reproj(
                        n, xyz.data_ptr(), uv.data_ptr(), err.data_ptr(), acc.data_ptr(), g,
                        slots, store, sh)) for _ in range(a.rounds))
                    emit(f"probe_reproj_A{slots}_{sname}_g{g}", {"probe": ms},
                         40 + (8 if store else 0))


if __name__ == "__main__":
    main()
