"""One-off measurement probes of the hot path (r03-r06), one subcommand each:

  python tools/probes.py <probe> [args]     (python tools/probes.py -h lists them)

Each probe's docstring says what it measures; profiles/README.md names the
logs each produced.  Probes only read the library through the public Python
package or the C-ABI; none is part of the product path.  (Folded from the
former tools/diag_*.py scripts in r06)"""
import argparse
import ctypes
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)


def probe_convert(argv):
    """Stage breakdown of the config-5 KB -> DS conversion (conversion.convert,
    camera_converter.rs:355-488) at 1e8 sampled cells: the initial reprojection
    statistics, the linear estimation, the bounded LM, the final reprojection
    statistics and the five-pixel validation, each synchronised and timed warm
    (one full convert() first), plus the whole convert() wall, cold and warm."""
    ap = argparse.ArgumentParser(prog="probes.py convert")
    ap.add_argument("--cells", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args(argv)
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, samples, util
    from apex_camera_models.optimizer import CONVERTER_BOUNDS, LevenbergMarquardt
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz = util.sample_points(src, a.cells)
    torch.cuda.synchronize()

    def wall(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3, r

    cold, _ = wall(lambda: conversion.convert(src, "double_sphere", xyz, uv))
    warm = [wall(lambda: conversion.convert(src, "double_sphere", xyz, uv))[0]
            for _ in range(a.reps)]
    stages = {k: [] for k in ("init_target", "initial_reproj", "linear_estimation",
                              "initial_and_linear_fused", "lm", "final_reproj", "validation")}
    for _ in range(a.reps):
        t, m = wall(lambda: conversion._init_target("double_sphere", src))
        stages["init_target"].append(t)
        stages["initial_reproj"].append(wall(lambda: util.compute_reprojection_error(
            m, xyz, uv))[0])
        stages["linear_estimation"].append(wall(lambda: m.linear_estimation(xyz, uv))[0])
        # what convert() runs (r04): the two stages above in one pass
        m2 = conversion._init_target("double_sphere", src)
        stages["initial_and_linear_fused"].append(wall(
            lambda: util.initial_error_and_linear_estimation(m2, xyz, uv))[0])
        t, res = wall(lambda: LevenbergMarquardt().optimize(
            m, xyz, uv, bounds=CONVERTER_BOUNDS["double_sphere"]))
        stages["lm"].append(t)
        stages["final_reproj"].append(wall(lambda: util.compute_reprojection_error(
            m, xyz, uv))[0])
        stages["validation"].append(wall(lambda: util.validate_conversion_accuracy(m, src))[0])
    print(json.dumps({"what": "config-5 convert() stage breakdown (ms, best of reps, warm)",
                      "correspondences": int(xyz.shape[0]), "convert_cold_ms": round(cold, 3),
                      "convert_warm_ms": round(min(warm), 3),
                      "convert_warm_all_ms": [round(x, 3) for x in warm],
                      "lm_evaluations": res.evaluations, "lm_iterations": res.iterations,
                      **{k: round(min(v), 3) for k, v in stages.items()}}), flush=True)


def probe_convert_sharded(argv):
    """Cost of the sharded conversion path on one GPU: the
    config-5 KB -> DS convert() at 1e8 sampled cells, warm, best of --reps,

      none   -- conversion.convert(collective=None): the 1-rank path;
      cells  -- the same with the LM on the cell form (r06, util.CellSample);
      py     -- a 1-rank process group and the torch.distributed callbacks
                (distributed.TorchCollective; before r06: rccl_allreduce);
      rccl   -- a 1-rank RCCL communicator driven from libacm
                (distributed.RcclCollective, no Python per collective),

    interleaved round by round.  Prints one JSON line: per mode the convert wall,
    the LM's evaluations and the parameters (which must agree bit for bit), and
    the per-evaluation overhead of each sharded mode over `none`."""
    ap = argparse.ArgumentParser(prog="probes.py convert_sharded")
    ap.add_argument("--cells", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="none,py,rccl")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, samples, util
    from apex_camera_models import distributed as D
    torch.cuda.set_device(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz, cs = util.sample_points(src, a.cells, cells=True)
    torch.cuda.synchronize()
    colls = {}
    for m in a.modes.split(","):
        if m in ("none", "cells"):
            colls[m] = None
        elif m == "rccl_cells" and hasattr(D, "RcclCollective"):
            colls[m] = D.RcclCollective()
        elif m == "py" and hasattr(D, "TorchCollective"):
            colls[m] = D.TorchCollective()
        elif m == "py":
            colls[m] = "legacy"
        elif m == "rccl" and hasattr(D, "RcclCollective"):
            colls[m] = D.RcclCollective()

    def run(m, c):
        if c == "legacy":
            return conversion.convert(src, "double_sphere", xyz, uv, allreduce=D.rccl_allreduce())
        kw = {"cells": cs} if m.endswith("cells") else {}
        if c is None:
            return conversion.convert(src, "double_sphere", xyz, uv, **kw)
        return conversion.convert(src, "double_sphere", xyz, uv, collective=c, **kw)

    best, info = {}, {}
    for m, c in colls.items():  # cold run: workspaces, communicator warm-up
        run(m, c)
    for _ in range(a.reps):
        for m, c in colls.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            met = run(m, c)
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) * 1e3
            best[m] = min(best.get(m, float("inf")), t)
            info[m] = {"lm_iterations": met.lm_iterations, "params": met.model.params(),
                       "final_mean": met.final_reprojection_error.mean,
                       "final_median": met.final_reprojection_error.median,
                       "initial_median": met.initial_reprojection_error.median,
                       "optimization_ms": round(met.optimization_time_ms, 3)}
    out = {"what": "config-5 convert() on one GPU: 1-rank path vs the sharded path at world 1 "
                   "(ms, warm, best of reps, modes interleaved)",
           "correspondences": int(xyz.shape[0]),
           "convert_ms": {m: round(v, 3) for m, v in best.items()}, "modes": info}
    if "none" in best:
        ref = info["none"]
        for m in best:
            if m == "none":
                continue
            out[f"{m}_over_none_pct"] = round(100 * (best[m] / best["none"] - 1), 2)
            out[f"{m}_same_bits"] = (info[m]["params"] == ref["params"]
                                     and info[m]["final_median"] == ref["final_median"]
                                     and info[m]["initial_median"] == ref["initial_median"])
    print(json.dumps(out), flush=True)
    for c in colls.values():
        if hasattr(c, "close"):
            c.close()
    dist.destroy_process_group()


def probe_lm(argv):
    """LM loop overhead on config-3 data (KB-sampled correspondences, DS target):
    wall time of acm_lm_optimize vs evaluations x the normal-equation kernel
    time, i.e. the host / launch / copy cost per evaluation, for the host loop
    with each ACM_TUNE_LM_HOST_RESULT mode (0 copy + sync, 1 pinned + sync, 2
    pinned + spin on the completion word, 3 (r06) pre-queued evaluations behind a
    host-written doorbell); the reported wall is the default.  Every mode must
    take the same iterates (same parameters bit for bit).
    (r04 also timed a device-resident loop here; it was removed in r05.)

      python tools/probes.py lm [--points N]"""
    ap = argparse.ArgumentParser(prog="probes.py lm")
    ap.add_argument("--points", type=int, default=10_000_000)
    a = ap.parse_args(argv)
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, factors, samples
    from apex_camera_models import util
    from apex_camera_models.optimizer import (CONVERTER_BOUNDS, LevenbergMarquardt,
                                              LevenbergMarquardtConfig)
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz = util.sample_points(src, a.points)
    n = xyz.shape[0]
    base = conversion._init_target("double_sphere", src)
    base.linear_estimation(xyz, uv)
    p0 = base.params()
    f = factors.DoubleSphereCameraParamsFactor(xyz, uv, Resolution(w, h))
    out = torch.empty((44,), dtype=torch.float64, device="cuda")
    for _ in range(3):
        f.normal_equations(p0, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f.normal_equations(p0, out)
    e1.record()
    torch.cuda.synchronize()
    ne_ms = e0.elapsed_time(e1) / 20
    from apex_camera_models import _lib
    L = _lib.load()
    by_mode = {}
    res = None
    modes = {"host0": 0, "host1": 1, "host2": 2, "host3": 3}
    params = {}
    for _ in range(3):
        for mode, host in modes.items():
            L.acm_set_tuning(_lib.TUNE_LM_HOST_RESULT, host)
            m = conversion._init_target("double_sphere", src)
            m._set_params(list(p0))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = LevenbergMarquardt(LevenbergMarquardtConfig()).optimize(
                m, xyz, uv, bounds=CONVERTER_BOUNDS["double_sphere"])
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            by_mode[mode] = min(by_mode.get(mode, 1e9), ms)
            params[mode] = (tuple(res.parameters), res.evaluations, res.termination)
    L.acm_set_tuning(_lib.TUNE_LM_HOST_RESULT, -1)
    default = "host2"  # lm_host_result() for -1 (csrc/acm.hip)
    wall = by_mode[default]
    ref = params["host2"]
    print(json.dumps({"what": "LM loop overhead", "points": n, "lm_wall_ms": round(wall, 3),
                      "default_mode": default,
                      "lm_wall_ms_by_mode": {k: round(v, 3) for k, v in by_mode.items()},
                      "same_iterates_as_host2": {k: v == ref for k, v in params.items()},
                      "evaluations": res.evaluations, "iterations": res.iterations,
                      "ne_ms": round(ne_ms, 4),
                      "overhead_per_eval_ms": {k: round((v - res.evaluations * ne_ms)
                                                        / res.evaluations, 4)
                                               for k, v in by_mode.items()}}))


def probe_radtan_tail(argv):
    """RadTan unproject on BASELINE config 4's own pixels (6.25M synthetic points
    projected by the sample camera, NaN for failed projections): where does the
    time go?  Times acm_unproject on (a) all pixels, (b) the finite ones, (c) the
    finite ones minus the ~0.01% whose reference Newton loop never converges
    (100 steps, NumericalError), each resized to the same count by repeating,
    plus the fraction of such pixels and of 128-pixel waves holding one.

      python tools/probes.py radtan_tail [--points N]"""
    ap = argparse.ArgumentParser(prog="probes.py radtan_tail")
    ap.add_argument("--points", type=int, default=6_250_000)
    ap.add_argument("--offset", type=int, default=3,
                    help="synthetic shard (rank) index: points seeded at offset * points")
    a = ap.parse_args(argv)
    import torch
    from apex_camera_models import _lib, samples
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    L = _lib.load()
    params, (w, h) = samples.SAMPLES[1]
    m = MODEL_CLASSES["rad_tan"]._from_params(list(params), Resolution(w, h))
    n = a.points
    pts = samples.synthetic_points_device(n, offset=a.offset * n)
    uv, st, _ = m.project_batch(pts)
    cam = m.acm_camera()
    sh = torch.cuda.current_stream().cuda_stream

    def timed(px, flag=0):
        k = px.shape[0]
        ray = torch.empty((k, 3), dtype=torch.float64, device="cuda")
        s2 = torch.empty((k,), dtype=torch.uint8, device="cuda")
        # >= 50 ms of calls first: the clocks ramp over milliseconds, and a
        # 3-call warm-up (r03 and earlier) timed the first set measured slow
        torch.cuda.synchronize()
        t0, w = time.perf_counter(), 0
        while w < 3 or time.perf_counter() - t0 < 0.05:
            L.acm_unproject(ctypes.byref(cam), k, px.data_ptr(), ray.data_ptr(), flag,
                            s2.data_ptr(), sh)
            torch.cuda.synchronize()
            w += 1
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                L.acm_unproject(ctypes.byref(cam), k, px.data_ptr(), ray.data_ptr(), flag,
                                s2.data_ptr(), sh)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 5)
        return best, s2

    def fill(px):  # repeat to n pixels
        r = (n + px.shape[0] - 1) // px.shape[0]
        return px.repeat(r, 1)[:n].contiguous()

    fin = torch.isfinite(uv).all(1)
    px_f = fill(uv[fin])
    t_all, s_all = timed(uv)
    t_fin, s_fin = timed(px_f)
    t_all = min(t_all, timed(uv)[0])  # again after the finite set (interleaved)
    bad = s_fin == 4
    px_c = fill(px_f[~bad])
    t_conv, _ = timed(px_c)
    waves = bad[: (n // 128) * 128].reshape(-1, 128).any(1).float().mean().item()
    gb = 41 * n / 1e9
    print(json.dumps({
        "what": "RadTan unproject on config-4 pixels", "points": n, "shard": a.offset,
        "nonconverging_pixels": int(bad.sum()),
        "nan_fraction": float((~fin).float().mean()),
        "nonconverging_fraction_of_finite": float(bad.float().mean()),
        "waves128_with_nonconverging": waves,
        "ms_all": round(t_all, 4), "TBps_all": round(gb / t_all, 2),
        "ms_finite": round(t_fin, 4), "TBps_finite": round(gb / t_fin, 2),
        "ms_converging": round(t_conv, 4), "TBps_converging": round(gb / t_conv, 2)}))


def probe_reproj_ceiling(argv):
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

      python tools/probes.py reproj_ceiling [--libs a.so,b.so] [--only real,probe]"""
    ap = argparse.ArgumentParser(prog="probes.py reproj_ceiling")
    ap.add_argument("--cells", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--libs", default="apex-camera-models_amd/lib/libacm.so")
    ap.add_argument("--only", default="real,probe")
    ap.add_argument("--grids", default="1024,2048")
    ap.add_argument("--rt-points", type=int, default=50_000_000)
    a = ap.parse_args(argv)
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
            # (r06) the libraries' results, bit for bit (the result vector,
            # and the per-point errors where the call writes them)
            got = []
            for tag, cs in per_lib:
                res.fill_(0.0)
                cs[name][1]()
                torch.cuda.synchronize()
                got.append((res.clone(), errs.clone() if name.startswith("reproj") else None))
            same = all(torch.equal(g[0].view(torch.int64), got[0][0].view(torch.int64)) and
                       (g[1] is None or torch.equal(g[1].view(torch.int64),
                                                    got[0][1].view(torch.int64)))
                       for g in got[1:])
            emit(name, best, per_lib[0][1][name][0], same_bits=same)
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


def probe_round_trip(argv):
    """Config-4 round trip (acm_project_unproject) A/B over ACM_TUNE_ROUND_TRIP
    settings (points per lane, LDS-staged or direct ray stores): every model at
    the bench leg's 50M points on one GPU, settings interleaved, HIP-event time
    per call (best of --rounds blocks of --reps calls).

      python tools/probes.py round_trip [--points N] [--settings -1,2,10,18,4,12,20]"""
    ap = argparse.ArgumentParser(prog="probes.py round_trip")
    ap.add_argument("--points", type=int, default=50_000_000)
    ap.add_argument("--settings", default="-1,1,2,4,9,10,12,17,18,20")
    ap.add_argument("--models", default="0,1,2,3,4,5")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args(argv)
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    n = a.points
    sh = torch.cuda.current_stream().cuda_stream
    pts = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    rays = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    st2 = torch.empty((n,), dtype=torch.uint8, device="cuda")
    settings = [int(v) for v in a.settings.split(",")]
    for mid in (int(m) for m in a.models.split(",")):
        params, (w, h) = samples.SAMPLES[mid]
        cam = _lib.AcmCamera()
        _lib.check(L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * len(params))(
            *params), len(params), w, h))

        def call():
            _lib.check(L.acm_project_unproject(ctypes.byref(cam), n, pts.data_ptr(), 0,
                                               uv.data_ptr(), st.data_ptr(), rays.data_ptr(),
                                               st2.data_ptr(), sh))
        best = {}
        for _ in range(a.rounds):
            for v in settings:
                L.acm_set_tuning(_lib.TUNE_ROUND_TRIP, v)
                for _ in range(3):
                    call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    call()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                best[v] = min(best.get(v, 1e9), ms)
        L.acm_set_tuning(_lib.TUNE_ROUND_TRIP, -1)
        print(json.dumps({"model": mid, "points": n,
                          "ms": {str(k): round(v, 4) for k, v in best.items()},
                          "TBps_66B": {str(k): round(66 * n / v / 1e9, 2) for k, v in best.items()}}),
              flush=True)


def probe_sample(argv):
    """sample_points A/B of every path (ACM_TUNE_SAMPLE_FUSED): the segment
    two-pass default ("seg"; "seg_nocert" = ACM_TUNE_SAMPLE_CERT 0, every
    segment counted cell by cell; "seg_w1".."seg_w4" = ACM_TUNE_SAMPLE_WRITE),
    the round-1 two-pass count / scan / write path ("two_pass") and the single
    pass with a decoupled look-back ("fused_r2" / "_r4" / "_r8"), the
    speculative segment path ("spec": write in place, repair after a drop), every
    model on the config-5 grid (1e8 requested cells), interleaved in one
    process.  The outputs must be bit-identical.

      python tools/probes.py sample [--cells N]"""
    ap = argparse.ArgumentParser(prog="probes.py sample")
    ap.add_argument("--cells", type=int, default=100_000_000)
    a = ap.parse_args(argv)
    import torch
    from apex_camera_models import _lib, samples, util
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    names = ["pinhole", "rad_tan", "kannala_brandt", "double_sphere", "ucm", "eucm", "fov"]
    L = _lib.load()
    out = {}
    for mid in [int(x) for x in os.environ.get("MODELS", "0,1,2,3,4,5,6").split(",")]:
        params, (w, h) = samples.SAMPLES[mid]
        m = MODEL_CLASSES[names[mid]]._from_params([float(p) for p in params], Resolution(w, h))

        # variant names: seg (default), seg_nocert, seg_w1..seg_w4
        # (ACM_TUNE_SAMPLE_WRITE), two_pass, fused_r2 / r4 / r8
        def run_knobs(v):
            fused = {"two_pass": 0, "fused_r2": 1, "fused_r4": 2, "fused_r8": 3,
                     "spec": 4}.get(v, -1)
            L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, fused)
            L.acm_set_tuning(_lib.TUNE_SAMPLE_CERT, 0 if v == "seg_nocert" else -1)
            L.acm_set_tuning(_lib.TUNE_SAMPLE_WRITE, int(v[-1]) if v.startswith("seg_w") else -1)

        def run(v):
            run_knobs(v)
            return util.sample_points(m, a.cells)

        VS = os.environ.get("VARIANTS", "seg,seg_nocert,two_pass,fused_r4").split(",")
        res = {v: run(v) for v in VS}
        same = all(torch.equal(res[VS[0]][k], res[v][k]) for k in (0, 1) for v in VS)
        kept = int(res[VS[0]][0].shape[0])
        del res
        # timing: the C-ABI call on preallocated buffers (no per-call 4 GB
        # allocation, no host read-back of the count between launches)
        cam = m.acm_camera()
        ncx, ncy = ctypes.c_uint32(), ctypes.c_uint32()
        L.acm_sample_points_grid(cam.width, cam.height, a.cells, ctypes.byref(ncx),
                                 ctypes.byref(ncy))
        cap = ncx.value * ncy.value
        uv = torch.empty((cap, 2), dtype=torch.float64, device="cuda")
        xyz = torch.empty((cap, 3), dtype=torch.float64, device="cuda")
        cnt = torch.zeros((2,), dtype=torch.int64, device="cuda")
        wsb = L.acm_sample_points_workspace_size(ctypes.byref(cam), a.cells)
        ws = torch.empty(((wsb + 7) // 8,), dtype=torch.float64, device="cuda")
        sh = torch.cuda.current_stream().cuda_stream

        def call(v):
            run_knobs(v)
            _lib.check(L.acm_sample_points(ctypes.byref(cam), a.cells, uv.data_ptr(),
                                           xyz.data_ptr(), cnt.data_ptr(), ws.data_ptr(), wsb,
                                           sh))
        cells = {}
        for _ in range(int(os.environ.get("REPS", "3"))):
            for v in VS:
                call(v)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    call(v)
                e1.record()
                torch.cuda.synchronize()
                cells[v] = min(cells.get(v, 1e9), e0.elapsed_time(e1) / 3)
        del uv, xyz, ws
        L.acm_set_tuning(_lib.TUNE_SAMPLE_FUSED, -1)
        L.acm_set_tuning(_lib.TUNE_SAMPLE_CERT, -1)
        L.acm_set_tuning(_lib.TUNE_SAMPLE_WRITE, -1)
        out[mid] = {"kept": kept, "identical": same,
                    **{k: {"ms": round(v, 4), "Gcells_s": round(a.cells / v / 1e6, 1),
                           "out_TBps": round(40 * kept / v / 1e9, 2)}
                       for k, v in cells.items()}}
        print(json.dumps({"model": mid, **out[mid]}), flush=True)
    print(json.dumps({"what": "sample_points paths", "cells": a.cells,
                      "models": out}))


PROBES = {n[len("probe_"):]: f for n, f in sorted(globals().items()) if n.startswith("probe_")}


def main():
    if len(sys.argv) < 2 or sys.argv[1] not in PROBES:
        print(__doc__)
        for n, f in PROBES.items():
            print(f"  {n:16s} {f.__doc__.strip().splitlines()[0]}")
        sys.exit(0 if len(sys.argv) > 1 and sys.argv[1] in ("-h", "--help") else 2)
    PROBES[sys.argv[1]](sys.argv[2:])


if __name__ == "__main__":
    main()
