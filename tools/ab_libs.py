"""Same-box A/B of two libacm builds on the hot-path calls the BASELINE
configs time: every library is loaded into this one process (ctypes, local
symbols) and the calls alternate between them (in alternating order), best
of --rounds blocks of --reps calls each (HIP events), so box-to-box clock
differences cancel.

  python tools/ab_libs.py --libs tools/build/libacm_r04.so,apex-camera-models_amd/lib/libacm.so

Calls: config 4's round trip (acm_project_unproject, 50M points, six
models), the headline KB project + 2x8 J (acm_project, 10M points) and KB /
RadTan acm_unproject (10M pixels).  Only the C-ABI symbols every round's
library exports are used (acm_camera_init, acm_project, acm_unproject,
acm_project_unproject)."""
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
    ap.add_argument("--libs", required=True)
    ap.add_argument("--rt-points", type=int, default=50_000_000)
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--only", default="round_trip,project,unproject")
    ap.add_argument("--unproject-ppt", default="-1",
                    help="ACM_TUNE_UNPROJECT_PPT values to time acm_unproject at (every library)")
    a = ap.parse_args()
    only = set(a.only.split(","))
    import torch
    from apex_camera_models import _lib, samples  # data generation only
    libs = []
    for path in a.libs.split(","):
        L = ctypes.CDLL(os.path.abspath(path))
        vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.acm_camera_init.argtypes = [vp, ci, vp, ci, ctypes.c_uint32, ctypes.c_uint32]
        L.acm_project.argtypes = [vp, sz, vp, ci, vp, vp, vp, vp]
        L.acm_unproject.argtypes = [vp, sz, vp, vp, ci, vp, vp]
        L.acm_project_unproject.argtypes = [vp, sz, vp, ci, vp, vp, vp, vp, vp]
        L.acm_set_tuning.argtypes = [ci, ci]
        libs.append((os.path.relpath(path, ROOT), L))
    sh = torch.cuda.current_stream().cuda_stream

    def cam_for(L, mid):
        params, (w, h) = samples.SAMPLES[mid]
        cam = _lib.AcmCamera()
        rc = L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * len(params))(*params),
                               len(params), w, h)
        assert rc == 0, rc
        return cam

    def timed_ab(name, units, bytes_per_unit, make_call):
        calls = [(tag, make_call(L)) for tag, L in libs]
        best = {}
        for rnd in range(a.rounds):
            # alternate the order every round: the first library measured after
            # a change of workload reads slow (profiles/r05k_ab_unproject.log vs
            # r05l_ab_unproject.log)
            for tag, fn in (calls if rnd % 2 == 0 else calls[::-1]):
                for _ in range(3):
                    fn()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                best[tag] = min(best.get(tag, 1e9), e0.elapsed_time(e1) / a.reps)
        print(json.dumps({"call": name, "units": units,
                          "ms": {k: round(v, 4) for k, v in best.items()},
                          "TBps": {k: round(bytes_per_unit * units / v / 1e9, 2)
                                   for k, v in best.items()}}), flush=True)

    m = a.rt_points
    pts = samples.synthetic_points_device(m)
    uv = torch.empty((m, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((m,), dtype=torch.uint8, device="cuda")
    rays = torch.empty((m, 3), dtype=torch.float64, device="cuda")
    st2 = torch.empty((m,), dtype=torch.uint8, device="cuda")
    names = {0: "pinhole", 1: "rad_tan", 2: "kannala_brandt", 3: "double_sphere", 4: "ucm",
             5: "eucm"}
    for mid, nm in (names.items() if "round_trip" in only else ()):
        def make(L, mid=mid):
            cam = cam_for(L, mid)
            return lambda: L.acm_project_unproject(ctypes.byref(cam), m, pts.data_ptr(), 0,
                                                   uv.data_ptr(), st.data_ptr(),
                                                   rays.data_ptr(), st2.data_ptr(), sh)
        timed_ab(f"round_trip_{nm}", m, 66, make)
        # every library's outputs, bit for bit (a timing A/B of two builds
        # that must not change results)
        outs = []
        for tag, L in libs:
            make(L)()
            torch.cuda.synchronize()
            outs.append((tag, [t.clone() for t in (uv, st, rays, st2)]))
        same = all(torch.equal(x.view(torch.uint8), y.view(torch.uint8))
                   for _, o in outs[1:] for x, y in zip(outs[0][1], o))
        rec = {"call": f"round_trip_{nm}", "same_bits": same}
        if not same:  # which outputs differ, and the rays by how much
            o0, o1 = outs[0][1], outs[-1][1]
            rec["same_pixels_and_statuses"] = (
                torch.equal(o0[0].view(torch.uint8), o1[0].view(torch.uint8))
                and torch.equal(o0[1], o1[1]) and torch.equal(o0[3], o1[3]))
            f0, f1 = torch.isfinite(o0[2]), torch.isfinite(o1[2])
            rec["same_ray_finiteness"] = torch.equal(f0, f1)
            both = f0 & f1
            rec["max_ray_abs_diff"] = float((o0[2][both] - o1[2][both]).abs().max())
            rec["rays_differing"] = int(((o0[2] != o1[2]) & both).any(1).sum())
        print(json.dumps(rec), flush=True)
        del outs
    del pts, uv, st, rays, st2
    n = a.points
    pts = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((8, n, 2), dtype=torch.float64, device="cuda")

    def make_proj(L):
        cam = cam_for(L, 2)
        return lambda: L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(),
                                     st.data_ptr(), jac.data_ptr(), sh)
    if "project" in only:
        timed_ab("kb_project_jacobian", n, 169, make_proj)
    for mid, nm in (((2, "kb"), (1, "radtan")) if "unproject" in only else ()):
        ref = cam_for(libs[-1][1], mid)
        libs[-1][1].acm_project(ctypes.byref(ref), n, pts.data_ptr(), 0, uv.data_ptr(),
                                st.data_ptr(), None, sh)
        px = torch.nan_to_num(uv, nan=1.0).contiguous()
        r3 = torch.empty((n, 3), dtype=torch.float64, device="cuda")

        def make_un(L, mid=mid):
            cam = cam_for(L, mid)
            return lambda: L.acm_unproject(ctypes.byref(cam), n, px.data_ptr(), r3.data_ptr(), 0,
                                           st.data_ptr(), sh)
        for v in (int(x) for x in a.unproject_ppt.split(",")):
            for _, L in libs:
                L.acm_set_tuning(13, v)  # ACM_TUNE_UNPROJECT_PPT
            timed_ab(f"{nm}_unproject_ppt{v}", n, 41, make_un)
        for _, L in libs:
            L.acm_set_tuning(13, -1)


if __name__ == "__main__":
    main()
