"""KB projection / unprojection A/B in one process: the default library (r, 1/r and
the atan2 quotient from v_rsq / v_rcp + Newton) against a build with the
IEEE sqrt / divisions (-DACM_IEEE_MATH: `make -C apex-camera-models_amd ieee`
builds lib/libacm_ieee.so).  Project with and without the Jacobian, 10M points; also the
largest relative difference between the two builds' outputs.  Then KB
unproject (10M pixels, the projections of the bench cloud): the default
library takes 1 / ru and 1 / |p| after the Newton loop from v_rcp / v_rsq +
Newton; the IEEE build divides.

  python tools/diag_fast_math.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    from apex_camera_models import _lib, samples
    libs = {"nr": _lib.load(),
            "ieee": ctypes.CDLL(os.path.join(ROOT, "apex-camera-models_amd", "lib",
                                             "libacm_ieee.so"), mode=os.RTLD_LOCAL)}
    vp = ctypes.c_void_p
    for L in libs.values():
        L.acm_camera_init.argtypes = [ctypes.POINTER(_lib.AcmCamera), ctypes.c_int,
                                      ctypes.POINTER(ctypes.c_double), ctypes.c_size_t,
                                      ctypes.c_uint32, ctypes.c_uint32]
        L.acm_project.argtypes = [ctypes.POINTER(_lib.AcmCamera), ctypes.c_size_t, vp,
                                  ctypes.c_int, vp, vp, vp, vp]
        L.acm_unproject.argtypes = [ctypes.POINTER(_lib.AcmCamera), ctypes.c_size_t, vp, vp,
                                    ctypes.c_int, vp, vp]
    n = 10_000_000
    pts = samples.synthetic_points_device(n)
    sh = torch.cuda.current_stream().cuda_stream

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    for mid in (2,):  # (FOV measured no gain from the same change and keeps IEEE)
        params, (w, h) = samples.SAMPLES[mid]
        P = len(params)
        outs = {k: (torch.empty((n, 2), dtype=torch.float64, device="cuda"),
                    torch.empty((n,), dtype=torch.uint8, device="cuda"),
                    torch.empty((P * n * 2,), dtype=torch.float64, device="cuda")) for k in libs}
        cams = {}
        for k, L in libs.items():
            cam = _lib.AcmCamera()
            assert L.acm_camera_init(ctypes.byref(cam), mid, (ctypes.c_double * P)(*params), P,
                                     w, h) == 0
            cams[k] = cam

        def call(k, wj):
            uv, st, jac = outs[k]
            return libs[k].acm_project(ctypes.byref(cams[k]), n, pts.data_ptr(), 0,
                                       uv.data_ptr(), st.data_ptr(),
                                       jac.data_ptr() if wj else None, sh)

        cells = {}
        for _ in range(8):
            for wj in (True, False):
                for k in libs:
                    key = f"{k}_{'j' if wj else 'noj'}"
                    cells[key] = min(cells.get(key, 1e9), timed(lambda: call(k, wj)))
        for k in libs:
            assert call(k, True) == 0
        torch.cuda.synchronize()
        (a_uv, a_st, a_j), (b_uv, b_st, b_j) = outs["nr"], outs["ieee"]
        ok = (b_st == 0) & torch.isfinite(b_uv).all(dim=1)
        rel_uv = ((a_uv[ok] - b_uv[ok]).abs().max() / b_uv[ok].abs().max()).item()
        jn, jb = a_j.view(P, n, 2)[:, ok], b_j.view(P, n, 2)[:, ok]
        scale = jb.abs().amax(dim=(0, 2)).clamp_min(1e-300)
        rel_j = ((jn - jb).abs().amax(dim=(0, 2)) / scale).max().item()
        print(json.dumps({"what": "projection: rsq/rcp+Newton vs IEEE sqrt/div", "model": mid,
                          "points": n, "ms": {k: round(v, 4) for k, v in cells.items()},
                          "status_identical": bool(torch.equal(a_st, b_st)),
                          "max_rel_uv_diff": rel_uv, "max_rel_jac_diff": rel_j}), flush=True)

        # unprojection of the projected cloud
        uvin = torch.nan_to_num(outs["nr"][0], nan=1.0).contiguous()
        un = {k: (torch.empty((n, 3), dtype=torch.float64, device="cuda"),
                  torch.empty((n,), dtype=torch.uint8, device="cuda")) for k in libs}

        def ucall(k):
            rays, st = un[k]
            return libs[k].acm_unproject(ctypes.byref(cams[k]), n, uvin.data_ptr(),
                                         rays.data_ptr(), 0, st.data_ptr(), sh)

        ucells = {}
        for _ in range(8):
            for k in libs:
                ucells[k] = min(ucells.get(k, 1e9), timed(lambda: ucall(k)))
        for k in libs:
            assert ucall(k) == 0
        torch.cuda.synchronize()
        (ra, sa), (rb, sb) = un["nr"], un["ieee"]
        okr = (sb == 0)
        rel_ray = ((ra[okr] - rb[okr]).abs().max()).item()  # unit rays: absolute = relative
        print(json.dumps({"what": "unprojection: rcp/rsq+Newton tail vs IEEE div/sqrt",
                          "model": mid, "points": n,
                          "ms": {k: round(v, 4) for k, v in ucells.items()},
                          "status_identical": bool(torch.equal(sa, sb)),
                          "max_abs_ray_diff": rel_ray}), flush=True)


if __name__ == "__main__":
    main()
