"""Fused normal equations timed per call, interleaved in one process over
the settings of --forms (values of the r04 experiment knob ACM_TUNE_NE_FORM
= 16, removed after the measurement: profiles/r04b-d_*; with --forms -1 the
default kernel only).
DS on the config-3 (9.29M) and config-5 (92.9M) KB-sampled correspondences
at the DS linear estimate; every model on 10M synthetic points.  Per form:
the fastest of 3 blocks of 20 calls after >= 50 ms of warm-up, GB/s of the
40 B/point read stream, and the largest relative difference from form 0.

  python tools/diag_ne.py [--forms 0,1,2] [--models 0,1,2,3,4,5,6] [--skip-ds]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--forms", default="-1")
    ap.add_argument("--models", default="0,1,2,3,4,5,6")
    ap.add_argument("--skip-ds", action="store_true")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--ntl", default="-1", help="ACM_TUNE_NT_LOADS values to cross with the forms")
    a = ap.parse_args()
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, conversion, factors
    from apex_camera_models import samples, util
    from bench_configs import timed
    L = _lib.load()
    # a form "6:128" = form 6 with ACM_TUNE_NE_RESIDENT_MIB = 128
    forms = [(f, int(t)) for f in a.forms.split(",") for t in a.ntl.split(",")]

    def sweep(tag, f, p, P, n):
        out = torch.empty((P * P + P + 2,), dtype=torch.float64, device="cuda")
        ms, res = {}, {}
        try:
            for _ in range(a.reps):
                for fm, ntl in forms:
                    if fm != "-1":
                        L.acm_set_tuning(16, int(fm.split(":")[0]))  # ACM_TUNE_NE_FORM (r04 exp.)
                    if ":" in fm:
                        L.acm_set_tuning(17, int(fm.split(":")[1]))  # its resident MiB
                    L.acm_set_tuning(_lib.TUNE_NT_LOADS, ntl)
                    key = f"{fm}" if len(a.ntl.split(",")) == 1 else f"{fm}/ntl{ntl}"
                    ms.setdefault(key, []).append(timed(lambda: f.normal_equations(p, out)))
                    res[key] = out.clone()
        finally:
            L.acm_set_tuning(_lib.TUNE_NT_LOADS, -1)
        ref = res[next(iter(res))]
        scale = ref.abs().clamp(min=float(ref.abs().max()) * 1e-6)
        print(json.dumps({
            "what": tag, "points": n,
            "ms": {str(k): round(min(v), 4) for k, v in ms.items()},
            "GBps": {str(k): round(40 * n / min(v) / 1e6, 1) for k, v in ms.items()},
            "n_valid": {str(k): int(r[-1]) for k, r in res.items()},
            "max_rel_diff_vs_first": {str(k): float(((r - ref).abs()[:-1] / scale[:-1]).max())
                                      for k, r in res.items()}}), flush=True)

    if not a.skip_ds:
        kp, (kw, kh) = samples.SAMPLES[2]
        src = KannalaBrandtModel._from_params(kp, Resolution(kw, kh))
        for cells in (10_000_000, 100_000_000):
            uv, xyz = util.sample_points(src, cells)
            ds = conversion._init_target("double_sphere", src)
            ds.linear_estimation(xyz, uv)
            f = factors.DoubleSphereCameraParamsFactor(xyz, uv, Resolution(kw, kh))
            sweep(f"DS normal equations, KB-sampled ({cells} cells)", f, ds.params(), 6,
                  xyz.shape[0])
            del uv, xyz, f
            torch.cuda.empty_cache()
    facs = [factors.PinholeCameraParamsFactor, factors.RadTanCameraParamsFactor,
            factors.KannalaBrandtCameraParamsFactor, factors.DoubleSphereCameraParamsFactor,
            factors.UcmCameraParamsFactor, factors.EucmCameraParamsFactor,
            factors.FovCameraParamsFactor]
    pts = samples.synthetic_points_device(10_000_000)
    pts = pts[torch.isfinite(pts).all(1)].contiguous()
    for mid in [int(m) for m in a.models.split(",")]:
        fcls = facs[mid]
        params, (w, h) = samples.SAMPLES[mid]
        m = fcls.MODEL._from_params(list(params), Resolution(w, h))
        uv, _, _ = m.project_batch(pts)
        obs = torch.nan_to_num(uv, nan=0.0) + 0.25
        f = fcls(pts, obs, Resolution(w, h))
        sweep(f"{fcls.MODEL.__name__} normal equations, synthetic", f, list(params), len(params),
              pts.shape[0])


if __name__ == "__main__":
    main()
