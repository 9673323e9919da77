"""LM loop overhead on config-3 data (KB-sampled correspondences, DS target):
wall time of acm_lm_optimize vs evaluations x the normal-equation kernel
time, i.e. the host / launch / copy cost per evaluation, for the host loop
with each ACM_TUNE_LM_HOST_RESULT mode (0 copy + sync, 1 pinned + sync, 2
pinned + spin on the completion word, 3 (r06) pre-queued evaluations behind a
host-written doorbell); the reported wall is the default.  Every mode must
take the same iterates (same parameters bit for bit).
(r04 also timed a device-resident loop here; it was removed in r05.)

  python tools/diag_lm.py [--points N]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=10_000_000)
    a = ap.parse_args()
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


if __name__ == "__main__":
    main()
