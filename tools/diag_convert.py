"""Stage breakdown of the config-5 KB -> DS conversion (conversion.convert,
camera_converter.rs:355-488) at 1e8 sampled cells: the initial reprojection
statistics, the linear estimation, the bounded LM, the final reprojection
statistics and the five-pixel validation, each synchronised and timed warm
(one full convert() first), plus the whole convert() wall, cold and warm."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
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


if __name__ == "__main__":
    main()
