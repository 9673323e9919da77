"""The reference's published conversion results (README.md:160-167: KB input
-> DS 0.008 px, UCM 0.145 px, EUCM 0.314 px, RadTan 184.95 px) next to this
engine's, for every target of camera_converter.rs, on the reference's own
setup (KB sample camera samples/kannala_brandt.yaml, sample_points with the
CLI default n = 500, camera_converter.rs:77-79) and at larger n.

Each line: target, n requested / sampled, initial and final mean / rmse
reprojection error (px), LM iterations, termination, wall time.

  python tools/conversions_table.py [--n 500,10000,1000000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)

README = {"double_sphere": 0.008, "ucm": 0.145, "eucm": 0.314, "rad_tan": 184.95}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="500,10000,1000000")
    ap.add_argument("--policy", default="skip,sentinel",
                    help="invalid-point policy of the factor: skip (r = 0, J = 0) and/or "
                         "sentinel (r = (1e6, 1e6), J = 0; doc/COMPREHENSIVE_ANALYSIS.md:116-121)")
    a = ap.parse_args()
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib, conversion, samples, util
    from apex_camera_models.optimizer import LevenbergMarquardtConfig
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    pol = {"skip": _lib.INVALID_SKIP, "sentinel": _lib.INVALID_SENTINEL}
    for policy in a.policy.split(","):
        for n in (int(x) for x in a.n.split(",")):
            uv, xyz = util.sample_points(src, n)
            for t in ("double_sphere", "ucm", "eucm", "rad_tan", "fov"):
                cfg = LevenbergMarquardtConfig()
                cfg.invalid_policy = pol[policy]
                met = conversion.convert(src, t, xyz, uv, config=cfg)
                d = {"target": t, "policy": policy, "n_requested": n,
                     "n_sampled": int(xyz.shape[0]),
                     "initial_mean_px": met.initial_reprojection_error.mean,
                     "final_mean_px": met.final_reprojection_error.mean,
                     "final_rmse_px": met.final_reprojection_error.rmse,
                     "final_median_px": met.final_reprojection_error.median,
                     "lm_iterations": met.lm_iterations, "termination": met.lm_termination,
                     "status": met.convergence_status, "ms": round(met.optimization_time_ms, 2),
                     "params": [round(p, 9) for p in met.model.params()],
                     "readme_final_px": README.get(t)}
                print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
