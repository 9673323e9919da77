"""The reference's known-answer tests (tests/golden/reference_kats.json, each
entry citing its /root/reference test), runnable against any backend of
tests/_backends.py.  test_oracle_kats.py runs them on the CPU oracle,
test_gpu_parity.py on the HIP kernels."""
import json
import os

import numpy as np

from _backends import MODEL_IDS, STATUS, parse_params

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))


def run_project_value(be):
    for k in KATS["project_value"]:
        uv, st, _ = be.project(MODEL_IDS[k["model"]], parse_params(k["params"]), *k["res"],
                               [k["point"]], want_jac=False)
        assert st[0] == 0, k["src"]
        assert np.all(np.abs(uv[0] - np.array(k["expect"])) < k["tol"]), k["src"]


def run_project_status(be):
    for k in KATS["project_status"]:
        _, st, _ = be.project(MODEL_IDS[k["model"]], parse_params(k["params"]), *k["res"],
                              [k["point"]], want_jac=False)
        assert st[0] == STATUS[k["status"]], (k["src"], st[0])


def run_project_near_center(be):
    for k in KATS["project_near_center"]:
        p = parse_params(k["params"])
        uv, st, _ = be.project(MODEL_IDS[k["model"]], p, *k["res"], [k["point"]], want_jac=False)
        if st[0] == 0:
            assert abs(uv[0, 0] - p[2]) < k["tol"] and abs(uv[0, 1] - p[3]) < k["tol"], k["src"]
        else:
            assert st[0] == STATUS["PointIsOutSideImage"], k["src"]


def run_project_near_center_if_ok(be):
    for k in KATS["project_near_center_if_ok"]:
        p = parse_params(k["params"])
        uv, st, _ = be.project(MODEL_IDS[k["model"]], p, *k["res"], [k["point"]], want_jac=False)
        if st[0] == 0:
            assert abs(uv[0, 0] - p[2]) < k["tol"] and abs(uv[0, 1] - p[3]) < k["tol"], k["src"]


def run_unproject_status(be):
    for k in KATS["unproject_status"]:
        _, st = be.unproject(MODEL_IDS[k["model"]], parse_params(k["params"]), *k["res"],
                             [k["point"]])
        assert st[0] == STATUS[k["status"]], (k["src"], st[0])


def run_round_trip(be):
    for k in KATS["round_trip"]:
        m, p, (w, h) = MODEL_IDS[k["model"]], parse_params(k["params"]), k["res"]
        pt = np.array(k["point"])
        uv, st, _ = be.project(m, p, w, h, [pt], want_jac=False)
        assert st[0] == 0, k["src"]
        if k.get("finite"):
            assert np.isfinite(uv[0]).all(), k["src"]
        if k.get("in_bounds"):
            assert 0 <= uv[0, 0] < w and 0 <= uv[0, 1] < h, k["src"]
        if "center_tol" in k:
            assert abs(uv[0, 0] - p[2]) < k["center_tol"], k["src"]
            assert abs(uv[0, 1] - p[3]) < k["center_tol"], k["src"]
        ray, st2 = be.unproject(m, p, w, h, uv)
        assert st2[0] == 0, k["src"]
        assert np.all(np.abs(ray[0] - pt / np.linalg.norm(pt)) <= k["tol"]), (k["src"], ray[0])


def run_round_trip_dot(be):
    for k in KATS["round_trip_dot"]:
        m, p, (w, h) = MODEL_IDS[k["model"]], parse_params(k["params"]), k["res"]
        pts = np.array(k["points"])
        uv, st, _ = be.project(m, p, w, h, pts, want_jac=False)
        ok = st == 0
        assert ok.any(), k["src"]
        uvk = uv[ok]
        assert np.all((uvk[:, 0] >= 0) & (uvk[:, 0] < w) & (uvk[:, 1] >= 0) & (uvk[:, 1] < h))
        ray, st2 = be.unproject(m, p, w, h, uvk)
        good = st2 == 0
        assert good.any(), k["src"]
        pn = pts[ok][good]
        pn = pn / np.linalg.norm(pn, axis=1, keepdims=True)
        dots = (pn * ray[good]).sum(1)
        assert np.all(dots > k["min_dot"]), (k["src"], dots)


ALL = [run_project_value, run_project_status, run_project_near_center,
       run_project_near_center_if_ok, run_unproject_status, run_round_trip, run_round_trip_dot]
