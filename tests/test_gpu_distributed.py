"""Multi-process GPU checks of the sharded path (gloo ranks sharing the box's
one MI355X; the same code runs over RCCL one rank per GPU): every rank's
result after the exchange equals the single-process result over the whole
batch -- reprojection statistics with the distributed exact median, the FOV
grid search, and whole KB -> X conversions (TSQR factors merged across
ranks, LM normal equations all-reduced)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from test_oracle import SAMPLES

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, tmp_path):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_gpu_dist_worker.py"),
                                       "--out", str(tmp_path)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=400)
        outs.append(out)
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out.decode()[-3000:]
    return [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gpu_path_matches_single_process(world, tmp_path):
    import torch
    from _gpu_dist_worker import shard_data
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, util
    from apex_camera_models.camera import FovModel, Intrinsics
    res = _run(world, tmp_path)

    # reprojection statistics + median of the union vs the oracle
    params, (w, h), xyz, obs = shard_data()
    stats, m = O.reprojection_error(3, params, w, h, xyz, obs)
    uvp, stp, _ = O.project(3, params, w, h, xyz)
    d = uvp - obs
    e = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])[stp == 0]
    for r in res:
        got = dict(zip(("rmse", "min", "max", "mean", "stddev", "n_valid", "median"), r["stats"]))
        assert got["n_valid"] == m
        for k in ("rmse", "mean", "stddev"):
            assert abs(got[k] - stats[k]) <= 1e-12 * abs(stats[k])
        assert got["min"] == stats["min"] and got["max"] == stats["max"]
        assert got["median"] == np.median(e)  # exact: radix select over the union

    # FOV grid search over shards == serial reference loop over all points
    fp, (fw, fh) = SAMPLES[6]
    rng = np.random.default_rng(3)
    nf = 8_003
    fxyz = np.stack([rng.uniform(-1, 1, nf), rng.uniform(-1, 1, nf), rng.uniform(0.5, 4, nf)], 1)
    fuv, _, _ = O.project(6, fp[:4] + [1.37], fw, fh, fxyz)
    fuv = np.where(np.isnan(fuv), 0.0, fuv) + rng.normal(0, 0.4, (nf, 2))
    bw, _, _ = O.fov_grid_search(fp[:4] + [1.0], fxyz, fuv)
    assert all(float(r["fov_w"][0]) == bw for r in res)

    # whole conversions: identical on every rank, equal to the 1-GPU run
    kp, (kw, kh) = SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(kw, kh))
    uv_all, xyz_all = util.sample_points(src, 4000)
    for tgt in ("double_sphere", "kannala_brandt", "rad_tan", "fov"):
        ref = conversion.convert(src, tgt, xyz_all, uv_all)
        p0 = res[0][f"lm_params_{tgt}"]
        for r in res:
            assert np.array_equal(r[f"lm_params_{tgt}"], p0)  # ranks agree bit for bit
        np.testing.assert_allclose(p0, ref.model.params(), rtol=1e-8, atol=1e-10)
        # the initial error of the sharded opening (one fused pass per
        # shard, one all-gather, the distributed median) == the 1-GPU one:
        # count, extrema and median exact, the mean to rounding
        for r in res:
            ie = r[f"init_err_{tgt}"]
            ri = ref.initial_reprojection_error
            assert ie[2] == ri.n_valid and ie[1] == ri.median
            assert ie[3] == ri.min and ie[4] == ri.max
            assert abs(ie[0] - ri.mean) <= 1e-12 * ri.mean
        fe = res[0][f"lm_err_{tgt}"]
        assert fe[2] == ref.final_reprojection_error.n_valid
        # the sharded sums round differently (~1e-16 relative); RadTan fitted
        # to this 180-degree fisheye is ill-conditioned (half the points fail
        # to project, mean error 34 px): parameters that agree to 1e-8 (the
        # check above) move the mean error by 4e-6 .. 1.3e-5 relative (runs
        # r03, r03h), so its check is 1e-4; the other targets 1e-5
        tol = 1e-4 if tgt == "rad_tan" else 1e-5
        assert abs(fe[0] - ref.final_reprojection_error.mean) <= \
            tol * ref.final_reprojection_error.mean + 1e-12

    # (r06) the sharded conversion on the cell form: every rank the same
    # bits, the pixel-form sharded run's parameters (the same sums: the cell
    # kernels rebuild the pixels exactly), and the 1-GPU run's to rounding
    ref = conversion.convert(src, "double_sphere", xyz_all, uv_all)
    for r in res:
        assert np.array_equal(r["cells_params"], res[0]["cells_params"])
        assert np.array_equal(r["cells_err"], res[0]["cells_err"])
        assert np.array_equal(r["cells_params"], r["lm_params_double_sphere"])
    np.testing.assert_allclose(res[0]["cells_params"], ref.model.params(), rtol=1e-8,
                               atol=1e-10)
    ce = res[0]["cells_err"]
    assert ce[3] == ref.final_reprojection_error.n_valid
    assert ce[6] == ref.initial_reprojection_error.n_valid
    assert ce[5] == ref.initial_reprojection_error.median
    torch.cuda.synchronize()
