"""Multi-process (gloo, world_size 2 and 3) checks of the sharded path:
every rank's view after the exchange equals the single-process result over
the full batch (the oracle stands in for the per-shard GPU kernels)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from test_oracle import SAMPLES

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
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_worker.py"),
                                       "--out", str(tmp_path)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out, _ = p.communicate(timeout=240)
        assert p.returncode == 0, out.decode()[-3000:]
    return [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]


def test_shard_range_partitions():
    from apex_camera_models.distributed import grid_row_range, shard_range
    for n in (0, 1, 7, 10, 10_000_001):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert grid_row_range(10, 5, 1, 2) == (30, 50)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_matches_single_process(world, tmp_path):
    res = _run(world, tmp_path)
    params, (w, h) = SAMPLES[3]
    rng = np.random.default_rng(5)
    n = 10_007
    xyz = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(-0.5, 4, n)], 1)
    uv0, _, _ = O.project(3, params, w, h, xyz)
    obs = np.where(np.isnan(uv0), 0.0, uv0) + rng.normal(0, 0.5, (n, 2))
    A, g, c, nv = O.normal_equations(3, params, w, h, xyz, obs)
    full = np.concatenate([A.ravel(), g, [c, nv]])
    stats, m = O.reprojection_error(3, params, w, h, xyz, obs)
    for r in res:
        # every rank holds the same summed vector
        np.testing.assert_allclose(r["ne"], full, rtol=1e-12, atol=1e-9)
        assert r["ne"][-1] == nv
        got = dict(zip(("rmse", "min", "max", "mean", "stddev", "n_valid"), r["stats"]))
        assert got["n_valid"] == m
        for k in ("rmse", "mean", "stddev"):
            assert abs(got[k] - stats[k]) <= 1e-12 * abs(stats[k])
        assert got["min"] == stats["min"] and got["max"] == stats["max"]
    assert all(np.array_equal(res[0]["ne"], r["ne"]) for r in res)
    # sample_points: rank-ordered concatenation == serial order, bit-exact
    kp, (kw, kh) = SAMPLES[2]
    uv_s, xyz_s, _ = O.sample_points(2, kp, kw, kh, 20_000)
    uv_c = np.concatenate([r["sp_uv"] for r in res])
    xyz_c = np.concatenate([r["sp_xyz"] for r in res])
    assert np.array_equal(uv_c, uv_s) and np.array_equal(xyz_c, xyz_s)
    offs = [int(r["sp_off"][0]) for r in res]
    assert offs == list(np.cumsum([0] + [len(r["sp_uv"]) for r in res[:-1]]))
    assert all(int(r["sp_off"][1]) == len(uv_s) for r in res)
