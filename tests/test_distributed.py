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


def test_reprojection_stats_merge_c_abi():
    """acm_reprojection_stats_merge (host code of libacm.so): merging the
    shard statistics of a split batch equals the statistics of the whole."""
    import ctypes
    import torch
    from apex_camera_models import _lib
    from apex_camera_models.distributed import local_reprojection_result
    rng = np.random.default_rng(3)
    e = np.abs(rng.normal(1.0, 0.7, 100_003))
    e[rng.random(e.size) < 0.05] = np.nan
    whole = local_reprojection_result(e).numpy()
    for cuts in ([50_000], [0, 10, 99_990], [33_333, 66_666]):
        parts = np.concatenate([local_reprojection_result(c).numpy()[None]
                                for c in np.split(e, cuts)])
        out = (ctypes.c_double * 8)()
        rc = _lib.load().acm_reprojection_stats_merge(
            len(parts), parts.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), out)
        assert rc == 0
        got = np.array(list(out))
        assert got[5] == whole[5] and got[1] == whole[1] and got[2] == whole[2]
        np.testing.assert_allclose(got, whole, rtol=1e-12)
    out = (ctypes.c_double * 8)()
    none = np.array([[np.nan, np.inf, -np.inf, np.nan, np.nan, 0, 0, 0]], dtype=np.float64)
    assert _lib.load().acm_reprojection_stats_merge(
        1, none.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), out) == 0
    assert out[5] == 0.0 and np.isnan(out[0])


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
    # ranks agree bit for bit on the merged statistics (one all-gather +
    # libacm's rank-ordered Chan merge), also with an all-NaN shard on rank 0
    assert all(np.array_equal(res[0]["stats"], r["stats"]) for r in res)
    assert all(np.array_equal(res[0]["stats_mixed"], r["stats_mixed"], equal_nan=True)
               for r in res)
    lo, hi = 0, (n + world - 1) // world  # rank 0's shard is excluded in stats_mixed
    st2, m2 = O.reprojection_error(3, params, w, h, xyz[hi:], obs[hi:])
    got2 = dict(zip(("rmse", "min", "max", "mean", "stddev", "n_valid"), res[0]["stats_mixed"]))
    assert got2["n_valid"] == m2
    for k in ("rmse", "mean", "stddev"):
        assert abs(got2[k] - st2[k]) <= 1e-12 * abs(st2[k])
    assert all(int(r["stats_none_n"][0]) == 0 for r in res)
    # sample_points: rank-ordered concatenation == serial order, bit-exact
    kp, (kw, kh) = SAMPLES[2]
    uv_s, xyz_s, _ = O.sample_points(2, kp, kw, kh, 20_000)
    uv_c = np.concatenate([r["sp_uv"] for r in res])
    xyz_c = np.concatenate([r["sp_xyz"] for r in res])
    assert np.array_equal(uv_c, uv_s) and np.array_equal(xyz_c, xyz_s)
    offs = [int(r["sp_off"][0]) for r in res]
    assert offs == list(np.cumsum([0] + [len(r["sp_uv"]) for r in res[:-1]]))
    assert all(int(r["sp_off"][1]) == len(uv_s) for r in res)


def test_rccl_setup_fails_on_every_rank():
    """RcclCollective's set-up agrees across ranks: when librccl is missing
    on one rank, every rank raises before the RCCL rendezvous (so
    make_collective falls back on all of them together) instead of the
    others blocking in it (gloo, 2 ranks)."""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                   WORLD_SIZE="2", OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable,
                                       os.path.join(HERE, "_rccl_consensus_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out, _ = p.communicate(timeout=120)
        assert p.returncode == 0, out.decode()[-3000:]
        assert b"raised" in out

