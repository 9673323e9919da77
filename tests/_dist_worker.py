"""One rank of the world_size>1 gloo tests (tests/test_distributed.py).

Runs the exchange logic of apex_camera_models.distributed with the CPU
oracle as the local (per-shard) evaluator and writes what it computed to
<out>/rank<r>.npz for the parent to compare against the single-process
oracle over the full batch.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "apex-camera-models_amd"), HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle as O  # noqa: E402
from apex_camera_models import distributed as D  # noqa: E402
from test_oracle import SAMPLES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    out = {}

    # --- normal equations: DS factor over a sharded 10k-point batch --------
    params, (w, h) = SAMPLES[3]
    rng = np.random.default_rng(5)
    n = 10_007
    xyz = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(-0.5, 4, n)], 1)
    uv0, st, _ = O.project(3, params, w, h, xyz)
    obs = np.where(np.isnan(uv0), 0.0, uv0) + rng.normal(0, 0.5, (n, 2))
    lo, hi = D.shard_range(n, rank, world)
    A, g, c, nv = O.normal_equations(3, params, w, h, xyz[lo:hi], obs[lo:hi])
    vec = torch.tensor(np.concatenate([A.ravel(), g, [c, nv]]), dtype=torch.float64)
    D.allreduce_normal_equations(vec)
    out["ne"] = vec.numpy()

    # --- reprojection statistics -------------------------------------------
    uvp, stp, _ = O.project(3, params, w, h, xyz[lo:hi])
    d = uvp - obs[lo:hi]
    e = np.sqrt(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1])
    e[stp != 0] = np.nan
    stats = D.combine_reprojection_stats(torch.tensor(e))
    out["stats"] = np.array([stats[k] for k in ("rmse", "min", "max", "mean", "stddev",
                                                "n_valid")])
    # a shard with no valid error at all (rank 0 here), then every rank's
    # errors NaN: n_valid 0 on every rank, no division by zero
    e_mixed = np.full_like(e, np.nan) if rank == 0 else e
    st_mixed = D.combine_reprojection_stats(torch.tensor(e_mixed))
    out["stats_mixed"] = np.array([st_mixed[k] for k in D.STAT_KEYS])
    st_none = D.combine_reprojection_stats(torch.tensor(np.full(5, np.nan)))
    out["stats_none_n"] = np.array([st_none["n_valid"]])

    # --- sharded sample_points (KB, 20k cells) ----------------------------
    kp, (kw, kh) = SAMPLES[2]
    nreq = 20_000
    ncx = int(round(np.sqrt(nreq * (kw / kh))))
    ncy = int(round(np.sqrt(nreq * (kh / kw))))
    cw, ch = kw / ncx, kh / ncy

    def local_fn(c0, c1):
        cells = np.arange(c0, c1)
        i, j = cells // ncx, cells % ncx
        pix = np.stack([(j + 0.5) * cw, (i + 0.5) * ch], 1)
        ray, s = O.unproject(2, kp, kw, kh, pix)
        keep = (s == 0) & (ray[:, 2] > 0)
        return torch.tensor(pix[keep]), torch.tensor(ray[keep])

    uv_l, xyz_l, off, total = D.sharded_sample_points(ncx, ncy, rank, world, local_fn)
    out["sp_uv"] = uv_l.numpy()
    out["sp_xyz"] = xyz_l.numpy()
    out["sp_off"] = np.array([off, total])
    np.savez(os.path.join(a.out, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
