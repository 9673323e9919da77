"""One rank of the multi-process GPU tests (tests/test_gpu_distributed.py).

Every rank drives libacm.so's kernels on cuda:0 over its shard of the
points and exchanges through torch.distributed (gloo: several ranks share
the box's one GPU; on a multi-GPU node the same code runs over RCCL).
Writes what it computed to <out>/rank<r>.npz for the parent to compare with
the single-process oracle / GPU result over the full batch."""
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

from test_oracle import SAMPLES  # noqa: E402


def shard_data():
    """The batch every rank slices (same seed as the parent)."""
    import oracle as O
    params, (w, h) = SAMPLES[3]
    rng = np.random.default_rng(21)
    n = 30_011
    xyz = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(-0.5, 4, n)], 1)
    uv0, _, _ = O.project(3, params, w, h, xyz)
    obs = np.where(np.isnan(uv0), 0.0, uv0) + rng.normal(0, 0.5, (n, 2))
    return params, (w, h), xyz, obs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, util
    from apex_camera_models import distributed as D
    from apex_camera_models.camera import DoubleSphereModel, FovModel, Intrinsics
    out = {}

    # --- reprojection statistics + exact median of the union ---------------
    params, (w, h), xyz, obs = shard_data()
    m = DoubleSphereModel._from_params(params, Resolution(w, h))
    rng_lo, rng_hi = D.shard_range(len(xyz), rank, world)
    if world == 3:  # rank 1 holds an empty shard
        cut = len(xyz) // 2
        rng_lo, rng_hi = {0: (0, cut), 1: (cut, cut), 2: (cut, len(xyz))}[rank]
    p3 = torch.as_tensor(xyz[rng_lo:rng_hi], device="cuda")
    p2 = torch.as_tensor(obs[rng_lo:rng_hi], device="cuda")
    errors = torch.empty((p3.shape[0],), dtype=torch.float64, device="cuda")
    util.reprojection_stats(m, p3, p2, errors)
    st = D.combine_reprojection_stats(errors)
    out["stats"] = np.array([st[k] for k in ("rmse", "min", "max", "mean", "stddev", "n_valid",
                                            "median")])

    # --- FOV linear estimation over sharded correspondences ----------------
    fp, (fw, fh) = SAMPLES[6]
    rng = np.random.default_rng(3)
    nf = 8_003
    fxyz = np.stack([rng.uniform(-1, 1, nf), rng.uniform(-1, 1, nf), rng.uniform(0.5, 4, nf)], 1)
    import oracle as O
    fuv, _, _ = O.project(6, fp[:4] + [1.37], fw, fh, fxyz)
    fuv = np.where(np.isnan(fuv), 0.0, fuv) + rng.normal(0, 0.4, (nf, 2))
    flo, fhi = D.shard_range(nf, rank, world)
    fm = FovModel(Intrinsics(*fp[:4]), Resolution(fw, fh), 1.0)
    D.distributed_fov_linear_estimation(fm, torch.as_tensor(fxyz[flo:fhi], device="cuda"),
                                        torch.as_tensor(fuv[flo:fhi], device="cuda"))
    out["fov_w"] = np.array([fm.w])

    # --- KB -> DS conversion with the LM's normal equations all-reduced ----
    kp, (kw, kh) = SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(kw, kh))
    uv_all, xyz_all = util.sample_points(src, 4000)
    slo, shi = D.shard_range(uv_all.shape[0], rank, world)
    coll = D.TorchCollective()  # gloo ranks share the box's one GPU (RCCL needs one each)
    for tgt in ("double_sphere", "kannala_brandt", "rad_tan", "fov"):
        met = conversion.convert(src, tgt, xyz_all[slo:shi], uv_all[slo:shi], collective=coll)
        out[f"lm_params_{tgt}"] = np.array(met.model.params())
        out[f"lm_iters_{tgt}"] = np.array([met.lm_iterations])
        fe = met.final_reprojection_error
        out[f"lm_err_{tgt}"] = np.array([fe.mean, fe.median, fe.n_valid])
        ie = met.initial_reprojection_error
        out[f"init_err_{tgt}"] = np.array([ie.mean, ie.median, ie.n_valid, ie.min, ie.max])
    # --- (r06) the same conversion on the cell form: each rank's slice of
    # the cells, the sharded opening / LM / final error reading 4-B cells
    uv_c, xyz_c, cs = util.sample_points(src, 4000, cells=True)
    shard_cs = util.CellSample(cells=cs.cells[slo:shi], grid=cs.grid)
    met = conversion.convert(src, "double_sphere", xyz_c[slo:shi], uv_c[slo:shi],
                             collective=coll, cells=shard_cs)
    out["cells_params"] = np.array(met.model.params())
    fe, ie = met.final_reprojection_error, met.initial_reprojection_error
    out["cells_err"] = np.array([met.lm_iterations, fe.mean, fe.median, fe.n_valid, ie.mean,
                                 ie.median, ie.n_valid])
    np.savez(os.path.join(a.out, f"rank{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
