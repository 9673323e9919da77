"""BASELINE.json configs 4 and 5 as multi-GPU runs (one process per GPU):

  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port 29511 tools/bench_multi.py [--configs 4,5]

Config 4: all six models, project -> unproject round trip over 50M points in
total (strong scaling: 50M / N per rank), the round-trip error sum of
squares and valid count all-reduced over RCCL.
Config 5: KB -> DS conversion on ~1e8 sampled correspondences: grid rows of
sample_points sharded over the ranks, then the sharded conversion (merged
TSQR factors, all-reduced LM normal equations, distributed median).

Times are max over ranks with a barrier + device sync on both sides.  One
JSON line per measurement from rank 0.  Without torchrun it runs as N = 1.
ACM_BENCH_BACKEND=gloo / ACM_BENCH_SAME_DEVICE=1 rehearse several ranks on
one GPU (correctness of the exchange only; the timings then share a GPU).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)

MODELS = {0: "pinhole", 1: "rad_tan", 2: "kannala_brandt", 3: "double_sphere", 4: "ucm",
          5: "eucm"}


class Ctx:
    def __init__(self):
        import torch
        import torch.distributed as dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if os.environ.get("ACM_BENCH_SAME_DEVICE") == "1":
            local = 0
        torch.cuda.set_device(local)
        self.dist = None
        if self.world > 1:
            backend = os.environ.get("ACM_BENCH_BACKEND", "nccl")
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(backend)
            self.dist = dist

    def sync(self):
        import torch
        if self.dist:
            self.dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(self, v):
        import torch
        if not self.dist:
            return v
        t = torch.tensor([v], dtype=torch.float64, device="cuda")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t)

    def sum_over_ranks(self, t):
        if self.dist:
            self.dist.all_reduce(t)
        return t

    def emit(self, d):
        if self.rank == 0:
            d["n_gpus"] = self.world
            print(json.dumps(d), flush=True)

    def close(self):
        if self.dist:
            self.dist.barrier()
            self.dist.destroy_process_group()


def timed(ctx, fn, reps=10):
    fn()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.sync()
    return ctx.max_over_ranks((time.perf_counter() - t0) / reps * 1e3)


def config4(ctx, n_total):
    import torch
    from apex_camera_models import _lib, samples
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    from apex_camera_models.distributed import shard_range
    lo, hi = shard_range(n_total, ctx.rank, ctx.world)
    n = hi - lo
    pts = samples.synthetic_points_device(n, offset=lo)
    L = _lib.load()
    sh = torch.cuda.current_stream().cuda_stream
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    ray = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    st2 = torch.empty((n,), dtype=torch.uint8, device="cuda")
    finite = torch.isfinite(pts).all(1)
    pn = pts / torch.linalg.norm(pts, dim=1, keepdim=True)
    for mid, name in MODELS.items():
        params, (w, h) = samples.SAMPLES[mid]
        cam = MODEL_CLASSES[name]._from_params(params, Resolution(w, h)).acm_camera()

        def rt():
            _lib.check(L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(),
                                     st.data_ptr(), None, sh))
            _lib.check(L.acm_unproject(ctypes.byref(cam), n, uv.data_ptr(), ray.data_ptr(), 0,
                                       st2.data_ptr(), sh))

        ms = timed(ctx, rt)
        ok = (st == 0) & (st2 == 0) & finite
        err = torch.linalg.norm(ray - pn, dim=1)
        red = torch.stack([torch.where(ok, err * err, torch.zeros_like(err)).sum(),
                           ok.sum().to(torch.float64)])
        ctx.sum_over_ranks(red)  # the RCCL residual all-reduce of config 4
        ctx.emit({"config": 4, "model": name, "points_total": n_total, "points_per_rank": n,
                  "round_trip_ms": round(ms, 4),
                  "round_trip_Mpoints_per_s": round(n_total / ms / 1e3, 1),
                  "round_trip_ok": int(red[1]), "sum_sq_round_trip_err": float(red[0])})


def config5(ctx, n_cells):
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, samples
    from apex_camera_models import distributed as D
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    ncx = int(round((n_cells * (w / h)) ** 0.5))
    ncy = int(round((n_cells * (h / w)) ** 0.5))
    fn = D.gpu_sample_points_range(src, n_cells)
    fn(0, min(ncx * ncy, 4096))  # warm-up (module load, workspace)
    ctx.sync()
    t0 = time.perf_counter()
    if ctx.dist:
        uv, xyz, off, total = D.sharded_sample_points(ncx, ncy, ctx.rank, ctx.world, fn)
    else:
        uv, xyz = fn(0, ncx * ncy)
        total = int(uv.shape[0])
    ctx.sync()
    t_s = ctx.max_over_ranks(time.perf_counter() - t0)
    allreduce = D.rccl_allreduce() if ctx.dist else None
    t0 = time.perf_counter()
    met = conversion.convert(src, "double_sphere", xyz, uv, allreduce=allreduce)
    ctx.sync()
    t_c = ctx.max_over_ranks(time.perf_counter() - t0)
    ctx.emit({"config": 5, "what": "KB->DS sharded conversion", "requested": n_cells,
              "correspondences_total": total, "correspondences_rank0": int(uv.shape[0]),
              "sample_points_s": round(t_s, 4), "convert_s": round(t_c, 4),
              "lm_iterations": met.lm_iterations, "termination": met.lm_termination,
              "final_mean_px": met.final_reprojection_error.mean,
              "final_median_px": met.final_reprojection_error.median,
              "ds_params": met.model.params()})
    del uv, xyz
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="4,5")
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    ctx = Ctx()
    cs = a.configs.split(",")
    if "4" in cs:
        config4(ctx, int(50_000_000 * a.scale))
    if "5" in cs:
        config5(ctx, int(100_000_000 * a.scale))
    ctx.close()


if __name__ == "__main__":
    main()
