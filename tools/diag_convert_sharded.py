"""Cost of the sharded conversion path on one GPU: the
config-5 KB -> DS convert() at 1e8 sampled cells, warm, best of --reps,

  none   -- conversion.convert(collective=None): the 1-rank path;
  cells  -- the same with the LM on the cell form (r06, util.CellSample);
  py     -- a 1-rank process group and the torch.distributed callbacks
            (distributed.TorchCollective; before r06: rccl_allreduce);
  rccl   -- a 1-rank RCCL communicator driven from libacm
            (distributed.RcclCollective, no Python per collective),

interleaved round by round.  Prints one JSON line: per mode the convert wall,
the LM's evaluations and the parameters (which must agree bit for bit), and
the per-evaluation overhead of each sharded mode over `none`."""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="none,py,rccl")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, samples, util
    from apex_camera_models import distributed as D
    torch.cuda.set_device(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    uv, xyz, cs = util.sample_points(src, a.cells, cells=True)
    torch.cuda.synchronize()
    colls = {}
    for m in a.modes.split(","):
        if m in ("none", "cells"):
            colls[m] = None
        elif m == "rccl_cells" and hasattr(D, "RcclCollective"):
            colls[m] = D.RcclCollective()
        elif m == "py" and hasattr(D, "TorchCollective"):
            colls[m] = D.TorchCollective()
        elif m == "py":
            colls[m] = "legacy"
        elif m == "rccl" and hasattr(D, "RcclCollective"):
            colls[m] = D.RcclCollective()

    def run(m, c):
        if c == "legacy":
            return conversion.convert(src, "double_sphere", xyz, uv, allreduce=D.rccl_allreduce())
        kw = {"cells": cs} if m.endswith("cells") else {}
        if c is None:
            return conversion.convert(src, "double_sphere", xyz, uv, **kw)
        return conversion.convert(src, "double_sphere", xyz, uv, collective=c, **kw)

    best, info = {}, {}
    for m, c in colls.items():  # cold run: workspaces, communicator warm-up
        run(m, c)
    for _ in range(a.reps):
        for m, c in colls.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            met = run(m, c)
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) * 1e3
            best[m] = min(best.get(m, float("inf")), t)
            info[m] = {"lm_iterations": met.lm_iterations, "params": met.model.params(),
                       "final_mean": met.final_reprojection_error.mean,
                       "final_median": met.final_reprojection_error.median,
                       "initial_median": met.initial_reprojection_error.median,
                       "optimization_ms": round(met.optimization_time_ms, 3)}
    out = {"what": "config-5 convert() on one GPU: 1-rank path vs the sharded path at world 1 "
                   "(ms, warm, best of reps, modes interleaved)",
           "correspondences": int(xyz.shape[0]),
           "convert_ms": {m: round(v, 3) for m, v in best.items()}, "modes": info}
    if "none" in best:
        ref = info["none"]
        for m in best:
            if m == "none":
                continue
            out[f"{m}_over_none_pct"] = round(100 * (best[m] / best["none"] - 1), 2)
            out[f"{m}_same_bits"] = (info[m]["params"] == ref["params"]
                                     and info[m]["final_median"] == ref["final_median"]
                                     and info[m]["initial_median"] == ref["initial_median"])
    print(json.dumps(out), flush=True)
    for c in colls.values():
        if hasattr(c, "close"):
            c.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
