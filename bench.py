"""Benchmark of the hot path: Kannala-Brandt project + dense 2x8 parameter
Jacobian over 10M f64 points per GPU (BASELINE.json configs[1], the config
the metric is quoted on).

One step = one pass of acm_project (the C-ABI of libacm.so) over the resident
10M-point batch: reads xyz (24 B/pt), writes uv (16 B), status (1 B) and the
2N x 8 column-major Jacobian (128 B) = 169 B/pt algorithmic traffic.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Multi-GPU: one process per GPU, each rank projects its own 10M-point shard
(weak scaling, disjoint seeded shards, no data-path collective -- the path is
a pure per-point map); timing is barrier + synchronize on both sides and the
max over ranks.  rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level table)
BYTES_PER_POINT = {  # algorithmic bytes / point for project (+J), SURVEY.md §8(d)
    ("kb", True): 24 + 16 + 1 + 16 * 8, ("kb", False): 24 + 16 + 1,
}
MODELS = {"pinhole": 0, "radtan": 1, "kb": 2, "ds": 3, "ucm": 4, "eucm": 5, "fov": 6}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--points", type=int, default=10_000_000, help="points per GPU")
    ap.add_argument("--model", default="kb", choices=sorted(MODELS))
    ap.add_argument("--layout", default="aos", choices=["aos", "soa"])
    ap.add_argument("--no-jacobian", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(model_id, params, w, h, n, seconds):
    """Oracle (C restatement of the reference's single-threaded per-point
    Rust loop) timed on this host, 1 thread, on the same 10M-point workload,
    repeated until `seconds` of CPU work; median throughput."""
    import numpy as np

    import oracle
    from apex_camera_models import samples
    pts = samples.synthetic_points(n)
    P = oracle.NUM_PARAMS[model_id]
    uv = np.empty((n, 2))
    st = np.empty(n, dtype=np.uint8)
    jac = np.empty((P, n, 2))
    L = oracle.lib()
    dp = oracle._dp
    pa = np.ascontiguousarray(params, dtype=np.float64)
    rates, t_total = [], 0.0
    while t_total < seconds or len(rates) < 3:
        t0 = time.perf_counter()
        L.oracle_project_batch(model_id, dp(pa), w, h, n, dp(pts), dp(uv), oracle._u8p(st),
                               dp(jac))
        dt = time.perf_counter() - t0
        t_total += dt
        rates.append(n / dt / 1e6)
        if len(rates) >= 60:
            break
    rates.sort()
    return {"value": rates[len(rates) // 2], "unit": "Mpoints/s", "cores": 1, "kind": "port",
            "sample": f"{len(rates)} x full {n}-point batch (project + 2x{P} J), "
                      f"{t_total:.1f} s of CPU work, median; oracle/acm_oracle.c -O2 "
                      f"-ffp-contract=off, 1 thread"}


def host_threads():
    """CPU threads this process may use: its affinity set, capped at 16 (the
    GPU box's per-GPU CPU share; os.cpu_count() there shows the whole host)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(16, avail))


def cpu_baseline_all_cores(model_id, params, w, h, n, seconds, threads):
    """The same oracle loop on `threads` host threads (disjoint contiguous
    chunks of the 10M-point batch, each with its own output buffers; ctypes
    drops the GIL for the C call), SURVEY.md §8(d)'s "and with all host
    cores" leg.  Median throughput of whole-batch passes."""
    import threading

    import numpy as np

    import oracle
    from apex_camera_models import samples
    pts = samples.synthetic_points(n)
    P = oracle.NUM_PARAMS[model_id]
    L = oracle.lib()
    dp = oracle._dp
    pa = np.ascontiguousarray(params, dtype=np.float64)
    bounds = [(n * t // threads, n * (t + 1) // threads) for t in range(threads)]
    bufs = []
    for s, e in bounds:
        m = e - s
        bufs.append((np.ascontiguousarray(pts[s:e]), np.empty((m, 2)),
                     np.empty(m, dtype=np.uint8), np.empty((P, m, 2))))

    def work(t):
        x, uv, st, jac = bufs[t]
        L.oracle_project_batch(model_id, dp(pa), w, h, len(x), dp(x), dp(uv),
                               oracle._u8p(st), dp(jac))

    rates, t_total = [], 0.0
    while t_total < seconds or len(rates) < 3:
        ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t0
        t_total += dt
        rates.append(n / dt / 1e6)
        if len(rates) >= 200:
            break
    rates.sort()
    return {"value": rates[len(rates) // 2], "unit": "Mpoints/s", "cores": threads,
            "kind": "port",
            "sample": f"{len(rates)} x full {n}-point batch (project + 2x{P} J) split over "
                      f"{threads} threads, {t_total:.1f} s wall, median; same oracle build"}


def load_traffic(workload, n):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this
    exact workload (profiles/*pmc*.json, written by profiles/collect_pmc.py),
    else None."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload and int(d.get("points", -1)) == n:
            best = d
    return best


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for a 1-GPU box (never set by the driver): run every
    # rank on device 0 and/or use gloo for the timing barrier/all-reduce.
    if os.environ.get("ACM_BENCH_SAME_DEVICE") == "1":
        local = 0
    backend = os.environ.get("ACM_BENCH_BACKEND", "nccl")
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from apex_camera_models import _lib, samples
    L = _lib.load()
    model_id = MODELS[a.model]
    params, (w, h) = samples.SAMPLES[model_id]
    P = len(params)
    want_j = not a.no_jacobian
    n = a.points
    lay = _lib.LAYOUT_SOA if a.layout == "soa" else _lib.LAYOUT_AOS

    cam = _lib.AcmCamera()
    arr = (ctypes.c_double * P)(*params)
    _lib.check(L.acm_camera_init(ctypes.byref(cam), model_id, arr, P, w, h))

    pts = samples.synthetic_points_device(n, offset=rank * n, layout=a.layout)
    uv = torch.empty((n, 2), dtype=torch.float64, device=dev)
    st = torch.empty((n,), dtype=torch.uint8, device=dev)
    jac = torch.empty((P, n, 2), dtype=torch.float64, device=dev) if want_j else None
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    jp = jac.data_ptr() if want_j else None

    def step():
        rc = L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), lay, uv.data_ptr(),
                           st.data_ptr(), jp, sh)
        if rc:
            _lib.check(rc)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()

    # One HIP event pair on the launch stream around the K back-to-back
    # launches: the average launch duration includes the (sub-microsecond)
    # gaps between launches, so `achieved` is conservative.  An event pair
    # around every launch put ~5 us of extra gap between launches (wall
    # 0.2499 vs 0.2433 ms per step, profiles/r01s8_diag_bench_gaps.log).
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / a.steps

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64,
                     device=dev if backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    ms_per_step = elapsed * 1e3 / a.steps
    total_points = n * world
    value = total_points / (ms_per_step / 1e3) / 1e6

    if rank == 0:
        bpp = 24 + 16 + 1 + (16 * P if want_j else 0)
        achieved = bpp * n / (kern_ms / 1e3) / 1e9
        workload = (f"{a.model}_project{'_jacobian' if want_j else ''}_f64_"
                    f"{a.layout}")
        pmc = load_traffic(workload, n)
        traffic = pmc["hbm_bytes_per_launch"] if pmc else None
        res = {
            "metric": "Mpoints/sec project+Jacobian (KB, f64) at 1/2/4/8 GPU; % HBM roofline",
            "value": round(value, 2),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seed 20251205 Philox on device; x,y~U[-1,1), z~U[0.5,4), "
                    "0.1% edge points)",
            "config": {"workload": workload, "points_per_gpu": n, "global_points": total_points,
                       "model_params": "samples/kannala_brandt.yaml" if a.model == "kb"
                       else a.model, "jacobian_layout": "2N x P column-major (nalgebra DMatrix)",
                       "parallelism": f"shard{world} (independent per-rank point batches)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "algorithmic_bytes_per_launch": bpp * n,
                         "kernel_ms": round(kern_ms, 5)},
        }
        if not a.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
            res["cpu_baseline"] = cpu_baseline(model_id, params, w, h, n,
                                               a.cpu_baseline_seconds)
            thr = host_threads()
            if thr > 1:
                res["cpu_baseline_all_cores"] = cpu_baseline_all_cores(
                    model_id, params, w, h, n, a.cpu_baseline_seconds / 2, thr)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
