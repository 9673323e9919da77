"""Benchmark of the hot path: Kannala-Brandt project + dense 2x8 parameter
Jacobian, 10M f64 points (BASELINE.json configs[1], the config the metric
is quoted on).

One step = one pass of acm_project (the C-ABI of libacm.so) over the resident
batch: reads xyz (24 B/pt), writes uv (16 B), status (1 B) and the 2N x 8
column-major Jacobian (128 B) = 169 B/pt algorithmic traffic.

  python bench.py [--gpus N --steps K --warmup W] [--scaling weak|strong]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Launch: under a launcher (torchrun sets WORLD_SIZE) every process is one
rank and --gpus must equal WORLD_SIZE (else exit 2).  Without one,
`bench.py --gpus N` (N > 1) starts its own N rank processes before importing
torch (launch_ranks) and exits non-zero if any of them fails.

Multi-GPU: one process per GPU.  --scaling weak (default): each rank
projects its own --points batch (disjoint seeded shards; total work grows
with N).  --scaling strong: --points is the GLOBAL batch, split into
contiguous shards (distributed.shard_range: 10M -> 1.25M per rank at 8 GPUs).
The path is a pure per-point map, so the timed steps have no data-path
collective; at N > 1 the line also carries the other scaling mode measured
in the same run, and the north-star collective -- one RCCL all-reduce of
(sum ||r||^2, n_valid) of a residual pass over each rank's shard -- timed on
its own.  Timing is barrier + synchronize on both sides and the max over
ranks; rank 0 prints ONE JSON line.

Robustness (r05): the process group is created with a bounded timeout and
every phase (init, the device census, the timed steps, each collective,
each BASELINE leg) runs under a per-rank watchdog (ACM_BENCH_TIMEOUT, 120 s
default): a rank that hangs exits 124 naming its rank, LOCAL_RANK and
device, and the launcher stops the others.  The line records every rank's
device (`ranks_devices`).  A BASELINE leg that raises is reported as
{"error": ...} in its sub-object; the headline line is printed regardless.
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
IC_BYTES = 256 << 20  # MI355X Infinity Cache (MI355X_MICROARCH.md)
RT_BYTES_PER_POINT = 24 + 16 + 1 + 24 + 1  # config 4's one-pass round trip


def roofline_block(bytes_per_launch, input_bytes_per_launch, kernel_ms):
    """Roofline of a sub-measurement: algorithmic bytes
    per launch / its time against the HBM peak.  When everything a launch
    touches fits the 256 MiB Infinity Cache (the strong-scaling shards at
    N = 8: 1.25M KB points, 211 MB), back-to-back launches are served partly
    from it: bound "effective (Infinity Cache)", not "hbm".  When only the
    re-read inputs fit (config 4's 6.25M-point shards at N = 8: 150 MB of
    input, 412 MB in all) the bound stays "hbm" and input_fits_infinity_cache
    says the reads may be cache-assisted."""
    ic = bytes_per_launch < IC_BYTES
    out = {"bound": "effective (Infinity Cache)" if ic else "hbm",
           "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "algorithmic_bytes_per_launch": int(bytes_per_launch),
           "input_bytes_per_launch": int(input_bytes_per_launch),
           "input_fits_infinity_cache": bool(input_bytes_per_launch < IC_BYTES),
           "achieved": None, "frac": None, "kernel_ms": kernel_ms}
    if kernel_ms:
        a = bytes_per_launch / (kernel_ms / 1e3) / 1e9
        out["achieved"] = round(a, 1)
        out["frac"] = round(a / HBM_PEAK_GBS, 4)
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--points", type=int, default=10_000_000,
                    help="points per GPU (weak) or in total (strong)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--verify-shards", action="store_true",
                    help="(tests) strong mode: gather every rank's uv/status and compare "
                         "with one projection of the global batch on rank 0")
    ap.add_argument("--model", default="kb", choices=sorted(MODELS))
    ap.add_argument("--layout", default="aos", choices=["aos", "soa"])
    ap.add_argument("--no-jacobian", action="store_true")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--legs", default="4,5",
                    help="BASELINE configs measured after the headline's timed region and "
                         "attached as sub-objects (config4 / config5); 'none' to skip")
    ap.add_argument("--leg4-points", type=int, default=50_000_000,
                    help="config 4: points in total over all ranks (strong scaling)")
    ap.add_argument("--leg5-cells", type=int, default=100_000_000,
                    help="config 5: requested sample_points cells in total")
    ap.add_argument("--leg-steps", type=int, default=10)
    return ap.parse_args()


def cpu_baseline(model_id, params, w, h, n, seconds, opt="O3"):
    """Oracle (C restatement of the reference's single-threaded per-point
    Rust loop) timed on this host, 1 thread, on the same 10M-point workload,
    repeated until `seconds` of CPU work; median throughput.  opt: the
    -O3 -ffp-contract=off build (the planned
    baseline) or the -O2 parity build."""
    import numpy as np

    import oracle
    from apex_camera_models import samples
    pts = samples.synthetic_points(n)
    P = oracle.NUM_PARAMS[model_id]
    uv = np.empty((n, 2))
    st = np.empty(n, dtype=np.uint8)
    jac = np.empty((P, n, 2))
    L = oracle.lib(opt)
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
                      f"{t_total:.1f} s of CPU work, median; oracle/acm_oracle.c -{opt} "
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
    L = oracle.lib("O3")
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
                      f"{threads} threads, {t_total:.1f} s wall, median; -O3 oracle build"}


def lib_sha256():
    import hashlib
    from apex_camera_models import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def load_traffic(workload, n):
    """HBM bytes per launch from a committed rocprofv3 PMC summary of this
    exact workload (profiles/*pmc*.json, profiles/collect_pmc.py), used only
    if it was collected on this very libacm.so (its sha256 is recorded in
    the summary) or on a rebuild of the very same sources and build
    variant; otherwise traffic is null and the source says why.  Among
    several summaries the one matching this library wins, whatever its
    file name.  Returns (bytes or None, source description)."""
    import glob
    cands = []
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") == workload and int(d.get("points", -1)) == n:
            cands.append((p, d))
    if not cands:
        return None, "no PMC summary for this workload"
    sha = lib_sha256()
    for p, d in reversed(cands):
        if d.get("libacm_sha256") == sha:
            return d["hbm_bytes_per_launch"], os.path.relpath(p, ROOT)
    # hipcc output is not byte-reproducible: accept a rebuild of the very
    # same sources (and build recipe), provided the library is newer than
    # every source file (so it was built from them)
    # The source hash ignores compile defines and which library file ran, so
    # the summary must also name this very build variant: the same file name
    # and acm_version() (which lists the defines) -- a counter file from a
    # diagnostic build is never reported for the production library.
    from apex_camera_models import _buildinfo, _lib
    src = _lib.source_sha256()
    ident = _buildinfo.lib_identity(_lib.LIB_PATH)
    fresh = os.path.getmtime(_lib.LIB_PATH) >= _latest_source_mtime()
    for p, d in reversed(cands):
        if fresh and d.get("libacm_source_sha256") == src and d.get("libacm_identity") == ident:
            return d["hbm_bytes_per_launch"], \
                os.path.relpath(p, ROOT) + " (same libacm sources, rebuilt library)"
    rel = os.path.relpath(cands[-1][0], ROOT)
    return None, f"{rel} was collected on another libacm.so build (stale): not reported"


def _latest_source_mtime():
    import glob
    pkg = os.path.join(ROOT, "apex-camera-models_amd")
    files = glob.glob(os.path.join(pkg, "csrc", "*.hip")) + \
        glob.glob(os.path.join(pkg, "csrc", "*.hpp")) + [os.path.join(ROOT, "include", "acm.h")]
    return max(os.path.getmtime(f) for f in files)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher around it: start N rank
    processes of this same script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT in their environment, torchrun's contract) and
    wait for them.  Runs BEFORE torch is imported: the parent never touches
    the GPU, it only forwards the children's output (rank 0 prints the one
    JSON line) and exits non-zero if any rank fails; a failed rank ends the
    others so a collective cannot hang."""
    import signal
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())

    def die_with_parent():
        # runs in the child between fork and exec (the parent has touched no
        # GPU): PR_SET_PDEATHSIG, so a parent killed outright (SIGKILL from
        # `timeout -k`) still takes its ranks with it
        try:
            ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except Exception:
            pass

    class _Stop(Exception):
        pass

    def on_signal(signum, _frame):
        raise _Stop(signum)

    def signal_all(procs_, sig):
        for q in procs_:
            try:
                os.killpg(q.pid, sig)
            except (ProcessLookupError, PermissionError):
                pass

    # a SIGTERM / SIGINT / SIGHUP to the parent (Ctrl-C, a timeout that
    # signals only the parent's group) is forwarded to every rank's own
    # process group below instead of leaving the ranks orphaned
    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)}
    procs = []
    live = []
    rc = 0
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                       MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
            p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                 env=env, start_new_session=True, preexec_fn=die_with_parent)
            procs.append(p)
            live.append(p)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the "
                          f"other ranks", file=sys.stderr, flush=True)
                    signal_all(live, signal.SIGTERM)
            time.sleep(0.05)
    except _Stop as e:
        sig = e.args[0]
        print(f"bench.py: received signal {sig}; stopping the ranks", file=sys.stderr, flush=True)
        rc = 128 + sig
    finally:
        # whatever ended the loop, no rank outlives the parent: SIGTERM to
        # each rank's process group, SIGKILL after a 5 s grace period
        live = [p for p in procs if p.poll() is None]
        if live:
            signal_all(live, signal.SIGTERM)
            t_end = time.time() + 5.0
            while time.time() < t_end and any(p.poll() is None for p in live):
                time.sleep(0.05)
            signal_all([p for p in live if p.poll() is None], signal.SIGKILL)
            for p in live:
                try:
                    p.wait(timeout=5)
                except subprocess.TimeoutExpired:
                    pass
        for s, h in old.items():
            signal.signal(s, h)
    return rc


class PhaseWatchdog:
    """One per rank: bounds every phase of the run (process-group init, the
    timed steps, each collective, each BASELINE leg) so that a rank stuck in
    an RCCL collective -- e.g. on the first 8-GPU run -- ends the job within
    the bound instead of at the driver's limit, with a message naming the
    rank, its LOCAL_RANK and device ordinal.  A daemon thread polls the
    armed deadline; on expiry it prints and leaves with os._exit(124) (the
    launcher -- launch_ranks or torchrun -- then stops the other ranks)."""

    def __init__(self, rank, local, device, seconds):
        import threading
        self.rank, self.local, self.device, self.seconds = rank, local, device, seconds
        self.phase, self.deadline = None, None
        self._lock = threading.Lock()
        threading.Thread(target=self._run, daemon=True, name="bench-watchdog").start()

    def arm(self, phase, seconds=None):
        with self._lock:
            self.phase = phase
            self.deadline = time.monotonic() + (seconds or self.seconds)

    def disarm(self):
        with self._lock:
            self.phase, self.deadline = None, None

    def who(self):
        return f"rank {self.rank} (LOCAL_RANK {self.local}, device {self.device})"

    def _run(self):
        while True:
            time.sleep(0.25)
            with self._lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                phase = self.phase
            if late:
                print(f"bench.py: {self.who()} did not finish '{phase}' within "
                      f"{self.seconds:.0f} s; exiting", file=sys.stderr, flush=True)
                os._exit(124)


def run_legs(want, runners, wd=None):
    """The BASELINE legs after the headline's timed region: each leg's result,
    or {"error": ...} when it raised -- a failing leg never costs the
    already measured headline line.  runners: [(key, name, fn)]."""
    legs = {}
    for key, name, fn in runners:
        if key not in want:
            continue
        if wd:
            wd.arm(f"leg {name}")
        try:
            legs[name] = fn()
        except Exception as e:  # noqa: BLE001 -- reported in the line
            legs[name] = {"error": f"{type(e).__name__}: {e}"[:500]}
            print(f"bench.py: leg {name} failed: {legs[name]['error']}", file=sys.stderr,
                  flush=True)
    return legs


class LegCtx:
    """What the BASELINE config-4/5 legs need of the run: rank, world, the
    process group (None at N = 1) and the device of the collectives'
    tensors (the GPU under RCCL, the CPU under the gloo rehearsal)."""

    def __init__(self, rank, world, dist, cdev):
        self.rank, self.world, self.dist, self.cdev = rank, world, dist, cdev

    def sync(self):
        import torch
        if self.dist:
            self.dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(self, v):
        import torch
        if not self.dist:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])


LEG4_MODELS = {0: "pinhole", 1: "rad_tan", 2: "kannala_brandt", 3: "double_sphere", 4: "ucm",
               5: "eucm"}


def leg_config4(ctx, n_total, reps):
    """BASELINE config 4: all six models, project -> unproject round trip over
    `n_total` points in total (strong scaling: contiguous shards of one global
    batch), then ONE all-reduce of every model's (sum of squared round-trip
    errors, round-trip-ok count) -- the residual all-reduce of the config.
    A step = the six round trips, one acm_project_unproject launch per model
    (r04: the pixels are written as by acm_project but unprojected from
    registers instead of being read back; the 12-launch form of acm_project +
    acm_unproject is timed beside it as `ms_per_step_two_calls`); the error
    reduction runs after the timed steps, the all-reduce is timed on its own.
    The reference loop this batches: project then unproject per point for
    every model (tests/projection_accuracy.rs, mod.rs:256/271)."""
    import torch
    from apex_camera_models import _lib, samples
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    from apex_camera_models.distributed import shard_range
    lo, hi = shard_range(n_total, ctx.rank, ctx.world)
    n = hi - lo
    dev = torch.device("cuda", torch.cuda.current_device())
    L = _lib.load()
    sh = torch.cuda.current_stream().cuda_stream
    # the global batch, then this rank's contiguous slice (the seeded
    # generator's edge points depend on the batch size, so generating a
    # shard on its own would not give the same points)
    full = samples.synthetic_points_device(n_total)
    pts = full[lo:hi].contiguous()
    del full
    uv = torch.empty((max(n, 1), 2), dtype=torch.float64, device=dev)
    cams, outs = [], []
    for mid, name in LEG4_MODELS.items():
        params, (w, h) = samples.SAMPLES[mid]
        cams.append(MODEL_CLASSES[name]._from_params(params, Resolution(w, h)).acm_camera())
        outs.append((torch.empty((max(n, 1),), dtype=torch.uint8, device=dev),
                     torch.empty((max(n, 1), 3), dtype=torch.float64, device=dev),
                     torch.empty((max(n, 1),), dtype=torch.uint8, device=dev)))

    def one(k):
        cam, (st, ray, st2) = cams[k], outs[k]
        _lib.check(L.acm_project_unproject(ctypes.byref(cam), n, pts.data_ptr(), 0,
                                           uv.data_ptr(), st.data_ptr(), ray.data_ptr(),
                                           st2.data_ptr(), sh))

    def one_two_calls(k):
        cam, (st, ray, st2) = cams[k], outs[k]
        rc = L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(), st.data_ptr(),
                           None, sh)
        rc = rc or L.acm_unproject(ctypes.byref(cam), n, uv.data_ptr(), ray.data_ptr(), 0,
                                   st2.data_ptr(), sh)
        if rc:
            _lib.check(rc)

    def step(f=one):
        for k in range(len(cams)):
            f(k)

    step()
    ctx.sync()
    per_model = []
    for k in range(len(cams)):  # each model's round trip on its own
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            one(k)
        ctx.sync()
        per_model.append(ctx.max_over_ranks((time.perf_counter() - t0) / reps * 1e3))
    step(one_two_calls)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        step(one_two_calls)
    ctx.sync()
    ms_two = ctx.max_over_ranks((time.perf_counter() - t0) / reps * 1e3)
    step()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    ctx.sync()
    ms = ctx.max_over_ranks((time.perf_counter() - t0) / reps * 1e3)
    # round-trip residuals: ||ray - p / |p|||^2 over the points whose
    # projection and unprojection are both Ok
    finite = torch.isfinite(pts).all(1)
    pn = pts / torch.linalg.norm(pts, dim=1, keepdim=True)
    red = torch.empty((2 * len(cams),), dtype=torch.float64, device=dev)
    for k, (st, ray, st2) in enumerate(outs):
        ok = (st[:n] == 0) & (st2[:n] == 0) & finite
        e2 = ((ray[:n] - pn) ** 2).sum(1)
        red[2 * k] = torch.where(ok, e2, torch.zeros_like(e2)).sum()
        red[2 * k + 1] = ok.sum().to(torch.float64)
    vec = red.to(ctx.cdev)
    coll_us = None
    if ctx.dist:
        tot = vec.clone()
        ctx.dist.all_reduce(tot)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            tot.copy_(vec)
            ctx.dist.all_reduce(tot)
        ctx.sync()
        coll_us = ctx.max_over_ranks((time.perf_counter() - t0) / reps * 1e6)
        vec = tot
    vec = vec.cpu().tolist()
    models = {}
    for k, name in enumerate(LEG4_MODELS.values()):
        models[name] = {"round_trip_ms": round(per_model[k], 4),
                        "Mpoints_per_s": round(n_total / per_model[k] / 1e3, 1),
                        "roofline": roofline_block(RT_BYTES_PER_POINT * n, 24 * n, per_model[k]),
                        "round_trip_ok": int(vec[2 * k + 1]),
                        "rms_round_trip_err": (vec[2 * k] / vec[2 * k + 1]) ** 0.5
                        if vec[2 * k + 1] else None}
    del pts, uv, outs, pn
    torch.cuda.empty_cache()
    return {"what": "6 models x project->unproject round trip (strong: one global batch "
                    "sharded over the ranks) + all-reduce of (sum err^2, n_ok) per model",
            "points_total": n_total, "points_per_rank": n, "steps": reps,
            "ms_per_step": round(ms, 4), "ms_per_step_two_calls": round(ms_two, 4),
            "value": round(len(cams) * n_total / ms / 1e3, 1),
            "unit": "Mround-trips/s (all 6 models, whole job)",
            "scaling": "strong", "allreduce_us": None if coll_us is None else round(coll_us, 2),
            "models": models}


def leg_config5(ctx, n_cells):
    """BASELINE config 5: KB -> DS conversion on ~`n_cells` sampled
    correspondences (camera_converter.rs:355-488: sample_points, linear
    estimation, bounded LM, reprojection errors).  Grid rows of sample_points
    are sharded over the ranks (each keeps its own correspondences, no data
    exchange), and the conversion runs over the union: merged TSQR factors,
    one all-reduce of the normal equations per LM evaluation, merged
    statistics and the distributed exact median (distributed.py)."""
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, conversion, samples
    from apex_camera_models import distributed as D
    kp, (w, h) = samples.SAMPLES[2]
    src = KannalaBrandtModel._from_params(kp, Resolution(w, h))
    from apex_camera_models import _lib
    # (r06) the cell form: sample_points also writes each kept point's grid
    # cell, and the LM's evaluations read those 4 B instead of the 16-B pixel
    # (acm_lm_optimize_cells; the same iterates, bit for bit)
    fn = D.gpu_sample_points_range(src, n_cells, cells=True)
    gx, gy = ctypes.c_uint32(), ctypes.c_uint32()  # the grid acm_sample_points uses
    _lib.check(_lib.load().acm_sample_points_grid(w, h, n_cells, ctypes.byref(gx),
                                                  ctypes.byref(gy)))
    ncx, ncy = gx.value, gy.value

    def sample():
        if ctx.dist:
            uv, xyz, cl, _, total = D.sharded_sample_points(ncx, ncy, ctx.rank, ctx.world, fn)
        else:
            uv, xyz, cl = fn(0, ncx * ncy)
            total = int(uv.shape[0])
        return uv, xyz, cl, total

    uv, xyz, cl, _ = sample()  # warm-up: the caching allocator's first multi-GB blocks
    del uv, xyz, cl
    ctx.sync()
    t0 = time.perf_counter()
    uv, xyz, cl, total = sample()
    ctx.sync()
    t_s = ctx.max_over_ranks(time.perf_counter() - t0)
    # N > 1: the sharded conversion over RCCL driven from libacm (r06; gloo
    # rehearsals: torch.distributed callbacks).  N = 1: the 1-GPU path, and
    # beside it the same sharded path under a 1-rank RCCL communicator
    # (its overhead on one GPU, and the same bits).
    coll = D.make_collective() if ctx.dist else None
    sharded1 = None
    if not ctx.dist:
        try:
            sharded1 = D.RcclCollective()
        except Exception as e:  # noqa: BLE001 -- reported in the line, headline kept
            sharded1 = f"{type(e).__name__}: {e}"[:200]

    def timed(c):
        # one untimed conversion first (its multi-GB workspaces' first
        # allocation), then the fastest of three, each the max over ranks
        conversion.convert(src, "double_sphere", xyz, uv, collective=c, cells=cl)
        t, m = float("inf"), None
        for _ in range(3):
            ctx.sync()
            t0 = time.perf_counter()
            m = conversion.convert(src, "double_sphere", xyz, uv, collective=c, cells=cl)
            ctx.sync()
            t = min(t, ctx.max_over_ranks(time.perf_counter() - t0))
        return t, m

    t_c, met = timed(coll)
    world1 = None
    if isinstance(sharded1, str):
        world1 = {"error": sharded1}
    elif sharded1 is not None:
        t1, m1 = timed(sharded1)
        world1 = {"what": "the sharded conversion (acm_*_sharded + RCCL from libacm) under a "
                          "1-rank communicator on this GPU",
                  "convert_ms": round(t1 * 1e3, 3),
                  "over_1gpu_path_pct": round(100 * (t1 / t_c - 1), 2),
                  "same_bits": (m1.model.params() == met.model.params()
                                and m1.final_reprojection_error.median ==
                                met.final_reprojection_error.median
                                and m1.initial_reprojection_error.median ==
                                met.initial_reprojection_error.median
                                and m1.lm_iterations == met.lm_iterations)}
        sharded1.close()
    out = {"what": "KB->DS conversion: sharded sample_points + linear estimation + bounded LM "
                   "+ reprojection errors",
           "requested_cells": n_cells, "grid": [ncx, ncy], "correspondences_total": total,
           "correspondences_rank0": int(uv.shape[0]), "sample_points_ms": round(t_s * 1e3, 3),
           "convert_ms": round(t_c * 1e3, 3), "convert_timing": "warm, best of 3",
           "optimization_ms_rank0": round(met.optimization_time_ms, 3),
           "lm_iterations": met.lm_iterations, "termination": met.lm_termination,
           "final_mean_px": met.final_reprojection_error.mean,
           "final_median_px": met.final_reprojection_error.median,
           "ds_params": met.model.params(), "scaling": "strong"}
    if ctx.dist:
        out["collective"] = type(coll).__name__
        if hasattr(coll, "close"):
            coll.close()
    if world1 is not None:
        out["sharded_world1"] = world1
    out["lm_observations"] = "cells (4 B per point, acm_lm_optimize_cells)"
    del uv, xyz, cl
    torch.cuda.empty_cache()
    return out


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    if env_world is not None and int(env_world) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_world} (the launcher started "
              f"a different number of ranks)", file=sys.stderr, flush=True)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs (never set by the driver): run every rank on device 0
    # and/or use gloo for the timing barrier/all-reduce on a 1-GPU box;
    # ACM_BENCH_CPU_REHEARSAL=1 (tests on a GPU-less host) stops after the
    # process-group init and the device census, touching no GPU.
    if os.environ.get("ACM_BENCH_SAME_DEVICE") == "1":
        local = 0
    backend = os.environ.get("ACM_BENCH_BACKEND", "nccl")
    rehearsal = os.environ.get("ACM_BENCH_CPU_REHEARSAL") == "1"
    # every phase (init, timed steps, each collective, each leg) is bounded
    tmo = float(os.environ.get("ACM_BENCH_TIMEOUT", "120"))
    device = None if rehearsal else (local if world > 1 else 0)
    wd = PhaseWatchdog(rank, local, device, tmo)
    global _WD
    _WD = wd
    wd.arm("process-group init")
    if world > 1:
        from datetime import timedelta
        if not rehearsal:
            torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                    timeout=timedelta(seconds=tmo))
        else:
            dist.init_process_group(backend, timeout=timedelta(seconds=tmo))
        world = dist.get_world_size()
        rank = dist.get_rank()
        wd.rank = rank
    elif not rehearsal:
        torch.cuda.set_device(0)
    # which device every rank runs on, recorded in the line (a first 8-GPU
    # run that maps two ranks to one device shows up here)
    wd.arm("device census")
    me = {"rank": rank, "local_rank": local, "device": device}
    if device is not None:
        pr = torch.cuda.get_device_properties(device)
        me["pci"] = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
    ranks_devices = [me]
    if world > 1:
        ranks_devices = [None] * world
        withhold = os.environ.get("ACM_BENCH_WITHHOLD_RANK")  # tests: a rank that never joins
        if withhold is not None and int(withhold) == rank:
            time.sleep(10 * tmo)
        dist.all_gather_object(ranks_devices, me)
    if rehearsal:
        wd.disarm()
        if rank == 0:
            # the labels the GPU run would attach for these shard sizes
            from apex_camera_models.distributed import shard_range
            bpp = 24 + 16 + 1 + (16 * 8 if not a.no_jacobian else 0)
            n_strong = shard_range(a.points, 0, world)[1]
            n4 = shard_range(a.leg4_points, 0, world)[1]
            planned = {"weak": roofline_block(bpp * a.points, 24 * a.points, None)["bound"],
                       "strong": roofline_block(bpp * n_strong, 24 * n_strong, None)["bound"],
                       "config4": roofline_block(RT_BYTES_PER_POINT * n4, 24 * n4, None)["bound"]}
            print(json.dumps({"rehearsal": "cpu", "n_ranks_seen": world,
                              "ranks_devices": ranks_devices, "planned_bounds": planned}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    wd.arm("setup")
    dev = torch.device("cuda", torch.cuda.current_device())
    cdev = dev if backend == "nccl" else torch.device("cpu")  # collectives' tensors

    from apex_camera_models import _lib, samples
    from apex_camera_models.distributed import shard_range
    L = _lib.load()
    model_id = MODELS[a.model]
    params, (w, h) = samples.SAMPLES[model_id]
    P = len(params)
    want_j = not a.no_jacobian
    lay = _lib.LAYOUT_SOA if a.layout == "soa" else _lib.LAYOUT_AOS

    cam = _lib.AcmCamera()
    arr = (ctypes.c_double * P)(*params)
    _lib.check(L.acm_camera_init(ctypes.byref(cam), model_id, arr, P, w, h))
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream

    def points(mode):
        """this rank's resident batch: (points tensor, n, global n)"""
        if mode == "weak":
            n = a.points
            return samples.synthetic_points_device(n, offset=rank * n, layout=a.layout), n, \
                n * world
        lo, hi = shard_range(a.points, rank, world)
        full = samples.synthetic_points_device(a.points, layout=a.layout)
        if a.layout == "soa":
            pts = full[:, lo:hi].contiguous()
        else:
            pts = full[lo:hi].contiguous()
        del full
        return pts, hi - lo, a.points

    def measure(mode):
        pts, n, n_global = points(mode)
        uv = torch.empty((n, 2), dtype=torch.float64, device=dev)
        st = torch.empty((n,), dtype=torch.uint8, device=dev)
        jac = torch.empty((P, n, 2), dtype=torch.float64, device=dev) if want_j else None
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
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=cdev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        ms_per_step = elapsed * 1e3 / a.steps
        out = {"value": round(n_global / (ms_per_step / 1e3) / 1e6, 2),
               "ms_per_step": round(ms_per_step, 5), "kernel_ms": round(kern_ms, 5),
               "points_per_rank": n, "global_points": n_global}
        if a.verify_shards and mode == "strong":
            out["shards_match_single_projection"] = verify(pts, n, uv, st, jac)
        return out, (pts, n)

    def verify(pts, n, uv, st, jac):
        """every rank's shard outputs, concatenated in rank order, equal one
        projection of the whole global batch (bit for bit)"""
        parts = [torch.cat([uv.reshape(-1), jac.reshape(-1) if jac is not None else
                            uv.new_empty(0)]).cpu(), st.cpu()]
        if world > 1:
            gathered = [None] * world
            dist.all_gather_object(gathered, parts)
        else:
            gathered = [parts]
        if rank != 0:
            return True
        full = samples.synthetic_points_device(a.points, layout=a.layout)
        N = a.points
        uv1 = torch.empty((N, 2), dtype=torch.float64, device=dev)
        st1 = torch.empty((N,), dtype=torch.uint8, device=dev)
        j1 = torch.empty((P, N, 2), dtype=torch.float64, device=dev) if want_j else None
        _lib.check(L.acm_project(ctypes.byref(cam), N, full.data_ptr(), lay, uv1.data_ptr(),
                                 st1.data_ptr(), j1.data_ptr() if want_j else None, sh))
        torch.cuda.synchronize()
        uv_c = torch.cat([g[0][: 2 * len(g[1])].reshape(-1, 2) for g in gathered])
        st_c = torch.cat([g[1] for g in gathered])
        ok = torch.equal(st_c, st1.cpu()) and torch.equal(
            uv_c.view(torch.int64), uv1.cpu().view(torch.int64))
        if want_j:
            jc = torch.cat([g[0][2 * len(g[1]):].reshape(P, -1, 2) for g in gathered], dim=1)
            ok = ok and torch.equal(jc.view(torch.int64), j1.cpu().view(torch.int64))
        return bool(ok)

    wd.arm(f"{a.scaling}-scaling timed steps")
    main_res, (pts, n) = measure(a.scaling)
    other = None
    if world > 1:  # the other scaling mode, same process group, same run
        del pts
        other_mode = "strong" if a.scaling == "weak" else "weak"
        wd.arm(f"{other_mode}-scaling timed steps")
        other, _ = measure(other_mode)
        other["mode"] = other_mode
        pts, n, _ = points(a.scaling)  # the residual pass below runs on the primary shard

    wd.arm("residual pass + all-reduce")
    # The north-star collective: per rank one residual pass over its shard
    # (acm_reprojection_stats against observations projected with fx * 1.01),
    # then ONE all-reduce of (sum ||r||^2, n_valid) -- timed on its own.
    pcam = _lib.AcmCamera()
    pparams = list(params)
    pparams[0] *= 1.01
    _lib.check(L.acm_camera_init(ctypes.byref(pcam), model_id,
                                 (ctypes.c_double * P)(*pparams), P, w, h))
    obs = torch.empty((n, 2), dtype=torch.float64, device=dev)
    sto = torch.empty((n,), dtype=torch.uint8, device=dev)
    pts_aos = pts if a.layout == "aos" else pts.t().contiguous()
    _lib.check(L.acm_project(ctypes.byref(pcam), n, pts_aos.data_ptr(), _lib.LAYOUT_AOS,
                             obs.data_ptr(), sto.data_ptr(), None, sh))
    res = torch.empty((8,), dtype=torch.float64, device=dev)
    ws_b = L.acm_reprojection_stats_workspace_size(n)
    ws = torch.empty(((ws_b + 7) // 8,), dtype=torch.float64, device=dev)
    _lib.check(L.acm_reprojection_stats(ctypes.byref(cam), n, pts_aos.data_ptr(),
                                        _lib.LAYOUT_AOS, obs.data_ptr(), res.data_ptr(), None,
                                        ws.data_ptr(), ws_b, sh))
    vec = torch.stack([res[7], res[5]]).to(cdev).contiguous()  # (sum ||r||^2, n_valid)
    coll = {"op": "all_reduce(sum) of [sum ||r||^2, n_valid] (16 B)", "ranks": world}
    if world > 1:
        red = vec.clone()
        for _ in range(3):
            red.copy_(vec)
            dist.all_reduce(red)
        torch.cuda.synchronize()
        reps = 20
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            red.copy_(vec)
            dist.all_reduce(red)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / reps * 1e6
        t = torch.tensor([us], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        coll["us"] = round(float(t[0]), 2)
        coll["backend"] = dist.get_backend()
    else:
        red = vec
        coll["us"] = None
        coll["backend"] = None
    red = red.cpu()
    coll["global_sum_sq_px2"] = float(red[0])
    coll["global_n_valid"] = int(red[1])
    coll["global_rmse_px"] = (float(red[0]) / float(red[1])) ** 0.5 if float(red[1]) else None

    # BASELINE configs 4 and 5 (the multi-GPU configs), after the headline's
    # timed region and its collective: sub-objects of the one line
    want_legs = set() if a.legs == "none" else set(a.legs.split(","))
    legs = {}
    if want_legs:
        del pts, obs, sto, pts_aos
        torch.cuda.empty_cache()
        ctx = LegCtx(rank, world, dist if world > 1 else None, cdev)
        legs = run_legs(want_legs, [("4", "config4",
                                     lambda: leg_config4(ctx, a.leg4_points, a.leg_steps)),
                                    ("5", "config5", lambda: leg_config5(ctx, a.leg5_cells))], wd)
        torch.cuda.empty_cache()

    if rank == 0:
        bpp = 24 + 16 + 1 + (16 * P if want_j else 0)
        kern_ms = main_res["kernel_ms"]
        achieved = bpp * main_res["points_per_rank"] / (kern_ms / 1e3) / 1e9
        workload = (f"{a.model}_project{'_jacobian' if want_j else ''}_f64_"
                    f"{a.layout}")
        traffic, traffic_src = load_traffic(workload, main_res["points_per_rank"])
        out = {
            "metric": "Mpoints/sec project+Jacobian (KB, f64) at 1/2/4/8 GPU; % HBM roofline",
            "value": main_res["value"],
            "unit": "Mpoints/s",
            "n_gpus": a.gpus,
            "n_ranks_seen": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seed 20251205 Philox on device; x,y~U[-1,1), z~U[0.5,4), "
                    "0.1% edge points)",
            "config": {"workload": workload, "points_per_gpu": main_res["points_per_rank"],
                       "global_points": main_res["global_points"],
                       "model_params": "samples/kannala_brandt.yaml" if a.model == "kb"
                       else a.model, "jacobian_layout": "2N x P column-major (nalgebra DMatrix)",
                       "parallelism": f"shard{world} ({a.scaling} scaling: "
                                      + ("independent per-rank point batches)" if
                                         a.scaling == "weak" else
                                         "contiguous shards of one global batch)")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": bpp * main_res["points_per_rank"],
                         "kernel_ms": kern_ms},
            "collective": coll,
            "ranks_devices": ranks_devices,
        }
        if "shards_match_single_projection" in main_res:
            out["shards_match_single_projection"] = main_res["shards_match_single_projection"]
        if other is not None:
            npr = other["points_per_rank"]
            other["roofline"] = roofline_block(bpp * npr, 24 * npr, other["kernel_ms"])
            out[other["mode"]] = other
        out.update(legs)
        wd.arm("cpu baseline", 10 * tmo)
        if not a.no_cpu_baseline and world == 1:  # rank 0 at N=1 only
            out["cpu_baseline"] = cpu_baseline(model_id, params, w, h, main_res["points_per_rank"],
                                               a.cpu_baseline_seconds)
            out["cpu_baseline_o2"] = cpu_baseline(model_id, params, w, h,
                                                  main_res["points_per_rank"],
                                                  a.cpu_baseline_seconds / 2, opt="O2")
            thr = host_threads()
            if thr > 1:
                out["cpu_baseline_all_cores"] = cpu_baseline_all_cores(
                    model_id, params, w, h, main_res["points_per_rank"],
                    a.cpu_baseline_seconds / 2, thr)
        print(json.dumps(out), flush=True)
    wd.arm("shutdown")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    wd.disarm()


_WD = None

if __name__ == "__main__":
    try:
        main()
    except Exception:
        if _WD is not None:  # name the rank and the phase that raised
            print(f"bench.py: {_WD.who()} failed in '{_WD.phase}'", file=sys.stderr, flush=True)
        raise
