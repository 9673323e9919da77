"""bench.py rehearsals on one GPU: the N=1 line, and world 2 (torch.distributed
.run, gloo for the barriers/collectives, both ranks on device 0) in strong
mode -- n_ranks_seen, the weak line measured beside it, the timed
north-star collective, and the strong shards concatenated in rank order equal
one projection of the global batch bit for bit."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    return json.loads(lines[0])


def test_bench_single_gpu_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3",
                        "--warmup", "1", "--points", "300000", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["n_ranks_seen"] == 1 and d["scaling"] == "weak"
    assert d["value"] > 0 and 0 < d["roofline"]["frac"] < 1.0
    assert d["collective"]["global_n_valid"] > 0.99 * 300000
    assert "traffic_source" in d["roofline"]


def test_bench_self_launch_world2():
    """the driver's own command form: plain `bench.py --gpus 2`, no launcher;
    bench.py starts both ranks itself (gloo, both on device 0 on this box)"""
    env = dict(os.environ, ACM_BENCH_SAME_DEVICE="1", ACM_BENCH_BACKEND="gloo",
               OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--points", "300000",
                        "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = _line(r.stdout)
    assert d["n_gpus"] == d["n_ranks_seen"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_points"] == 600000
    assert d["strong"]["mode"] == "strong" and d["strong"]["global_points"] == 300000
    assert d["collective"]["ranks"] == 2 and d["collective"]["us"] > 0


def test_bench_world2_strong_rehearsal():
    env = dict(os.environ, ACM_BENCH_SAME_DEVICE="1", ACM_BENCH_BACKEND="gloo",
               OMP_NUM_THREADS="1")
    n = 400_003  # ragged: shards 200002 + 200001
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                        "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--points", str(n),
                        "--scaling", "strong", "--verify-shards", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["n_ranks_seen"] == 2 and d["scaling"] == "strong"
    assert d["config"]["global_points"] == n and d["config"]["points_per_gpu"] == 200002
    assert d["shards_match_single_projection"] is True
    assert d["weak"]["mode"] == "weak" and d["weak"]["global_points"] == 2 * n
    c = d["collective"]
    assert c["ranks"] == 2 and c["us"] > 0 and c["backend"] == "gloo"
    assert c["global_n_valid"] > 0.99 * n
    assert "cpu_baseline" not in d
