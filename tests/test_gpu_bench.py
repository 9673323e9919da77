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
    assert d["config4"]["points_total"] == 50_000_000 and d["config4"]["value"] > 0
    # the one-pass round trip and the twelve-launch form it replaces, both timed
    assert 0 < d["config4"]["ms_per_step"] and 0 < d["config4"]["ms_per_step_two_calls"]
    assert d["config5"]["correspondences_total"] == 92_935_075
    assert d["config5"]["final_mean_px"] < 0.01


def test_bench_self_launch_world2():
    """the driver's own command form: plain `bench.py --gpus 2`, no launcher;
    bench.py starts both ranks itself (gloo, both on device 0 on this box)"""
    env = dict(os.environ, ACM_BENCH_SAME_DEVICE="1", ACM_BENCH_BACKEND="gloo",
               OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--points", "300000",
                        "--no-cpu-baseline", "--leg4-points", "600001",
                        "--leg5-cells", "2000000", "--leg-steps", "2"],
                       capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    d = _line(r.stdout)
    assert d["n_gpus"] == d["n_ranks_seen"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_points"] == 600000
    assert d["strong"]["mode"] == "strong" and d["strong"]["global_points"] == 300000
    assert d["collective"]["ranks"] == 2 and d["collective"]["us"] > 0
    # BASELINE config 4 over both ranks: the all-reduced counts equal the
    # single-process leg's (same global batch, sharded)
    c4 = d["config4"]
    assert c4["points_total"] == 600001 and c4["points_per_rank"] == 300001
    assert c4["allreduce_us"] > 0 and c4["value"] > 0 and len(c4["models"]) == 6
    one = _line(subprocess.run(
        [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0",
         "--points", "1000", "--no-cpu-baseline", "--legs", "4", "--leg4-points", "600001",
         "--leg-steps", "1"], capture_output=True, text=True, timeout=300, cwd=ROOT).stdout)
    for name, m in c4["models"].items():
        m1 = one["config4"]["models"][name]
        assert m["round_trip_ok"] == m1["round_trip_ok"] > 0.8 * 600001, name
        assert abs(m["rms_round_trip_err"] - m1["rms_round_trip_err"]) <= \
            1e-9 * m1["rms_round_trip_err"] + 1e-300, name
    # BASELINE config 5: row-sharded sample_points + the sharded conversion
    c5 = d["config5"]
    assert c5["correspondences_total"] > c5["correspondences_rank0"] > 0
    assert c5["final_mean_px"] < 0.05 and c5["lm_iterations"] > 0
    assert c5["convert_ms"] > 0 and c5["sample_points_ms"] > 0


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
