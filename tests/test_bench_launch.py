"""bench.py's process launch, on the CPU (no GPU work happens in these runs):
a WORLD_SIZE that disagrees with --gpus exits 2 before torch is imported,
and `bench.py --gpus N` without a launcher starts N ranks with torchrun's
environment and exits non-zero when a rank fails."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_world_size_mismatch_exits_2():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--steps", "1"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=2" in r.stderr


def test_launcher_default_gpus_under_torchrun_mismatch():
    # torchrun with 2 ranks but no --gpus: --gpus defaults to 1 -> refused
    r = subprocess.run([sys.executable, BENCH, "--steps", "1"],
                       env=_env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2


def test_self_launch_spawns_ranks_with_torchrun_env(tmp_path):
    """launch_ranks gives every child RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*;
    a stand-in script records them (the real bench would need a GPU)."""
    import bench
    rec = tmp_path / "rec"
    rec.mkdir()
    child = tmp_path / "child.py"
    child.write_text(
        "import os, sys\n"
        f"open(os.path.join({str(rec)!r}, os.environ['RANK']), 'w').write(\n"
        "    ' '.join(os.environ[k] for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', "
        "'MASTER_ADDR', 'MASTER_PORT')))\n"
        "sys.exit(int(os.environ['RANK']) == int(os.environ.get('FAIL_RANK', -1)) and 7)\n")
    old_file, old_argv = bench.__file__, sys.argv
    env_keep = dict(os.environ)
    try:
        bench.__file__ = str(child)
        sys.argv = ["bench.py", "--gpus", "3"]
        os.environ.pop("MASTER_PORT", None)
        assert bench.launch_ranks(3) == 0
        got = sorted((rec / str(r)).read_text().split() for r in range(3))
        assert [g[:3] for g in got] == [["0", "0", "3"], ["1", "1", "3"], ["2", "2", "3"]]
        assert all(g[3] == "127.0.0.1" for g in got) and len({g[4] for g in got}) == 1
        os.environ["FAIL_RANK"] = "1"
        assert bench.launch_ranks(3) == 7
    finally:
        bench.__file__, sys.argv = old_file, old_argv
        os.environ.clear()
        os.environ.update(env_keep)


def test_self_launch_failing_ranks_exit_nonzero():
    """on this GPU-less host every rank fails at its first device call: the
    parent must report failure, not print a line"""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--points", "1000", "--no-cpu-baseline"],
                       env=_env(ACM_BENCH_BACKEND="gloo"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def _start_parent(tmp_path):
    """A launch_ranks parent (bench.launch_ranks(2)) whose ranks are stand-ins
    that record their pid and sleep; returns (parent Popen, rank pids)."""
    import time
    rec = tmp_path / "pids"
    rec.mkdir()
    child = tmp_path / "child.py"
    child.write_text(
        "import os, time\n"
        f"open(os.path.join({str(rec)!r}, os.environ['RANK']), 'w').write(str(os.getpid()))\n"
        "time.sleep(600)\n")
    parent = tmp_path / "parent.py"
    parent.write_text(
        "import sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import bench\n"
        f"bench.__file__ = {str(child)!r}\n"
        "sys.argv = ['bench.py', '--gpus', '2']\n"
        "sys.exit(bench.launch_ranks(2))\n")
    p = subprocess.Popen([sys.executable, str(parent)], env=_env(), stderr=subprocess.PIPE,
                         text=True)
    t_end = time.time() + 60
    while time.time() < t_end and len(list(rec.iterdir())) < 2:
        time.sleep(0.05)
    time.sleep(0.2)
    pids = [int((rec / str(r)).read_text()) for r in range(2)]
    return p, pids


def _gone(pids, timeout=15.0):
    import time
    t_end = time.time() + timeout
    while time.time() < t_end:
        alive = []
        for pid in pids:
            try:
                os.kill(pid, 0)
                # a zombie awaiting its (dead) parent's reaping is gone too
                with open(f"/proc/{pid}/stat") as f:
                    if f.read().split(")")[-1].split()[0] != "Z":
                        alive.append(pid)
            except (ProcessLookupError, FileNotFoundError):
                pass
        if not alive:
            return True
        time.sleep(0.1)
    return False


def test_parent_sigterm_stops_ranks(tmp_path):
    """a SIGTERM to the parent (which started its ranks in their
    own sessions) is forwarded to every rank; the parent exits 128 + 15"""
    import signal
    p, pids = _start_parent(tmp_path)
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    assert _gone(pids), pids


def test_parent_sigkill_stops_ranks(tmp_path):
    """a parent killed outright (timeout -k's SIGKILL) still takes its ranks
    with it (PR_SET_PDEATHSIG in each rank)"""
    import signal
    p, pids = _start_parent(tmp_path)
    p.send_signal(signal.SIGKILL)
    p.wait(timeout=30)
    assert _gone(pids), pids


def _tagged_pids(tag):
    """pids of live (non-zombie) processes whose environment carries tag"""
    out = []
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            with open(f"/proc/{d}/environ", "rb") as f:
                if f"ACM_TEST_TAG={tag}".encode() not in f.read():
                    continue
            with open(f"/proc/{d}/stat") as f:
                if f.read().split(")")[-1].split()[0] == "Z":
                    continue
        except (FileNotFoundError, PermissionError, ProcessLookupError):
            continue
        out.append(int(d))
    return out


def test_cpu_rehearsal_device_census_world2():
    """`bench.py --gpus 2` on gloo up to the device census (no GPU touched):
    both ranks join within the bounded init and rank 0's line records every
    rank's (rank, LOCAL_RANK, device)"""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"],
                       env=_env(ACM_BENCH_BACKEND="gloo", ACM_BENCH_CPU_REHEARSAL="1",
                                ACM_BENCH_TIMEOUT="60"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    import json
    d = json.loads(lines[0])
    assert d["n_ranks_seen"] == 2
    assert [(x["rank"], x["local_rank"]) for x in d["ranks_devices"]] == [(0, 0), (1, 1)]


def test_cpu_rehearsal_labels_infinity_cache_shards_world2():
    """at world 2 with a small strong batch (2M KB
    points: 1M per rank, 169 MB with the Jacobian) and config 4's shards
    (1M points per rank, 66 MB) everything a launch touches fits the
    256 MiB Infinity Cache, and the line's planned bounds say "effective
    (Infinity Cache)"; the weak shard (2M points per rank, 338 MB) stays
    "hbm"."""
    import json
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--points", "2000000",
                        "--leg4-points", "2000000"],
                       env=_env(ACM_BENCH_BACKEND="gloo", ACM_BENCH_CPU_REHEARSAL="1",
                                ACM_BENCH_TIMEOUT="60"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["planned_bounds"] == {"weak": "hbm", "strong": "effective (Infinity Cache)",
                                   "config4": "effective (Infinity Cache)"}


def test_roofline_block_rule():
    import bench
    big = bench.roofline_block(169 * 10_000_000, 24 * 10_000_000, 0.25)
    assert big["bound"] == "hbm" and abs(big["frac"] - 0.845) < 1e-9
    # N = 8 strong shard: 1.25M KB points, 211 MB in all
    assert bench.roofline_block(169 * 1_250_000, 24 * 1_250_000, 0.03)["bound"] == \
        "effective (Infinity Cache)"
    # config 4 at N = 8: 6.25M points, 412 MB in all but 150 MB of re-read input
    c4 = bench.roofline_block(66 * 6_250_000, 24 * 6_250_000, None)
    assert c4["bound"] == "hbm" and c4["input_fits_infinity_cache"]
    assert bench.roofline_block(66 * 50_000_000, 24 * 50_000_000, 0.6)["bound"] == "hbm"


def test_withheld_collective_exits_within_bound():
    """one rank never joins the first collective; the job
    ends non-zero within the bound (ACM_BENCH_TIMEOUT = 5 s, not the
    driver's 600 s), stderr names the rank, no line is printed and no rank
    process outlives the parent"""
    import time
    import uuid
    tag = uuid.uuid4().hex
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"],
                       env=_env(ACM_BENCH_BACKEND="gloo", ACM_BENCH_CPU_REHEARSAL="1",
                                ACM_BENCH_TIMEOUT="5", ACM_BENCH_WITHHOLD_RANK="1",
                                ACM_TEST_TAG=tag),
                       capture_output=True, text=True, timeout=300)
    dt = time.time() - t0
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "LOCAL_RANK" in r.stderr and "device census" in r.stderr, r.stderr[-2000:]
    # 5 s bound + interpreter / torch import time of the ranks
    assert dt < 120, dt
    assert _gone(_tagged_pids(tag)), _tagged_pids(tag)


def test_failing_leg_keeps_the_headline():
    """a BASELINE leg that raises becomes {"error": ...} in its
    sub-object; the legs after it still run (the headline line is built from
    run_legs' result, so it is printed either way)"""
    import bench

    def boom():
        raise MemoryError("HIP out of memory")
    legs = bench.run_legs({"4", "5"}, [("4", "config4", boom),
                                       ("5", "config5", lambda: {"value": 1.0})])
    assert legs["config4"]["error"].startswith("MemoryError")
    assert legs["config5"] == {"value": 1.0}
    assert bench.run_legs(set(), [("4", "config4", boom)]) == {}
