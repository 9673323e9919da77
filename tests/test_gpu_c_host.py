"""The C-ABI used from a torch-free host program (what a Rust `extern "C"`
binding does): compile examples/c_host_project.c with gcc and
run it on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _compile(tmp_path):
    exe = str(tmp_path / "c_host_project")
    libdir = os.path.join(ROOT, "apex-camera-models_amd", "lib")
    subprocess.run(["gcc", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "c_host_project.c"), "-L", libdir, "-lacm",
                    f"-Wl,-rpath,{libdir}", "-lm", "-o", exe], check=True)
    return exe


def test_c_host_program_compiles(tmp_path):
    assert os.path.exists(_compile(tmp_path))


@pytest.mark.gpu
def test_c_host_program_runs(tmp_path):
    exe = _compile(tmp_path)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("OK")
    assert "status 3" in r.stdout and "status 2" in r.stdout
