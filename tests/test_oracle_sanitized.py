"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer
(sanitizers on the CPU checker; the GPU side has none
on this pool).  tests/oracle_san_driver.c drives every oracle entry point on
edge-heavy inputs (origin, behind the camera, NaN, inf, huge values,
out-of-image pixels, every model and policy); any sanitizer report fails."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_is_clean_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "oracle_san")
    subprocess.run(["gcc", "-O1", "-g", "-std=c11", "-ffp-contract=off", "-D_GNU_SOURCE",
                    "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests", "oracle_san_driver.c"),
                    os.path.join(ROOT, "oracle", "acm_oracle.c"), "-lm", "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert r.stdout.startswith("ok"), r.stdout
    assert "runtime error" not in r.stderr, r.stderr[-4000:]
