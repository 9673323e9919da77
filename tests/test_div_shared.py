"""CPU check of the shared-divisor division the HIP kernels use in place of
K IEEE divisions by one divisor (camera_models.hpp div_shared / div_rn):
one reciprocal y = RN(1/b), then RN(a*y) corrected by one FMA residual step
(Markstein) must be bit-identical to a/b inside the kernels' guard range
|a|, |b| in [2^-500, 2^500].  tools/div_check.c runs the same binary64
mul/fma/div sequence on the host; here 7 x 3M cases (random and adversarial
significands, guard-limit exponents).  The full 1.8e9-case run is
`tools/div_check 300000000 <mode> 1` per mode."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def div_check(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("divc") / "div_check")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tools", "div_check.c"), "-lm"], check=True)
    return exe


@pytest.mark.parametrize("mode", range(7))
def test_shared_divisor_division_is_correctly_rounded(div_check, mode):
    r = subprocess.run([div_check, "3000000", str(mode), "1"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "bad 0" in r.stdout
