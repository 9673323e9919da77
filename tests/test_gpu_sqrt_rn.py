"""camera_models.hpp's sqrt_rn (r06) is the compiler's correctly rounded f64
sqrt without its rescaling of inputs below 2^-767 and its 0 / inf fixup, with
the full sqrt() kept for those inputs.  The claim every bit-exact model path
rests on: the same result bit for bit for every input.  Checked on the GPU
through tools/build/libhbmprobe.so (acm_probe_sqrt_rn) over random bit
patterns of every exponent (the rescaled range, denormals, zeros, infinities
and NaNs included), sums of squares as the kernels form them, and perfect
squares with their neighbours -- 2.4e8 inputs."""
import ctypes
import os

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sqrt_rn_is_the_compiler_sqrt():
    import torch
    lib = os.path.join(ROOT, "tools", "build", "libhbmprobe.so")
    if not os.path.exists(lib):
        pytest.fail("tools/build/libhbmprobe.so missing: run __graft_entry__.build()")
    P = ctypes.CDLL(lib)
    vp = ctypes.c_void_p
    P.acm_probe_sqrt_rn.argtypes = [vp, ctypes.c_size_t, vp, vp, vp]
    sh = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(11)
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    first = torch.zeros(24, dtype=torch.float64, device="cuda")
    n = 20_000_000
    tested = 0

    def check(a):
        nonlocal tested
        a = a.contiguous()
        assert P.acm_probe_sqrt_rn(a.data_ptr(), a.numel(), bad.data_ptr(), first.data_ptr(),
                                   sh) == 0
        tested += a.numel()

    for k in range(3):
        bits = torch.randint(-2 ** 63, 2 ** 63 - 1, (n,), device="cuda", generator=g,
                             dtype=torch.int64)
        check((bits & 0x7FFFFFFFFFFFFFFF).view(torch.float64))  # every exponent, sign clear
        check(bits.view(torch.float64))                         # and both signs
        x = torch.randn(n, device="cuda", generator=g, dtype=torch.float64) * 10.0 ** (3 * k - 3)
        y = torch.randn(n, device="cuda", generator=g, dtype=torch.float64) * 10.0 ** (3 * k - 3)
        check(x * x + y * y)
        m = torch.randint(1, 2 ** 26, (n,), device="cuda", generator=g, dtype=torch.int64).double()
        sq = m * m
        check(torch.nextafter(sq, sq * 2))
    special = torch.tensor([0.0, -0.0, float("inf"), float("-inf"), float("nan"), 2.0 ** -767,
                            2.0 ** -767 * (1 - 2.0 ** -53), 2.0 ** -1074, 1.7976931348623157e308,
                            1.0, 4.0, 2.0], dtype=torch.float64, device="cuda")
    check(special)
    torch.cuda.synchronize()
    assert tested > 2e8
    nbad = int(bad.item())
    assert nbad == 0, first.view(8, 3)[:min(nbad, 8)].tolist()
