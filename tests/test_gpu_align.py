"""Line-aligned +Jacobian store path (k_project_al, ACM_TUNE_ALIGN_J).

Column c of the 2N x P Jacobian starts at byte 16*c*N, so for N not a
multiple of 8 the default kernel's stores straddle 128-B lines; the aligned
kernel re-maps which lane stores which element.  It must be bit-identical to
the direct kernel for every model, size, layout, store policy and buffer
offset, and must never write outside [0, N) of any stream (guard cells
around every buffer stay untouched).
"""
import ctypes

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

SIZES = [1, 5, 7, 8, 9, 247, 248, 249, 255, 256, 257, 495, 496, 1000, 4099, 65537]
GUARD = 32  # f64 guard cells (256 B) before and after every output: window 0 is line-aligned


def _setup(model):
    import torch
    from apex_camera_models import _lib, samples
    params, (w, h) = samples.SAMPLES[model]
    L = _lib.load()
    cam = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam), model, (ctypes.c_double * len(params))(*params),
                                 len(params), w, h))
    return torch, _lib, L, cam, params, w, h


def _guarded(torch, n_f64, off):
    """device f64 buffer with at least GUARD sentinel cells on both sides of
    an n_f64 window starting GUARD + off doubles in (off shifts the window's
    alignment by 8-B steps)"""
    buf = torch.full((n_f64 + 2 * GUARD + 16,), 7.25, dtype=torch.float64, device="cuda")
    start = GUARD + off
    return buf, start


def _set_align(_lib, L, align):
    """align 0 = direct kernel, 1 = line-aligned kernel, -1 = library
    default; returns an undo callable"""
    oa = L.acm_set_tuning(_lib.TUNE_ALIGN_J, align)

    def undo():
        L.acm_set_tuning(_lib.TUNE_ALIGN_J, oa)
    return undo


def _run_project(torch, _lib, L, cam, pts, P, layout, align, off_uv=0, off_j=0):
    n = pts.shape[0] if layout == 0 else pts.shape[1]
    uvb, su = _guarded(torch, 2 * n, off_uv)
    jb, sj = _guarded(torch, 2 * n * P, off_j)
    stb = torch.full((n + 2 * GUARD,), 0xAB, dtype=torch.uint8, device="cuda")
    undo = _set_align(_lib, L, align)
    try:
        _lib.check(L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), layout,
                                 uvb.data_ptr() + 8 * su, stb.data_ptr() + GUARD,
                                 jb.data_ptr() + 8 * sj, None))
        torch.cuda.synchronize()
    finally:
        undo()
    uvb, jb, stb = uvb.cpu(), jb.cpu(), stb.cpu()
    assert torch.all(uvb[:su] == 7.25) and torch.all(uvb[su + 2 * n:] == 7.25), "uv guard"
    assert torch.all(jb[:sj] == 7.25) and torch.all(jb[sj + 2 * n * P:] == 7.25), "J guard"
    assert torch.all(stb[:GUARD] == 0xAB) and torch.all(stb[GUARD + n:] == 0xAB), "status guard"
    return uvb[su:su + 2 * n], stb[GUARD:GUARD + n], jb[sj:sj + 2 * n * P]


@pytest.mark.parametrize("model", range(7))
def test_aligned_project_bit_identical(model):
    torch, _lib, L, cam, params, w, h = _setup(model)
    from apex_camera_models import samples
    P = len(params)
    for n in SIZES:
        pts_np = samples.synthetic_points(n)
        for layout in (0, 1):
            pts = torch.as_tensor(pts_np if layout == 0 else pts_np.T.copy(), device="cuda")
            a = _run_project(torch, _lib, L, cam, pts, P, layout, 0)
            for al in (1, -1):
                b = _run_project(torch, _lib, L, cam, pts, P, layout, al)
                for x, y, name in zip(a, b, ("uv", "status", "J")):
                    assert torch.equal(x.view(torch.int64) if x.dtype == torch.float64 else x,
                                       y.view(torch.int64) if y.dtype == torch.float64 else y), \
                        (model, n, layout, al, name)
        st0 = O.project(model, params, w, h, pts_np)[1]
        assert np.array_equal(b[1].numpy(), st0), (model, n)


@pytest.mark.parametrize("model", [2, 3])
@pytest.mark.parametrize("offs", [(1, 0), (0, 1), (3, 5), (2, 6), (1, 1)])
def test_aligned_project_buffer_offsets(model, offs):
    """8-byte and 16k-byte offsets of uv / J: same bits as the plain path."""
    torch, _lib, L, cam, params, w, h = _setup(model)
    from apex_camera_models import samples
    P = len(params)
    n = 10_007
    pts = torch.as_tensor(samples.synthetic_points(n), device="cuda")
    ref = _run_project(torch, _lib, L, cam, pts, P, 0, 0)
    for align in (-1, 1):
        got = _run_project(torch, _lib, L, cam, pts, P, 0, align, off_uv=offs[0], off_j=offs[1])
        for x, y in zip(ref, got):
            assert torch.equal(x, y) if x.dtype == torch.uint8 else \
                torch.equal(x.view(torch.int64), y.view(torch.int64))


@pytest.mark.parametrize("policy", [0, 1])
@pytest.mark.parametrize("model", range(7))
def test_aligned_residual_bit_identical(model, policy):
    torch, _lib, L, cam, params, w, h = _setup(model)
    from apex_camera_models import samples
    P = len(params)
    for n in (1, 9, 249, 1000, 65537):
        pts_np = samples.synthetic_points(n)
        uv0 = O.project(model, params, w, h, pts_np)[0]
        obs = torch.as_tensor(np.where(np.isnan(uv0), 3.0, uv0) + 0.25, device="cuda")
        pts = torch.as_tensor(pts_np, device="cuda")
        outs = []
        for align in (0, 1):
            for with_status in (True, False):
                rb, sr = _guarded(torch, 2 * n, 0)
                jb, sj = _guarded(torch, 2 * n * P, 0)
                stb = torch.full((n + 2 * GUARD,), 0xAB, dtype=torch.uint8, device="cuda")
                undo = _set_align(_lib, L, align)
                try:
                    _lib.check(L.acm_residual_jacobian(
                        ctypes.byref(cam), n, pts.data_ptr(), 0, obs.data_ptr(), policy,
                        rb.data_ptr() + 8 * sr, jb.data_ptr() + 8 * sj,
                        stb.data_ptr() + GUARD if with_status else None, None))
                    torch.cuda.synchronize()
                finally:
                    undo()
                rb, jb, stb = rb.cpu(), jb.cpu(), stb.cpu()
                assert torch.all(rb[:sr] == 7.25) and torch.all(rb[sr + 2 * n:] == 7.25)
                assert torch.all(jb[:sj] == 7.25) and torch.all(jb[sj + 2 * n * P:] == 7.25)
                if with_status:
                    assert torch.all(stb[:GUARD] == 0xAB) and torch.all(stb[GUARD + n:] == 0xAB)
                else:
                    assert torch.all(stb == 0xAB)
                outs.append((rb[sr:sr + 2 * n].view(torch.int64), jb[sj:sj + 2 * n * P]
                             .view(torch.int64), stb[GUARD:GUARD + n] if with_status else None))
        r_ref, j_ref, s_ref = outs[0]
        for r, j, s in outs[1:]:
            assert torch.equal(r, r_ref) and torch.equal(j, j_ref), (model, n, policy)
            if s is not None:
                assert torch.equal(s, s_ref)
        r0, J0, st0 = O.residual_jacobian(model, params, w, h, pts_np,
                                          obs.cpu().numpy(), policy)
        assert np.array_equal(s_ref.numpy(), st0)
