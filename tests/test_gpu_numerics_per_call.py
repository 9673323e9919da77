"""Per-call numerics (ACM_REFERENCE_NEWTON), VERDICT r02 item 5.

The reference's CameraModel is Send + Sync and used from &self on any thread
(/root/reference/src/camera/mod.rs:241-340).  The choice between the
certified fast Newton loops and the reference's own loops is therefore a
per-call flag, not process state: two threads that call acm_unproject /
acm_sample_points_ex at the same time with different flags each get exactly
their single-threaded results."""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cam(model, params, w, h):
    from apex_camera_models import _lib
    L = _lib.load()
    cam = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam), model,
                                 (ctypes.c_double * len(params))(*params), len(params), w, h))
    return cam


def _unproject(cam, px, flag, stream):
    import torch
    from apex_camera_models import _lib
    n = px.shape[0]
    with torch.cuda.stream(stream):  # every allocation / fill / copy on this thread's stream
        rays = torch.empty((n, 3), dtype=torch.float64, device="cuda")
        st = torch.empty((n,), dtype=torch.uint8, device="cuda")
        _lib.check(_lib.load().acm_unproject(ctypes.byref(cam), n, px.data_ptr(),
                                             rays.data_ptr(), flag, st.data_ptr(),
                                             stream.cuda_stream))
    stream.synchronize()
    return rays, st


def _sample(cam, n, flag, stream):
    import torch
    from apex_camera_models import _lib
    L = _lib.load()
    ncx, ncy = ctypes.c_uint32(), ctypes.c_uint32()
    _lib.check(L.acm_sample_points_grid(cam.width, cam.height, n, ctypes.byref(ncx),
                                        ctypes.byref(ncy)))
    cap = ncx.value * ncy.value
    # (a torch.zeros here would be a fill kernel on the thread's current
    # stream, unordered with the library's kernels on `stream`: everything
    # goes on `stream`)
    with torch.cuda.stream(stream):
        uv = torch.empty((cap, 2), dtype=torch.float64, device="cuda")
        xyz = torch.empty((cap, 3), dtype=torch.float64, device="cuda")
        counts = torch.empty((2,), dtype=torch.int64, device="cuda")
        wsb = L.acm_sample_points_workspace_size(ctypes.byref(cam), n)
        ws = torch.empty(((wsb + 7) // 8,), dtype=torch.float64, device="cuda")
        _lib.check(L.acm_sample_points_ex(ctypes.byref(cam), n, 0, cap, flag, uv.data_ptr(),
                                          xyz.data_ptr(), counts.data_ptr(), ws.data_ptr(), wsb,
                                          stream.cuda_stream))
        m = int(counts[0].item())
        out = uv[:m].clone(), xyz[:m].clone()
    stream.synchronize()
    return out


def _bits_equal(a, b):
    import torch
    return a.shape == b.shape and torch.equal(a.contiguous().view(torch.int64),
                                              b.contiguous().view(torch.int64))


def test_unproject_flag_changes_only_rays_not_statuses():
    """RadTan: the flag gives the oracle's rays bit for bit, the default a
    few ulp off; statuses identical either way."""
    import torch

    import oracle as O
    from apex_camera_models import _lib, samples
    params, (w, h) = samples.SAMPLES[1]
    cam = _cam(1, params, w, h)
    rng = np.random.default_rng(5)
    pxh = np.stack([rng.uniform(-5, w + 5, 50_000), rng.uniform(-5, h + 5, 50_000)], 1)
    px = torch.as_tensor(pxh, device="cuda")
    s = torch.cuda.Stream()
    r_ref, st_ref = _unproject(cam, px, _lib.REFERENCE_NEWTON, s)
    r_def, st_def = _unproject(cam, px, 0, s)
    ro, so = O.unproject(1, params, w, h, pxh)
    assert np.array_equal(st_ref.cpu().numpy(), so) and torch.equal(st_ref, st_def)
    assert np.array_equal(r_ref.cpu().numpy(), ro, equal_nan=True)
    ok = so == 0
    d = np.abs(r_def.cpu().numpy()[ok] - ro[ok]).max()
    assert d <= 8 * 2.0 ** -52


def test_unknown_flag_bits_rejected():
    import torch
    from apex_camera_models import _lib
    params = [461.629, 460.152, 362.680, 246.049]
    cam = _cam(0, params, 752, 480)
    L = _lib.load()
    buf = torch.zeros((8,), dtype=torch.float64, device="cuda")
    assert L.acm_sample_points_ex(ctypes.byref(cam), 100, 0, 10, 0x400, buf.data_ptr(),
                                  buf.data_ptr(), buf.data_ptr(), buf.data_ptr(), 64,
                                  None) == _lib.ERR_INVALID_ARGUMENT
    assert L.acm_unproject(ctypes.byref(cam), 1, buf.data_ptr(), buf.data_ptr(), 0x400,
                           buf.data_ptr(), None) == _lib.ERR_INVALID_ARGUMENT


@pytest.mark.parametrize("model", [1, 2, 6])
def test_two_threads_different_numerics(model):
    """Two threads, each on its own stream, alternate acm_unproject and
    acm_sample_points_ex calls -- one with ACM_REFERENCE_NEWTON, one without
    -- 6 times each, concurrently.  Every result equals that thread's
    single-threaded result bit for bit."""
    import torch
    from apex_camera_models import _lib, samples
    params, (w, h) = samples.SAMPLES[model]
    cam = _cam(model, params, w, h)
    rng = np.random.default_rng(model)
    px = torch.as_tensor(np.stack([rng.uniform(0, w, 400_000), rng.uniform(0, h, 400_000)], 1),
                         device="cuda")
    base_s = torch.cuda.Stream()
    single = {f: (_unproject(cam, px, f, base_s), _sample(cam, 300_000, f, base_s))
              for f in (0, _lib.REFERENCE_NEWTON)}
    if model == 1:  # the two numerics really differ somewhere (RadTan rays)
        assert not _bits_equal(single[0][0][0], single[_lib.REFERENCE_NEWTON][0][0])
    errors = []

    def worker(flag):
        try:
            s = torch.cuda.Stream()
            for _ in range(6):
                (r, st), (uv, xyz) = _unproject(cam, px, flag, s), _sample(cam, 300_000, flag, s)
                (r0, st0), (uv0, xyz0) = single[flag]
                if not (_bits_equal(r, r0) and torch.equal(st, st0) and _bits_equal(uv, uv0)
                        and _bits_equal(xyz, xyz0)):
                    errors.append(flag)
        except Exception as e:  # surfaced by the assert below
            errors.append(repr(e))

    ths = [threading.Thread(target=worker, args=(f,)) for f in (0, _lib.REFERENCE_NEWTON)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors
