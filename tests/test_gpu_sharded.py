"""The sharded conversion path (r06) on one GPU.

acm_linear_estimation_with_error_sharded / acm_reprojection_error_sharded
and the LM's all-reduce under a 1-rank collective must return the bits of
the 1-GPU path: every merge of a single part is the identity and the sums
of one rank are unchanged.  Two 1-rank collectives are checked: the local
one (no callbacks; the C code's own merge and median) and an RCCL
communicator that libacm drives itself (acm_rccl_init; no process group).
The 2/3-rank exchange is tests/test_gpu_distributed.py.  Reference loops:
bin/camera_converter.rs:371-420 (opening, LM), error_metrics.rs:62-121."""
import ctypes

import numpy as np
import pytest

from test_oracle import SAMPLES

pytestmark = pytest.mark.gpu
KB = 2


def _source(n):
    from apex_camera_models import KannalaBrandtModel, Resolution, util
    params, (w, h) = SAMPLES[KB]
    src = KannalaBrandtModel._from_params(params, Resolution(w, h))
    uv, xyz = util.sample_points(src, n)
    return src, uv, xyz


def _same_conversion(a, b):
    assert a.model.params() == b.model.params()
    assert a.lm_iterations == b.lm_iterations and a.lm_termination == b.lm_termination
    assert a.convergence_status == b.convergence_status
    for ea, eb in ((a.initial_reprojection_error, b.initial_reprojection_error),
                   (a.final_reprojection_error, b.final_reprojection_error)):
        for k in ("rmse", "min", "max", "mean", "stddev", "median", "n_valid"):
            va, vb = getattr(ea, k), getattr(eb, k)
            assert va == vb or (va != va and vb != vb), (k, va, vb)


@pytest.mark.parametrize("target", ["double_sphere", "kannala_brandt", "rad_tan", "ucm", "eucm",
                                    "fov"])
def test_sharded_world1_local_is_the_1gpu_path(target):
    from apex_camera_models import conversion
    from apex_camera_models.distributed import LocalCollective
    src, uv, xyz = _source(20_000)
    a = conversion.convert(src, target, xyz, uv)
    b = conversion.convert(src, target, xyz, uv, collective=LocalCollective())
    _same_conversion(a, b)


@pytest.mark.parametrize("target", ["double_sphere", "fov"])
def test_sharded_world1_rccl_is_the_1gpu_path(target):
    """The RCCL-backed collective (no Python per collective): the LM's
    all-reduce, the histogram all-reduces and the record all-gather run
    through a 1-rank RCCL communicator, and the bits are unchanged."""
    from apex_camera_models import _lib, conversion
    from apex_camera_models.distributed import RcclCollective
    if not _lib.load().acm_rccl_available():
        pytest.skip("librccl.so.1 not loadable")
    src, uv, xyz = _source(50_000)
    coll = RcclCollective()
    try:
        a = conversion.convert(src, target, xyz, uv)
        b = conversion.convert(src, target, xyz, uv, collective=coll)
        _same_conversion(a, b)
    finally:
        coll.close()


def test_rccl_collective_primitives():
    """coll.allreduce is an in-place sum (identity at world 1) and
    coll.allgather a rank-ordered gather, both on the caller's stream."""
    import torch
    from apex_camera_models import _lib
    from apex_camera_models.camera import _stream_handle
    from apex_camera_models.distributed import RcclCollective
    if not _lib.load().acm_rccl_available():
        pytest.skip("librccl.so.1 not loadable")
    coll = RcclCollective()
    try:
        v = torch.arange(91, dtype=torch.float64, device="cuda") * 0.5
        w = v.clone()
        assert coll.c.allreduce(coll.c.ctx, w.data_ptr(), 91, _stream_handle()) == 0
        out = torch.full((91,), -1.0, dtype=torch.float64, device="cuda")
        assert coll.c.allgather(coll.c.ctx, v.data_ptr(), out.data_ptr(), 91,
                                _stream_handle()) == 0
        torch.cuda.synchronize()
        assert torch.equal(w, v) and torch.equal(out, v)
        assert coll.c.world == 1 and coll.c.rank == 0
    finally:
        coll.close()


def test_sharded_reprojection_error_matches_unsharded():
    """acm_reprojection_error_sharded at world 1 (local collective) ==
    acm_reprojection_error, all 9 doubles bit for bit, and the shard's
    per-point errors are the same."""
    import torch
    from apex_camera_models import DoubleSphereModel, Resolution, _lib
    from apex_camera_models.camera import _stream_handle
    from apex_camera_models.distributed import LocalCollective
    L = _lib.load()
    params, (w, h) = SAMPLES[3]
    m = DoubleSphereModel._from_params(params, Resolution(w, h))
    rng = np.random.default_rng(5)
    n = 100_003
    xyz = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(-0.5, 4, n)], 1)
    obs = rng.uniform(0, 700, (n, 2))
    p3 = torch.as_tensor(xyz, device="cuda")
    p2 = torch.as_tensor(obs, device="cuda")
    cam = m.acm_camera()
    r1 = torch.empty(9, dtype=torch.float64, device="cuda")
    e1 = torch.empty(n, dtype=torch.float64, device="cuda")
    ws1 = torch.empty(L.acm_reprojection_error_workspace_size(n) // 8 + 1, dtype=torch.float64,
                      device="cuda")
    _lib.check(L.acm_reprojection_error(ctypes.byref(cam), n, p3.data_ptr(), 0, p2.data_ptr(),
                                        r1.data_ptr(), e1.data_ptr(), ws1.data_ptr(),
                                        ws1.numel() * 8, _stream_handle()))
    coll = LocalCollective()
    nb = L.acm_reprojection_error_sharded_workspace_size(n, 1)
    ws2 = torch.empty(nb // 8 + 1, dtype=torch.float64, device="cuda")
    r2 = torch.empty(9, dtype=torch.float64, device="cuda")
    e2 = torch.empty(n, dtype=torch.float64, device="cuda")
    _lib.check(L.acm_reprojection_error_sharded(ctypes.byref(cam), n, p3.data_ptr(), 0,
                                                p2.data_ptr(), None, None, r2.data_ptr(),
                                                e2.data_ptr(),
                                                ctypes.byref(coll.c), ws2.data_ptr(), nb,
                                                _stream_handle()))
    torch.cuda.synchronize()
    assert torch.equal(r1.view(torch.int64), r2.view(torch.int64))
    assert torch.equal(e1.view(torch.int64), e2.view(torch.int64))


def test_sharded_opening_counts_the_union():
    """The count checks see the union's size (kannala_brandt.rs:174-178):
    three points on one rank is too few for KB, and the initial error is
    still written first (camera_converter.rs:371-375 order)."""
    import torch
    from apex_camera_models import KannalaBrandtModel, Resolution, _lib
    from apex_camera_models.camera import _stream_handle
    from apex_camera_models.distributed import LocalCollective
    L = _lib.load()
    params, (w, h) = SAMPLES[KB]
    m = KannalaBrandtModel._from_params(params[:4] + [0.0] * 4, Resolution(w, h))
    xyz = torch.tensor([[0.1, 0.2, 1.0], [0.3, -0.1, 2.0], [-0.2, 0.1, 1.5]], dtype=torch.float64,
                       device="cuda")
    uv = torch.tensor([[300.0, 260.0], [270.0, 250.0], [240.0, 265.0]], dtype=torch.float64,
                      device="cuda")
    coll = LocalCollective()
    nb = L.acm_linear_estimation_with_error_sharded_workspace_size(KB, 3, 1)
    ws = torch.empty(nb // 8 + 1, dtype=torch.float64, device="cuda")
    res = torch.full((9,), float("nan"), dtype=torch.float64, device="cuda")
    host = (ctypes.c_double * 8)()
    cam = m.acm_camera()
    rc = L.acm_linear_estimation_with_error_sharded(ctypes.byref(cam), 3, xyz.data_ptr(), 0,
                                                    uv.data_ptr(), None, None, res.data_ptr(),
                                                    host,
                                                    ctypes.byref(coll.c), ws.data_ptr(), nb,
                                                    _stream_handle())
    assert rc == _lib.ERR_INVALID_PARAMS
    torch.cuda.synchronize()
    assert host[5] == 3.0 and res[5].item() == 3.0 and res[8].item() == res[8].item()
