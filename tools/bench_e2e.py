"""End-to-end (PCIe-inclusive) rate of the headline path when the caller's
points live in HOST memory, as a Rust caller holding nalgebra Matrix3xX
would have them ("separately end-to-end with H2D/D2H").
Never the bench `value` -- that is measured with the inputs resident in HBM.

For KB project (+ the 2N x 8 Jacobian) over 10M f64 points, host buffers
pinned:
  * copy bandwidth alone: one 240 MB H2D, one 1.45 GB D2H;
  * serial: H2D all points -> acm_project -> D2H uv, status, J;
  * pipelined: 1M-point chunks round-robin over 3 HIP streams (H2D of one
    chunk, the kernel of another and the D2H of a third overlap; the
    column-major J of a chunk comes back as P contiguous column pieces).

  python tools/bench_e2e.py [--points N] [--chunk M] [--streams S]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--chunk", type=int, default=1_000_000)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    params, (w, h) = samples.SAMPLES[2]
    P = len(params)
    cam = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam), 2, (ctypes.c_double * P)(*params), P, w, h))
    N = a.points
    pts_h = samples.synthetic_points_device(N).cpu().pin_memory()
    uv_h = torch.empty((N, 2), dtype=torch.float64).pin_memory()
    st_h = torch.empty((N,), dtype=torch.uint8).pin_memory()
    jac_h = torch.empty((P, N, 2), dtype=torch.float64).pin_memory()
    dev = torch.device("cuda", 0)

    def timed(fn):
        best = 1e30
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    out = {"what": "KB project (+2x8 J), host pinned buffers, PCIe-inclusive", "points": N}
    # copy bandwidth alone
    pts_d = torch.empty((N, 3), dtype=torch.float64, device=dev)
    big_d = torch.empty((P * N * 2,), dtype=torch.float64, device=dev)
    t = timed(lambda: pts_d.copy_(pts_h, non_blocking=True))
    out["h2d_GBps"] = round(pts_h.numel() * 8 / t / 1e9, 1)
    t = timed(lambda: jac_h.view(-1).copy_(big_d, non_blocking=True))
    out["d2h_GBps"] = round(jac_h.numel() * 8 / t / 1e9, 1)
    del big_d

    for want_j in (True, False):
        tag = "with_jacobian" if want_j else "no_jacobian"
        bpp_h2d, bpp_d2h = 24, 17 + (16 * P if want_j else 0)
        uv_d = torch.empty((N, 2), dtype=torch.float64, device=dev)
        st_d = torch.empty((N,), dtype=torch.uint8, device=dev)
        jac_d = torch.empty((P, N, 2), dtype=torch.float64, device=dev) if want_j else None
        s0 = torch.cuda.current_stream()

        def serial():
            pts_d.copy_(pts_h, non_blocking=True)
            _lib.check(L.acm_project(ctypes.byref(cam), N, pts_d.data_ptr(), 0, uv_d.data_ptr(),
                                     st_d.data_ptr(), jac_d.data_ptr() if want_j else None,
                                     s0.cuda_stream))
            uv_h.copy_(uv_d, non_blocking=True)
            st_h.copy_(st_d, non_blocking=True)
            if want_j:
                jac_h.copy_(jac_d, non_blocking=True)

        t_ser = timed(serial)
        # kernel alone, same buffers
        t_k = timed(lambda: L.acm_project(ctypes.byref(cam), N, pts_d.data_ptr(), 0,
                                          uv_d.data_ptr(), st_d.data_ptr(),
                                          jac_d.data_ptr() if want_j else None, s0.cuda_stream))

        M = a.chunk
        streams = [torch.cuda.Stream() for _ in range(a.streams)]
        bufs = [(torch.empty((M, 3), dtype=torch.float64, device=dev),
                 torch.empty((M, 2), dtype=torch.float64, device=dev),
                 torch.empty((M,), dtype=torch.uint8, device=dev),
                 torch.empty((P, M, 2), dtype=torch.float64, device=dev) if want_j else None)
                for _ in streams]

        def pipelined():
            for c, lo in enumerate(range(0, N, M)):
                hi = min(N, lo + M)
                m = hi - lo
                s = streams[c % len(streams)]
                pd, ud, sd, jd = bufs[c % len(streams)]
                with torch.cuda.stream(s):
                    pd[:m].copy_(pts_h[lo:hi], non_blocking=True)
                    jv = jd[:, :m] if want_j else None
                    if want_j and m != M:  # the kernel writes a dense (P, m, 2) block
                        jv = torch.empty((P, m, 2), dtype=torch.float64, device=dev)
                    _lib.check(L.acm_project(ctypes.byref(cam), m, pd.data_ptr(), 0,
                                             ud.data_ptr(), sd.data_ptr(),
                                             jv.data_ptr() if want_j else None, s.cuda_stream))
                    uv_h[lo:hi].copy_(ud[:m], non_blocking=True)
                    st_h[lo:hi].copy_(sd[:m], non_blocking=True)
                    if want_j:
                        for p in range(P):
                            jac_h[p, lo:hi].copy_(jv[p], non_blocking=True)

        t_pipe = timed(pipelined)
        # the pipelined outputs equal the serial ones
        ok = True
        uv_ref, st_ref = uv_h.clone(), st_h.clone()
        jac_ref = jac_h.clone() if want_j else None
        serial()
        torch.cuda.synchronize()
        ok = torch.equal(uv_ref.view(torch.int64), uv_h.view(torch.int64)) and \
            torch.equal(st_ref, st_h)
        if want_j:
            ok = ok and torch.equal(jac_ref.view(torch.int64), jac_h.view(torch.int64))
        del bufs, uv_ref, st_ref, jac_ref, uv_d, st_d, jac_d
        out[tag] = {
            "bytes_h2d_per_point": bpp_h2d, "bytes_d2h_per_point": bpp_d2h,
            "kernel_ms": round(t_k * 1e3, 3),
            "serial_ms": round(t_ser * 1e3, 3),
            "serial_Mpoints_s": round(N / t_ser / 1e6, 1),
            "pipelined_ms": round(t_pipe * 1e3, 3),
            "pipelined_Mpoints_s": round(N / t_pipe / 1e6, 1),
            "pipelined_equals_serial": bool(ok),
            "chunk_points": M, "streams": a.streams,
        }
        print(json.dumps({tag: out[tag]}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
