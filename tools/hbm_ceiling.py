"""Zero-compute HBM ceilings for the hot path's access patterns, measured on
this GPU (tools/hbm_probe.hip): pure read, pure 16-B-store write, and a
"mimic" of k_project<*, J> that moves exactly the same bytes in the same
instruction shape without the camera-model math.  The gap between a kernel
and its mimic is what the math costs; the mimic itself is the practical
ceiling for that traffic mix.

  python tools/hbm_ceiling.py [--points N] [--reps R]
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)
LIB = os.path.join(HERE, "build", "libhbmprobe.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    L = ctypes.CDLL(LIB)
    vp, sz, ci = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.acm_probe_read.argtypes = [vp, sz, vp, ci, ci, ci, vp]
    L.acm_probe_write.argtypes = [vp, sz, ci, vp]
    L.acm_probe_read_pts.argtypes = [vp, vp, sz, vp, ci, ci, vp]
    L.acm_probe_mimic.argtypes = [sz, vp, vp, vp, vp, ci, ci, ci, vp]
    sh = torch.cuda.current_stream().cuda_stream
    n = a.points
    cus = torch.cuda.get_device_properties(0).multi_processor_count

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(reps)]
        for e0, e1 in evs:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        return sum(e0.elapsed_time(e1) for e0, e1 in evs) / reps

    out = {}

    def cell(key, fn, nbytes):
        ms = min(timed(fn) for _ in range(a.reps))
        out[key] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                    "bytes": nbytes}

    acc = torch.zeros((cus * 32 * 4,), dtype=torch.float64, device="cuda")  # wave partials
    for nb in (40 * n, 160 * n):  # NE's 40 B/pt stream; a 4x larger one
        buf = torch.empty((nb // 8,), dtype=torch.float64, device="cuda").fill_(1.0)
        for g in (cus * 4, cus * 8, cus * 16, cus * 32):
            for un in (1, 2, 4, 8):
                for nt in (0, 1):
                    if nb > 40 * n and (un != 2 or g != cus * 8):
                        continue
                    cell(f"read_{nb >> 20}MiB_grid{g}_u{un}{'_nt' if nt else ''}",
                         lambda: L.acm_probe_read(buf.data_ptr(), nb, acc.data_ptr(), g, un, nt,
                                                  sh), nb)
        del buf
    pts = torch.ones((5 * n,), dtype=torch.float64, device="cuda")  # xyz, then obs
    for g in (cus * 4, cus * 8, cus * 16):
        for stage in (0, 1):
            cell(f"read_pts_aos_grid{g}_{'staged' if stage else 'strided'}_nt",
                 lambda: L.acm_probe_read_pts(pts.data_ptr(), pts.data_ptr() + 24 * n, n,
                                              acc.data_ptr(), g, stage, sh), 40 * n)
    del pts
    wb = 169 * n
    buf = torch.empty((wb // 8,), dtype=torch.float64, device="cuda")
    for nt in (0, 1):
        cell(f"write_{wb >> 20}MiB_{'nt' if nt else 'plain'}",
             lambda: L.acm_probe_write(buf.data_ptr(), wb, nt, sh), wb)
    del buf
    xyz = torch.rand((5 * n,), dtype=torch.float64, device="cuda")  # points, then obs
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((9, n, 2), dtype=torch.float64, device="cuda")
    for cols in (4, 6, 8, 9):
        for nt in (0, 1):
            cell(f"mimic_project_J{cols}_{'nt' if nt else 'plain'}",
                 lambda: L.acm_probe_mimic(n, xyz.data_ptr(), uv.data_ptr(), st.data_ptr(),
                                           jac.data_ptr(), cols, nt, 0, sh),
                 (24 + 16 + 1 + 16 * cols) * n)
    for cols in (6, 8):  # residual + J traffic: + 16 B observation read per point
        cell(f"mimic_residual_J{cols}_nt",
             lambda: L.acm_probe_mimic(n, xyz.data_ptr(), uv.data_ptr(), st.data_ptr(),
                                       jac.data_ptr(), cols, 1, 1, sh),
             (24 + 16 + 16 + 1 + 16 * cols) * n)
    print(json.dumps({"what": "HBM ceilings (zero-compute probes)", "points": n,
                      "device": torch.cuda.get_device_name(0), "cus": cus, "cells": out}))


if __name__ == "__main__":
    main()
