"""Where bench.py's wall time per step exceeds the kernel time: K launches of
the headline KB project+J (10M points) timed by the wall clock with (a) an
event pair around every launch (bench.py's timed region), (b) only one
event pair around all K, (c) the K launches captured once in a HIP graph
and replayed.  Interleaved, min over repeats.

  python tools/diag_bench_gaps.py [--steps 50]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--points", type=int, default=10_000_000)
    a = ap.parse_args()
    import torch
    from apex_camera_models import _lib, samples
    L = _lib.load()
    n, K = a.points, a.steps
    params, (w, h) = samples.SAMPLES[2]
    cam = _lib.AcmCamera()
    _lib.check(L.acm_camera_init(ctypes.byref(cam), 2, (ctypes.c_double * 8)(*params), 8, w, h))
    pts = samples.synthetic_points_device(n)
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    st = torch.empty((n,), dtype=torch.uint8, device="cuda")
    jac = torch.empty((8, n, 2), dtype=torch.float64, device="cuda")
    side = torch.cuda.Stream()
    out = {}

    def launch(stream):
        _lib.check(L.acm_project(ctypes.byref(cam), n, pts.data_ptr(), 0, uv.data_ptr(),
                                 st.data_ptr(), jac.data_ptr(), stream.cuda_stream))

    def per_step_events(stream):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(K)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for e0, e1 in ev:
            e0.record(stream)
            launch(stream)
            e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / K
        return wall, sum(e0.elapsed_time(e1) for e0, e1 in ev) / K

    def end_events(stream):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(K):
            launch(stream)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / K
        return wall, e0.elapsed_time(e1) / K

    # graph of K launches on a side stream (torch's capture API)
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.stream(side):
            launch(side)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=side):
                for _ in range(K):
                    launch(side)
        torch.cuda.synchronize()
        have_graph = True
    except Exception as e:  # capture refused: report and skip that cell
        print(json.dumps({"graph_capture_error": str(e)}), flush=True)
        have_graph = False

    def graph(stream):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        g.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / K
        return wall, e0.elapsed_time(e1) / K

    cur = torch.cuda.current_stream()
    for _ in range(5):
        cases = [("per_step_events", per_step_events), ("end_events", end_events)]
        for k, f in cases + ([("graph", graph)] if have_graph else []):
            wall, ev = f(cur)
            o = out.setdefault(k, {"wall_ms": 1e9, "event_ms": 1e9})
            o["wall_ms"] = min(o["wall_ms"], round(wall, 5))
            o["event_ms"] = min(o["event_ms"], round(ev, 5))
    print(json.dumps({"what": "bench wall vs kernel time", "steps": K, "points": n,
                      "cells": out}))


if __name__ == "__main__":
    main()
