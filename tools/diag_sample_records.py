"""Per-tile timeline of k_sample_fused from the ACM_DIAG_SAMPLE=7 build
(lib/libacm_diag7.so): wall-clock (100 MHz) stamps at entry, after the
first compute pass, after the look-back and after the stores were issued,
plus look-back loads / waits / windows / help passes per tile.  Shows how a
tile's lifetime splits between compute, look-back and stores, and how many
tiles sit in each phase at once.

  ACM_LIB_PATH=apex-camera-models_amd/lib/libacm_diag7.so python tools/diag_sample_records.py
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "apex-camera-models_amd"))


def main():
    import torch
    from apex_camera_models import _lib, samples, util
    from apex_camera_models.camera import MODEL_CLASSES, Resolution
    L = _lib.load()
    L.acm_diag_sample_records.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.acm_diag_sample_records.restype = ctypes.c_int
    names = {0: "pinhole", 2: "kannala_brandt", 3: "double_sphere"}
    cells = int(os.environ.get("CELLS", "100000000"))
    for mid in [int(x) for x in os.environ.get("MODELS", "2,0").split(",")]:
        params, (w, h) = samples.SAMPLES[mid]
        m = MODEL_CLASSES[names[mid]]._from_params([float(p) for p in params], Resolution(w, h))
        for _ in range(3):
            util.sample_points(m, cells)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        uv, xyz = util.sample_points(m, cells)
        e1.record()
        torch.cuda.synchronize()
        ntiles = -(-cells // 1024)
        rec = np.zeros((1 << 18, 8), dtype=np.uint64)
        assert L.acm_diag_sample_records(rec.ctypes.data, rec.nbytes) == 0
        r = rec[:ntiles].astype(np.int64)
        t0 = r[:, 0] - r[:, 0].min()
        t1, t2, t3 = r[:, 1] - r[:, 0].min(), r[:, 2] - r[:, 0].min(), r[:, 3] - r[:, 0].min()
        span = t3.max()
        us = lambda x: x / 100.0  # noqa: E731  (100 MHz ticks -> us)
        comp, lb, st, life = t1 - t0, t2 - t1, t3 - t2, t3 - t0

        def dist(x):
            q = np.percentile(x, [10, 50, 90, 99])
            return {"mean_us": round(us(x.mean()), 3), "p10": round(us(q[0]), 3),
                    "p50": round(us(q[1]), 3), "p90": round(us(q[2]), 3), "p99": round(us(q[3]), 3)}
        pred_later = float(np.mean(t1[1:] < t1[:-1]))
        out = {"model": names[mid], "cells": cells, "kept": int(uv.shape[0]), "tiles": ntiles,
               "event_ms": round(e0.elapsed_time(e1), 4), "span_us": round(us(span), 1),
               "compute": dist(comp), "lookback": dist(lb), "store_issue": dist(st), "lifetime": dist(life),
               "mean_tiles_resident": round(float(life.sum() / span), 1),
               "mean_tiles_in_lookback": round(float(lb.sum() / span), 1),
               "mean_tiles_in_compute": round(float(comp.sum() / span), 1),
               "predecessor_published_later_frac": round(pred_later, 4),
               "start_order_inversions_frac": round(float(np.mean(t0[1:] < t0[:-1])), 4),
               "polls": dist(r[:, 4] * 100), "polls_total": int(r[:, 4].sum()),
               "waits_total": int(r[:, 5].sum()), "tiles_that_waited": int((r[:, 5] > 0).sum()),
               "windows_total": int(r[:, 6].sum()), "max_windows": int(r[:, 6].max()),
               "helps_total": int(r[:, 7].sum())}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
