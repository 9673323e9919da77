"""Store ceiling of the sample_points write pass: write-only
kernels over the config-5 output shape, 92,935,075
kept points x (16-B pixel + 24-B ray) = 3.72 GB (acm_probe_write_sample in
tools/hbm_probe.hip, built by `make -C tools`), timed with HIP events on the
stream they run on; torch's fill_ beside them.  Compare with the write
pass `k_seg_write<TagKbPoly>` (tools/diag_sample.py)."""
import argparse
import ctypes
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "build", "libhbmprobe.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=92_935_075)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch
    lib = ctypes.CDLL(SO)
    lib.acm_probe_write_sample.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64,
                                           ctypes.c_void_p]
    n = a.points
    uv = torch.empty((n, 2), dtype=torch.float64, device="cuda")
    xyz = torch.empty((n, 3), dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    nbytes = 40 * n

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best

    def probe(v, blocks, chunk=0):
        def f():
            assert lib.acm_probe_write_sample(v, uv.data_ptr(), xyz.data_ptr(), n, blocks,
                                              chunk, ctypes.c_void_p(s.cuda_stream)) == 0
        ms = timed(f)
        return {"ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 3)}

    out = {"what": "write-only kernels over the config-5 sample_points output",
           "points": n, "bytes": nbytes}
    for blocks in (2048, 8192, 32768, (n + 255) // 256):
        out[f"aos_b{blocks}"] = probe(0, blocks)
        out[f"v4_b{blocks}"] = probe(1, blocks)
    for chunk in (256, 1024, 4096):
        waves = (n + chunk - 1) // chunk
        out[f"runs_c{chunk}"] = probe(2, (waves + 3) // 4, chunk)
    ms = timed(lambda: (uv.fill_(1.0), xyz.fill_(2.0)))
    out["torch_fill"] = {"ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 3)}
    ms = timed(lambda: (uv.zero_(), xyz.zero_()))
    out["torch_zero"] = {"ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
