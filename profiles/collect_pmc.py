"""Turns rocprofv3 --pmc passes (tools/pmc_round.sh) into the per-launch HBM
traffic figure bench.py reports as roofline.traffic.

Corrections, exactly as /opt/skills/guides/MI355X_MICROARCH.md §HBM says:
  * FETCH_SIZE is in KiB and on gfx950 reads exactly 1/2 of the bytes of a
    wide coalesced streaming read (FETCH_SIZE = TCC_EA0_RDREQ x 64 B while the
    requests are 128 B) -> bytes = FETCH_SIZE * 1024 * 2;
  * WRITE_SIZE is in KiB and exact for 16-B-per-lane streaming stores
    -> bytes = WRITE_SIZE * 1024.
The TCC_EA0_RDREQ/WRREQ pass is kept as a cross-check (x64 B, reads x2).

  python profiles/collect_pmc.py gpurun_out/pmc_r01 --kernel k_project \
      --workload kb_project_jacobian_f64_aos --points 10000000 --out profiles/r01_pmc_kb.json
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import statistics
import importlib.util

_BI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "apex-camera-models_amd", "apex_camera_models", "_buildinfo.py")
_spec = importlib.util.spec_from_file_location("_acm_buildinfo", _BI)
_buildinfo = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_buildinfo)
source_sha256 = _buildinfo.source_sha256


def read_counters(d, kernel_pat):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_pat not in row["Kernel_Name"]:
                    continue
                key = (row["Counter_Name"], f, row["Dispatch_Id"])
                vals[key] = float(row["Counter_Value"])
    by = {}
    for (name, _, _), v in vals.items():
        by.setdefault(name, []).append(v)
    return by


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="directory prefix, e.g. gpurun_out/pmc_r01 (matches _1.._N)")
    ap.add_argument("--kernel", default="k_project")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--points", type=int, required=True)
    ap.add_argument("--algorithmic-bytes", type=int, default=None)
    ap.add_argument("--out", required=True)
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "apex-camera-models_amd", "lib", "libacm.so"),
        help="the libacm.so the passes ran (its sha256 is recorded: bench.py reports the "
             "traffic only for that build)")
    a = ap.parse_args()
    by = {}
    for d in sorted(glob.glob(a.prefix + "_*")):
        if os.path.isdir(d):
            for k, v in read_counters(d, a.kernel).items():
                by.setdefault(k, []).extend(v)
    med = {k: statistics.median(v) for k, v in by.items()}
    fetch = med["FETCH_SIZE"] * 1024 * 2 if "FETCH_SIZE" in med else None
    write = med["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in med else None
    out = {
        "workload": a.workload,
        "points": a.points,
        "kernel_filter": a.kernel,
        "hbm_bytes_per_launch": (fetch + write) if fetch is not None and write is not None
        else None,
        "read_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "cross_check_rdreq_bytes": med.get("TCC_EA0_RDREQ_sum", 0) * 64 * 2 or None,
        "cross_check_wrreq_bytes": med.get("TCC_EA0_WRREQ_sum", 0) * 64 or None,
        "algorithmic_bytes_per_launch": a.algorithmic_bytes,
        "dispatches_per_counter": {k: len(v) for k, v in by.items()},
        "raw_median": med,
        "corrections": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count of 128-B reads); "
                       "WRITE_SIZE KiB x1024",
        "libacm_sha256": hashlib.sha256(open(a.lib, "rb").read()).hexdigest(),
        "libacm_source_sha256": source_sha256(),
        "libacm_identity": _buildinfo.lib_identity(a.lib),
    }
    if a.algorithmic_bytes and out["hbm_bytes_per_launch"]:
        out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / a.algorithmic_bytes
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
