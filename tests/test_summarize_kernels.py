"""profiles/summarize_kernels.py: counter rows are split by launch size (grid
size, then duration class for persistent kernels whose grid does not change
with the problem size), and a rate above the physical peak is refused, not
printed."""
import csv
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "profiles"))

import summarize_kernels as S  # noqa: E402

NAME = "void acm::k_normal_eq<acm::Tag<acm::DoubleSphere>, 0, 1, 3, true>(acm::acm_camera)"
OTHER = "void acm::k_fast<acm::Tag<acm::Pinhole>>(acm::acm_camera)"


def write_kt(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "kt_kernel_trace.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp",
                    "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"])
        for i, (name, grid, us) in enumerate(rows):
            w.writerow([i + 1, name, 1000, 1000 + int(us * 1000), grid, 1, 1])


def write_pmc(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "pmc_counter_collection.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for i, (name, grid, ctrs) in enumerate(rows):
            for cn, v in ctrs.items():
                w.writerow([i + 1, grid, name, cn, v])


def test_sizes_split_and_peak_refused(tmp_path):
    p = str(tmp_path / "fp64_t")
    # one persistent kernel (same grid) at two sizes: 60 us (9.3M) and 600 us
    # (93M), interleaved; a second kernel whose counters claim 2x the peak
    write_kt(p + "_kt", [(NAME, 262144, 60.0), (NAME, 262144, 600.0),
                         (NAME, 262144, 61.0), (NAME, 262144, 598.0),
                         (OTHER, 1024, 10.0)])
    small = {"FETCH_SIZE": 372e6 / 2048, "WRITE_SIZE": 1.0}
    large = {"FETCH_SIZE": 3.72e9 / 2048, "WRITE_SIZE": 1.0}
    write_pmc(p + "_pmc1", [(NAME, 262144, small), (NAME, 262144, large),
                            (NAME, 262144, small), (NAME, 262144, large),
                            (OTHER, 1024, {"FETCH_SIZE": 160e6 / 2048, "WRITE_SIZE": 0.0})])
    dur, classes = S.durations(p + "_kt")
    out = S.summarize(dur, S.counters(p, classes))
    rows = {(r["kernel"], r["size_class"]): r for r in out.values()}
    k = S.short(NAME)
    # each size's bytes over its own duration: 6.2 TB/s both, never mixed
    assert abs(rows[(k, 0)]["hbm_GBps"] - 372e6 / 60.5e-6 / 1e9) < 5
    assert abs(rows[(k, 1)]["hbm_GBps"] - 3.72e9 / 599e-6 / 1e9) < 5
    assert rows[(k, 0)]["calls"] == 2 and rows[(k, 1)]["calls"] == 2
    bad = rows[(S.short(OTHER), 0)]
    assert "hbm_GBps" not in bad and bad["rejected"]
    assert bad["in_infinity_cache"]
    table = S.table(out)
    assert "rejected (> peak)" in table
    for line in table.splitlines()[2:]:
        assert "16000" not in line


def test_dispatch_count_mismatch_gives_no_rate(tmp_path):
    p = str(tmp_path / "fp64_u")
    write_kt(p + "_kt", [(NAME, 262144, 60.0), (NAME, 262144, 600.0)])
    write_pmc(p + "_pmc1", [(NAME, 262144, {"FETCH_SIZE": 1e5, "WRITE_SIZE": 1.0})])
    dur, classes = S.durations(p + "_kt")
    out = S.summarize(dur, S.counters(p, classes))
    (row,) = out.values()
    assert row["size_class"] == -1 and "hbm_GBps" not in row
