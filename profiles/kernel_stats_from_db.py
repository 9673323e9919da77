"""Summarise a rocprofv3 --kernel-trace results.db (sqlite) into per-kernel
CSV rows: name, calls, average / min / max duration (us), VGPRs, scratch.

  python profiles/kernel_stats_from_db.py gpurun_out/<dir>/<name>_results.db [filter]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), avg(end-start), min(end-start), max(end-start), "
        "max(vgpr_count), max(scratch_size) from kernels where name like ? "
        "group by name order by name", (f"%{filt}%",)).fetchall()
    print("kernel,calls,avg_us,min_us,max_us,vgpr,scratch_bytes")
    for n, k, a, lo, hi, vg, sc in rows:
        n = n.split("(")[0].replace(",", ";")
        print(f"{n},{k},{a / 1e3:.1f},{lo / 1e3:.1f},{hi / 1e3:.1f},{vg},{sc}")


if __name__ == "__main__":
    main()
