"""Per-kernel counter summary of a tools/pmc_fp64.sh run (kernel-trace
--stats pass + SQ / FETCH_SIZE / WRITE_SIZE passes): duration, HBM bytes and
fraction of the 8 TB/s HBM peak, VALU instructions per wave, VALU busy, and
FP64 FLOP rate against the 78.6 TF vector FP64 peak.

Counter arithmetic (MI355X_MICROARCH.md "rocprofv3 PMC slots" / "HBM"):
  * SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES count quad-cycles;
    GRBM_GUI_ACTIVE is summed over the 8 XCDs, so one XCD's cycles of the
    dispatch are GRBM_GUI_ACTIVE / 8;
  * VALU busy = SQ_ACTIVE_INST_VALU * 4 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8),
    the share of SIMD cycles with a VALU instruction issuing (the ceiling of
    an FP64-VALU-bound kernel);
  * FP64 FLOPs = 64 * SQ_INSTS_VALU_FLOPS_FP64 (per-wave instruction counts,
    FMA counted twice, every lane assumed active), rate vs 78.6 TF
    (MI355X FP64 vector, spec);
  * HBM bytes = FETCH_SIZE * 1024 * 2 (gfx950 half-count of 128-B reads) +
    WRITE_SIZE * 1024.

  python profiles/summarize_kernels.py gpurun_out/fp64_r02 --out profiles/r02_fp64_kernels.json
"""
import argparse
import collections
import csv
import glob
import json
import os
import re

FP64_PEAK_TF = 78.6
HBM_PEAK_GBS = 8000.0
SIMDS = 1024


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("acm::", "")
    n = re.sub(r"Tag<(\w+)>", r"\1", n)
    return n.replace(", ", ",")[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="e.g. gpurun_out/fp64_r02 (reads <prefix>_kt, <prefix>_pmc*)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dur = {}
    for r in csv.DictReader(open(f"{a.prefix}_kt/kt_kernel_stats.csv")):
        if "acm::" in r["Name"]:
            dur[short(r["Name"])] = {"calls": int(r["Calls"]),
                                     "avg_us": float(r["AverageNs"]) / 1e3,
                                     "min_us": float(r["MinNs"]) / 1e3}
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(glob.glob(f"{a.prefix}_pmc*")):
        if not os.path.isdir(d):
            continue
        for r in csv.DictReader(open(os.path.join(d, "pmc_counter_collection.csv"))):
            if "acm::" not in r["Kernel_Name"]:
                continue
            k = short(r["Kernel_Name"])
            ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, c in ctr.items():
        med = {n: sorted(v)[len(v) // 2] for n, v in c.items()}
        row = {"counters_median": med}
        if k in dur:
            row.update(dur[k])
        us = dur.get(k, {}).get("avg_us")
        if "SQ_ACTIVE_INST_VALU" in med and med.get("GRBM_GUI_ACTIVE"):
            row["valu_busy"] = med["SQ_ACTIVE_INST_VALU"] * 4 / (
                SIMDS * med["GRBM_GUI_ACTIVE"] / 8)
        # per-CU unit busy / stall shares (TA, TD, TCP: one instance per CU,
        # 256 CUs, summed over instances; GRBM_GUI_ACTIVE summed over 8 XCDs)
        if med.get("GRBM_GUI_ACTIVE"):
            cyc = 256 * med["GRBM_GUI_ACTIVE"] / 8
            for cn, key in (("TA_TA_BUSY_sum", "ta_busy"),
                            ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "ta_addr_stalled_by_tc"),
                            ("TD_TD_BUSY_sum", "td_busy"), ("TD_TC_STALL_sum", "td_tc_stall"),
                            ("TCP_PENDING_STALL_CYCLES_sum", "tcp_pending_stall"),
                            ("TCP_TCR_TCP_STALL_CYCLES_sum", "tcp_tcr_stall")):
                if cn in med:
                    row[key] = med[cn] / cyc
        if med.get("SQ_WAVE_CYCLES"):
            for cn, key in (("SQ_WAIT_ANY", "wait_any_share"),
                            ("SQ_WAIT_INST_ANY", "wait_inst_share"),
                            ("SQ_ACTIVE_INST_ANY", "active_inst_share")):
                if cn in med:
                    row[key] = med[cn] / med["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in med and med.get("SQ_WAVES"):
            row["valu_insts_per_wave"] = med["SQ_INSTS_VALU"] / med["SQ_WAVES"]
        if "SQ_INSTS_VALU_FLOPS_FP64" in med and us:
            tf = 64 * med["SQ_INSTS_VALU_FLOPS_FP64"] / (us * 1e-6) / 1e12
            row["fp64_tflops"] = tf
            row["fp64_frac_of_peak"] = tf / FP64_PEAK_TF
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med and us:
            b = med["FETCH_SIZE"] * 1024 * 2 + med["WRITE_SIZE"] * 1024
            row["hbm_bytes"] = b
            row["hbm_GBps"] = b / (us * 1e-6) / 1e9
            row["hbm_frac_of_peak"] = row["hbm_GBps"] / HBM_PEAK_GBS
        out[k] = row
    json.dump(out, open(a.out, "w"), indent=1)
    print(f"| kernel | avg us | VALU busy | VALU inst/wave | FP64 TF (frac) | HBM GB/s (frac) "
          f"| TA busy | TD busy | wait / issue-stall / active |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k, r in sorted(out.items(), key=lambda kv: -kv[1].get("avg_us", 0)):
        f = lambda x, fmt: (fmt % x) if x is not None else "-"  # noqa: E731
        print(f"| {k} | {f(r.get('avg_us'), '%.1f')} | {f(r.get('valu_busy'), '%.2f')} | "
              f"{f(r.get('valu_insts_per_wave'), '%.0f')} | "
              f"{f(r.get('fp64_tflops'), '%.1f')} ({f(r.get('fp64_frac_of_peak'), '%.2f')}) | "
              f"{f(r.get('hbm_GBps'), '%.0f')} ({f(r.get('hbm_frac_of_peak'), '%.2f')}) | "
              f"{f(r.get('ta_busy'), '%.2f')} | {f(r.get('td_busy'), '%.2f')} | "
              f"{f(r.get('wait_any_share'), '%.2f')} / {f(r.get('wait_inst_share'), '%.2f')} / "
              f"{f(r.get('active_inst_share'), '%.2f')} |")


if __name__ == "__main__":
    main()
