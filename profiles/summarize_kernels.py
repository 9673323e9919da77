"""Per-kernel counter summary of a tools/gpu.sh `fp64` run (one kernel-trace
pass + SQ / TA-TD / FETCH_SIZE / WRITE_SIZE passes): duration, HBM bytes and
fraction of the 8 TB/s HBM peak, VALU instructions per wave, VALU busy, and
FP64 FLOP rate against the 78.6 TF vector FP64 peak.

Rows are (kernel, launch size): the counter rows of every pass and the
dispatches of the kernel-trace pass are grouped by the kernel's short name
AND its grid size, so a kernel the driver launches at several sizes (e.g.
the DS normal equations at 9.29M and 92.9M points) gets one row per size,
and bytes are never divided by a duration averaged over other sizes (the
r04 summaries did, and printed 1.45x the HBM peak).  A rate above the
physical peak (HBM 8 TB/s, FP64 78.6 TF) is not evidence: it is not printed
(the cell says "rejected") and the JSON row carries `rejected`.

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
  * A working set below the 256 MiB Infinity Cache (HBM bytes of one launch
    < 256 MiB) can be served from it across back-to-back launches: such a
    row's rate is labelled "effective (IC)", not HBM.

  python profiles/summarize_kernels.py gpurun_out/fp64_r05a --out profiles/r05a_fp64_kernels.json
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
IC_BYTES = 256 << 20


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("acm::", "")
    n = re.sub(r"Tag<(\w+)>", r"\1", n)
    return n.replace(", ", ",")[:70]


def size_classes(durs, ratio=1.5):
    """Occurrence index -> class id for one (kernel, grid) dispatch sequence:
    persistent kernels keep their grid size whatever the problem size, so
    the launches of one grid are split further by duration (sorted, a new
    class wherever the next duration is more than `ratio` x the previous)."""
    order = sorted(range(len(durs)), key=lambda i: durs[i])
    cls, c, prev = [0] * len(durs), 0, None
    for i in order:
        if prev is not None and durs[i] > ratio * prev:
            c += 1
        cls[i] = c
        prev = durs[i]
    return cls


def waves_per_simd(r):
    """register-limited waves per SIMD (512 VGPRs + AGPRs per lane-slot on
    CDNA3/4 in 8-register granules, at most 8 waves), ignoring LDS"""
    v = r["vgprs"] + r["agprs"]
    if v <= 0:
        return None
    v = (v + 7) // 8 * 8
    return min(8, 512 // v)


def durations(kt_dir):
    """(short name, grid size, size class) -> {calls, avg_us, min_us} from the
    per-dispatch kernel trace (the --stats table aggregates over launch
    sizes), plus the occurrence -> class map of every (name, grid)."""
    acc = collections.defaultdict(list)
    res = {}
    for r in csv.DictReader(open(os.path.join(kt_dir, "kt_kernel_trace.csv"))):
        if "acm::" not in r["Kernel_Name"]:
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        acc[(short(r["Kernel_Name"]), grid)].append(
            (int(r["Dispatch_Id"]),
             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
        res[(short(r["Kernel_Name"]), grid)] = {
            # rocprofv3 (ROCm 7.2) reports gfx950 wave64 VGPR_Count as HALF the
            # allocated registers: k_tsqr<DS, +error> 52 vs the compiler's 104
            # (-Rpass-analysis=kernel-resource-usage, occupancy 4), KB normal
            # equations 68 vs 134 (occupancy 3), k_fov_grid_pl 80 vs 153 -- so
            # the allocation is taken as twice the trace's figure
            "vgprs": 2 * int(r.get("VGPR_Count") or 0),
            "agprs": 2 * int(r.get("Accum_VGPR_Count") or 0),
            "sgprs": int(r.get("SGPR_Count") or 0), "lds_bytes": int(r.get("LDS_Block_Size") or 0),
            "block": int(r.get("Workgroup_Size_X") or 0)}
    out, classes = {}, {}
    for k, v in acc.items():
        v.sort()
        durs = [d for _, d in v]
        cls = size_classes(durs)
        classes[k] = cls
        for c in set(cls):
            ds = [d for d, ci in zip(durs, cls) if ci == c]
            out[k + (c,)] = {"calls": len(ds), "avg_us": sum(ds) / len(ds), "min_us": min(ds),
                             **res[k], "waves_per_simd_max": waves_per_simd(res[k])}
    return out, classes


def counters(prefix, classes):
    """(short name, grid size, size class) -> counter name -> per-dispatch
    values.  Every pass runs the same driver, so the k-th dispatch of a
    (name, grid) in a counter pass is the k-th of the kernel-trace pass and
    takes its size class; a pass whose dispatch count differs is grouped as
    one class -1 (sizes unknown: no rate is derived from it)."""
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(glob.glob(f"{prefix}_pmc*")):
        f = os.path.join(d, "pmc_counter_collection.csv")
        if not os.path.isdir(d) or not os.path.exists(f):
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(dict))
        for r in csv.DictReader(open(f)):
            if "acm::" not in r["Kernel_Name"]:
                continue
            k = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            per[k][int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
        for k, disp in per.items():
            ids = sorted(disp)
            cls = classes.get(k)
            if cls is None or len(cls) != len(ids):
                cls = [-1] * len(ids)
            for c, i in zip(cls, ids):
                for name, val in disp[i].items():
                    ctr[k + (c,)][name].append(val)
    return ctr


def summarize(dur, ctr):
    out = {}
    for key, c in ctr.items():
        med = {n: sorted(v)[len(v) // 2] for n, v in c.items()}
        row = {"kernel": key[0], "grid_size": key[1], "size_class": key[2],
               "counters_median": med}
        if key in dur:
            row.update(dur[key])
        us = dur.get(key, {}).get("avg_us")
        rejected = []
        if "SQ_ACTIVE_INST_VALU" in med and med.get("GRBM_GUI_ACTIVE"):
            row["valu_busy"] = med["SQ_ACTIVE_INST_VALU"] * 4 / (
                SIMDS * med["GRBM_GUI_ACTIVE"] / 8)
        # per-CU unit busy / stall shares (TA, TD, TCP: one instance per CU,
        # 256 CUs, summed over instances; GRBM_GUI_ACTIVE summed over 8 XCDs)
        if med.get("GRBM_GUI_ACTIVE"):
            cyc = 256 * med["GRBM_GUI_ACTIVE"] / 8
            for cn, k in (("TA_TA_BUSY_sum", "ta_busy"),
                          ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "ta_addr_stalled_by_tc"),
                          ("TD_TD_BUSY_sum", "td_busy"), ("TD_TC_STALL_sum", "td_tc_stall"),
                          ("TCP_PENDING_STALL_CYCLES_sum", "tcp_pending_stall"),
                          ("TCP_TCR_TCP_STALL_CYCLES_sum", "tcp_tcr_stall")):
                if cn in med:
                    row[k] = med[cn] / cyc
        if med.get("SQ_WAVE_CYCLES"):
            for cn, k in (("SQ_WAIT_ANY", "wait_any_share"),
                          ("SQ_WAIT_INST_ANY", "wait_inst_share"),
                          ("SQ_ACTIVE_INST_ANY", "active_inst_share")):
                if cn in med:
                    row[k] = med[cn] / med["SQ_WAVE_CYCLES"]
        if med.get("SQ_WAVES"):
            row["waves"] = med["SQ_WAVES"]
            if "SQ_INSTS_VALU" in med:
                row["valu_insts_per_wave"] = med["SQ_INSTS_VALU"] / med["SQ_WAVES"]
            if "SQ_INSTS_VALU_FLOPS_FP64" in med:
                row["fp64_insts_per_wave"] = med["SQ_INSTS_VALU_FLOPS_FP64"] / med["SQ_WAVES"]
        if "SQ_INSTS_VALU_FLOPS_FP64" in med and us:
            tf = 64 * med["SQ_INSTS_VALU_FLOPS_FP64"] / (us * 1e-6) / 1e12
            if tf > FP64_PEAK_TF:
                rejected.append(f"FP64 {tf:.1f} TF > {FP64_PEAK_TF} peak")
            else:
                row["fp64_tflops"] = tf
                row["fp64_frac_of_peak"] = tf / FP64_PEAK_TF
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            b = med["FETCH_SIZE"] * 1024 * 2 + med["WRITE_SIZE"] * 1024
            row["hbm_bytes"] = b
            row["in_infinity_cache"] = b < IC_BYTES
            if us:
                gbs = b / (us * 1e-6) / 1e9
                if gbs > HBM_PEAK_GBS:
                    rejected.append(f"HBM {gbs:.0f} GB/s > {HBM_PEAK_GBS:.0f} peak")
                else:
                    row["hbm_GBps"] = gbs
                    row["hbm_frac_of_peak"] = gbs / HBM_PEAK_GBS
        if rejected:
            row["rejected"] = rejected
        out[f"{key[0]} @grid {key[1]} #{key[2]}"] = row
    return out


def table(out):
    lines = ["| kernel | grid | calls | avg us | VGPR (waves/SIMD) | VALU busy | VALU inst/wave | "
             "FP64 TF (frac) | HBM GB/s (frac) | TA busy | TD busy | wait / issue-stall / active |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    f = lambda x, fmt: (fmt % x) if x is not None else "-"  # noqa: E731
    for _, r in sorted(out.items(), key=lambda kv: -kv[1].get("avg_us", 0)):
        hbm = f(r.get("hbm_GBps"), "%.0f") + f" ({f(r.get('hbm_frac_of_peak'), '%.2f')})"
        if any(x.startswith("HBM") for x in r.get("rejected", [])):
            hbm = "rejected (> peak)"
        elif r.get("in_infinity_cache") and r.get("hbm_GBps") is not None:
            hbm += " effective (IC)"
        fp = f(r.get("fp64_tflops"), "%.1f") + f" ({f(r.get('fp64_frac_of_peak'), '%.2f')})"
        if any(x.startswith("FP64") for x in r.get("rejected", [])):
            fp = "rejected (> peak)"
        lines.append(
            f"| {r['kernel']} | {r['grid_size']}"
            f"{'' if r['size_class'] == 0 else ' #%d' % r['size_class']} | {r.get('calls', '-')} | "
            f"{f(r.get('avg_us'), '%.1f')} | {r.get('vgprs', '-')} "
            f"({r.get('waves_per_simd_max', '-')}) | {f(r.get('valu_busy'), '%.2f')} | "
            f"{f(r.get('valu_insts_per_wave'), '%.0f')} | {fp} | {hbm} | "
            f"{f(r.get('ta_busy'), '%.2f')} | {f(r.get('td_busy'), '%.2f')} | "
            f"{f(r.get('wait_any_share'), '%.2f')} / {f(r.get('wait_inst_share'), '%.2f')} / "
            f"{f(r.get('active_inst_share'), '%.2f')} |")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="e.g. gpurun_out/fp64_r05a (reads <prefix>_kt, <prefix>_pmc*)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dur, classes = durations(f"{a.prefix}_kt")
    out = summarize(dur, counters(a.prefix, classes))
    json.dump(out, open(a.out, "w"), indent=1)
    print(table(out))


if __name__ == "__main__":
    main()
