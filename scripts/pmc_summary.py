#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc counter CSVs (one per pass) to per-kernel medians:
MFMA busy % of SIMD cycles, MFMA bf16 TFLOP/s, LDS bank-conflict ratio,
HBM fetch TB/s. Usage: pmc_summary.py <counter_collection.csv>..."""
import csv
import statistics as st
import sys
from collections import defaultdict

SIMDS = 256 * 4


def main(paths):
    vals = defaultdict(lambda: defaultdict(list))    # kernel -> counter -> per-dispatch values
    ncalls: dict = defaultdict(int)                  # kernel -> dispatches (max over passes)
    for p in paths:
        per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> sum
        names = {}
        for r in csv.DictReader(open(p)):
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            names[d] = r["Kernel_Name"].split("(")[0][:60]
            c, v = r["Counter_Name"], float(r["Counter_Value"])
            per[d]["_dur_s"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            # GRBM counters repeat per XCD instance: the kernel's cycles are the max
            per[d][c] = max(per[d][c], v) if c.startswith("GRBM_") else per[d][c] + v
        calls: dict = defaultdict(int)
        for d, cs in per.items():
            calls[names[d]] += 1
            for c, v in cs.items():
                vals[names[d]][c].append(v)
        for k, n in calls.items():
            ncalls[k] = max(ncalls[k], n)
    print(f"{'kernel':60s} {'MFMA busy %':>11s} {'bf16 TF/s':>9s} {'LDS confl':>9s} "
          f"{'HBM TB/s':>8s} {'us':>8s} {'calls':>7s}")
    # heaviest first: calls x median duration
    order = sorted(vals, key=lambda k: -ncalls[k] * st.median(vals[k]["_dur_s"] or [0.0]))
    for k in order:
        cs = vals[k]
        med = {c: st.median(v) for c, v in cs.items()}
        # the dispatch's own timestamps give its duration (GRBM_GUI_ACTIVE is
        # aggregated over hardware instances); cycles at the 2.4 GHz peak clock
        secs = med.get("_dur_s")
        out = [k]
        mfma = med.get("SQ_VALU_MFMA_BUSY_CYCLES")
        out.append(f"{100 * mfma / (secs * 2.4e9 * SIMDS):11.1f}" if mfma is not None and secs
                   else f"{'-':>11s}")
        mops = med.get("SQ_INSTS_VALU_MFMA_MOPS_BF16")
        out.append(f"{mops * 512 / secs / 1e12:9.1f}" if mops is not None and secs else f"{'-':>9s}")
        bc, act = med.get("SQ_LDS_BANK_CONFLICT"), med.get("SQ_LDS_IDX_ACTIVE")
        out.append(f"{bc / max(1.0, act - bc):9.3f}" if bc is not None and act else f"{'-':>9s}")
        fs = med.get("FETCH_SIZE")
        out.append(f"{fs * 1024 / secs / 1e12:8.2f}" if fs is not None and secs else f"{'-':>8s}")
        out.append(f"{secs * 1e6:8.1f}" if secs else f"{'-':>8s}")
        out.append(f"{ncalls[k]:7d}")
        print(f"{out[0]:60s} " + " ".join(out[1:]))


if __name__ == "__main__":
    main(sys.argv[1:])
