#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc counter CSVs (one per pass) to per-kernel medians:
MFMA busy % of SIMD cycles, MFMA bf16 TFLOP/s, LDS bank-conflict ratio and the
bytes the kernel read from memory.

Rows are per (kernel, grid size), not per template: one template runs several
GEMM shapes (qkv / o / down share ``skinny_fused_kernel`` instances), and a
median over all of them describes none.

Read bytes, two independent counters:
* ``FETCH_SIZE`` (KiB, rocprofv3 derived from TCC_EA0_RDREQ): on gfx950 it
  reports exactly HALF the bytes of a wide (16-B-per-lane) coalesced streaming
  read - 128-B requests tallied at 64 B (MI355X_MICROARCH.md, HBM) - so the
  table doubles it ("fetch x2");
* ``TCC_EA0_RDREQ_sum`` x 128 B (the request count itself) when that pass ran.
With ``--shapes`` (the JSON of scripts/pmc_gemm.py) each matching row also
gets its ALGORITHMIC bytes and the measured / algorithmic ratio.

Usage: pmc_summary.py [--shapes shapes.json] <counter_collection.csv>..."""
import argparse
import csv
import json
import re
import statistics as st
from collections import defaultdict

SIMDS = 256 * 4
_TPL = re.compile(r"skinny_fused_kernel<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+)")


def shape_label(shapes: list, name: str, grid: str):
    """(label, algorithmic bytes) of a pmc_gemm.py dispatch - same grid, same
    tile rows / waves along rows / epilogue in the template - or None."""
    m = _TPL.search(name)
    if m is None:
        return None
    rt, wr, mode = int(m.group(1)), int(m.group(4)), int(m.group(5))
    hits = [e for e in shapes
            if str(e["grid"]) == grid and rt == e["layout"][1] and wr == e["layout"][2]
            and mode == {"rope": 3, "resid": 2, "silu": 1}[e["mode"]]]
    if not hits:
        return None
    return "|".join(e["label"] for e in hits), hits[0]["algorithmic_bytes"]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=None)
    ap.add_argument("csv", nargs="+")
    a = ap.parse_args(argv)
    shapes = json.load(open(a.shapes)) if a.shapes else []
    vals = defaultdict(lambda: defaultdict(list))    # (kernel, grid) -> counter -> per-dispatch values
    ncalls: dict = defaultdict(int)
    for p in a.csv:
        per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> sum
        keys = {}
        for r in csv.DictReader(open(p)):
            d = r.get("Dispatch_Id") or r.get("Correlation_Id")
            keys[d] = (r["Kernel_Name"].split("(")[0][:60], r.get("Grid_Size", "?"))
            c, v = r["Counter_Name"], float(r["Counter_Value"])
            per[d]["_dur_s"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            # GRBM counters repeat per XCD instance: the kernel's cycles are the max
            per[d][c] = max(per[d][c], v) if c.startswith("GRBM_") else per[d][c] + v
        calls: dict = defaultdict(int)
        for d, cs in per.items():
            calls[keys[d]] += 1
            for c, v in cs.items():
                vals[keys[d]][c].append(v)
        for k, n in calls.items():
            ncalls[k] = max(ncalls[k], n)
    hdr = (f"{'kernel':60s} {'grid':>7s} {'MFMA %':>6s} {'bf16TF':>6s} {'LDScf':>6s} "
           f"{'us':>7s} {'fetchx2 MB':>10s} {'rdreq MB':>8s} {'TB/s':>5s} {'algo MB':>8s} "
           f"{'meas/algo':>9s} {'label':>8s} {'calls':>6s}")
    print(hdr)
    order = sorted(vals, key=lambda k: -ncalls[k] * st.median(vals[k]["_dur_s"] or [0.0]))
    for k in order:
        cs = vals[k]
        med = {c: st.median(v) for c, v in cs.items()}
        secs = med.get("_dur_s")
        mfma = med.get("SQ_VALU_MFMA_BUSY_CYCLES")
        mops = med.get("SQ_INSTS_VALU_MFMA_MOPS_BF16")
        bc, act = med.get("SQ_LDS_BANK_CONFLICT"), med.get("SQ_LDS_IDX_ACTIVE")
        fs = med.get("FETCH_SIZE")
        rq = med.get("TCC_EA0_RDREQ_sum", med.get("TCC_EA0_RDREQ"))
        fetch_b = 2 * fs * 1024 if fs is not None else None
        rq_b = 128 * rq if rq is not None else None
        meas = rq_b if rq_b is not None else fetch_b
        lab = shape_label(shapes, k[0], k[1]) if shapes else None
        cols = [
            f"{100 * mfma / (secs * 2.4e9 * SIMDS):6.1f}" if mfma is not None and secs else f"{'-':>6s}",
            f"{mops * 512 / secs / 1e12:6.1f}" if mops is not None and secs else f"{'-':>6s}",
            f"{bc / max(1.0, act - bc):6.3f}" if bc is not None and act else f"{'-':>6s}",
            f"{secs * 1e6:7.1f}" if secs else f"{'-':>7s}",
            f"{fetch_b / 1e6:10.2f}" if fetch_b is not None else f"{'-':>10s}",
            f"{rq_b / 1e6:8.2f}" if rq_b is not None else f"{'-':>8s}",
            f"{meas / secs / 1e12:5.2f}" if meas is not None and secs else f"{'-':>5s}",
            f"{lab[1] / 1e6:8.2f}" if lab else f"{'-':>8s}",
            f"{meas / lab[1]:9.3f}" if lab and meas is not None else f"{'-':>9s}",
            f"{lab[0]:>8s}" if lab else f"{'-':>8s}",
            f"{ncalls[k]:6d}"]
        print(f"{k[0]:60s} {k[1]:>7s} " + " ".join(cols))


if __name__ == "__main__":
    main()
