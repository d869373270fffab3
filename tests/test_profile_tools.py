"""The profile reducers that turn rocprofv3 CSVs into the files under
``profiles/`` (scripts/pmc_summary.py, scripts/kernel_summary.py), on
synthetic CSVs of the same columns."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, fields, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        w.writerows(rows)


def _run(*args):
    p = subprocess.run([sys.executable, *args], cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    return p.stdout.splitlines()


def test_pmc_summary_two_passes(tmp_path):
    """Counters of two passes merge per kernel; GRBM counters take the max
    over instances, SQ counters sum; calls are per pass, not doubled; the
    heaviest kernel (calls x median time) comes first."""
    fields = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp",
              "End_Timestamp"]
    a, b = [], []
    for d in range(4):     # gemm: 4 dispatches of 10 us, 2 XCD instances of each counter
        for inst in range(2):
            a += [dict(Dispatch_Id=d, Kernel_Name="gemm(Args)", Counter_Name=c, Counter_Value=v,
                       Start_Timestamp=0, End_Timestamp=10000)
                  for c, v in (("SQ_VALU_MFMA_BUSY_CYCLES", 6144.0), ("SQ_LDS_IDX_ACTIVE", 100.0),
                               ("SQ_LDS_BANK_CONFLICT", 0.0), ("GRBM_GUI_ACTIVE", 24000.0))]
            b.append(dict(Dispatch_Id=d, Kernel_Name="gemm(Args)", Counter_Name="FETCH_SIZE",
                          Counter_Value=25000.0, Start_Timestamp=0, End_Timestamp=10000))
    for d in range(4, 5):  # attn: 1 dispatch of 5 us with 2-way conflicts
        a += [dict(Dispatch_Id=d, Kernel_Name="attn(Args)", Counter_Name=c, Counter_Value=v,
                   Start_Timestamp=0, End_Timestamp=5000)
              for c, v in (("SQ_LDS_IDX_ACTIVE", 200.0), ("SQ_LDS_BANK_CONFLICT", 100.0))]
    pa, pb = tmp_path / "a_counter_collection.csv", tmp_path / "b_counter_collection.csv"
    _write(pa, fields, a)
    _write(pb, fields, b)
    out = _run("scripts/pmc_summary.py", str(pa), str(pb))
    assert out[0].split()[0] == "kernel" and out[0].split()[-1] == "calls"
    gemm, attn = out[1].split(), out[2].split()
    assert gemm[0] == "gemm" and attn[0] == "attn"
    # columns: kernel grid MFMA% bf16TF LDScf us fetchx2 rdreq TB/s algo meas/algo label calls
    # MFMA busy: 2 x 6144 cycles over 10 us x 2.4 GHz x 1024 SIMDs = 0.05 %
    assert abs(float(gemm[2]) - 100 * 12288 / (10e-6 * 2.4e9 * 1024)) < 0.05
    assert float(gemm[4]) == 0.0 and gemm[-1] == "4"
    # FETCH_SIZE reports half of a streaming read's bytes on gfx950: 2 x 2 x
    # 25000 KiB per dispatch (two instances summed), doubled -> 204.8 MB in 10 us
    assert abs(float(gemm[6]) - 4 * 25000 * 1024 / 1e6) < 0.01
    assert abs(float(gemm[8]) - 4 * 25000 * 1024 / 10e-6 / 1e12) < 0.01
    assert float(attn[4]) == 1.0 and attn[-1] == "1"      # 100 extra / 100 conflict-free cycles


def test_pmc_summary_shapes_and_rdreq(tmp_path):
    """Rows split by grid (one template, two shapes); TCC_EA0_RDREQ_sum x 128 B
    is the measured read bytes when present; pmc_gemm.py shapes add the
    algorithmic bytes and the ratio."""
    import json
    fields = ["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value",
              "Start_Timestamp", "End_Timestamp"]
    tpl = "void skinny_fused_kernel<2, 1, 4, 1, 2, 0, 0>(FusedArgs)"
    rows = []
    for d, (grid, req) in enumerate([(65536, 1e6), (65536, 1e6), (32768, 5e5)]):
        rows.append(dict(Dispatch_Id=d, Kernel_Name=tpl, Grid_Size=grid, Counter_Name="TCC_EA0_RDREQ_sum",
                         Counter_Value=req, Start_Timestamp=0, End_Timestamp=20000))
    pa = tmp_path / "c_counter_collection.csv"
    _write(pa, fields, rows)
    shapes = [{"label": "down", "mode": "resid", "grid": 65536, "algorithmic_bytes": 128e6,
               "layout": [2, 2, 1]}]
    sp = tmp_path / "shapes.json"
    sp.write_text(json.dumps(shapes))
    out = _run("scripts/pmc_summary.py", "--shapes", str(sp), str(pa))
    # the kernel name (with spaces) fills the first 60 columns
    big, small = out[1][61:].split(), out[2][61:].split()
    assert big[0] == "65536" and small[0] == "32768" and big[-1] == "2"
    assert abs(float(big[6]) - 128.0) < 1e-6             # 1e6 requests x 128 B
    assert big[10] == "down" and abs(float(big[9]) - 1.0) < 1e-6
    assert small[10] == "-"


def test_kernel_summary_top_n(tmp_path):
    fields = ["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"]
    rows = [dict(Name="small", Calls=10, TotalDurationNs=1e6, AverageNs=1e5, Percentage=10.0),
            dict(Name="big", Calls=3, TotalDurationNs=9e6, AverageNs=3e6, Percentage=90.0)]
    p = tmp_path / "k_kernel_stats.csv"
    _write(p, fields, rows)
    out = _run("scripts/kernel_summary.py", str(p), "1")
    assert out[0].startswith("total kernel time: 10.00 ms over 13 dispatches")
    assert len(out) == 3 and out[2].split()[-1] == "big"
