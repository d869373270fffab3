"""Per-decode-step anatomy from a rocprofv3 kernel trace: for the stream that
runs the Llama gate|up GEMM, split the kernel sequence into steps at each
masked argmax and report, per step, the GPU span, the summed kernel time,
the in-step gaps and the host gap before the next step (median over steps)."""
import csv
import statistics as st
import sys


def main(path, key="skinny_fused_kernel<2, 1, 4, 4, 1, 1>"):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         (r["Queue_Id"], r["Stream_Id"])))
    rows.sort()
    qs = {r[3] for r in rows if key in r[2]}
    for q in sorted(qs):
        ks = [r for r in rows if r[3] == q]
        steps, cur = [], []
        for r in ks:
            cur.append(r)
            if "masked_argmax" in r[2] or "argmax" in r[2]:
                steps.append(cur)
                cur = []
        steps = [s for s in steps if sum(key in r[2] for r in s) >= 8]
        if not steps:
            continue
        span = [(s[-1][1] - s[0][0]) / 1e3 for s in steps]
        busy = [sum(r[1] - r[0] for r in s) / 1e3 for s in steps]
        host = [(b[0][0] - a[-1][1]) / 1e3 for a, b in zip(steps, steps[1:])]
        by = {}
        for s in steps:
            for r in s:
                n = r[2].split("(")[0][:60]
                by.setdefault(n, []).append((r[1] - r[0]) / 1e3)
        print(f"queue {q}: {len(steps)} steps; median span {st.median(span):.1f} us, "
              f"busy {st.median(busy):.1f} us, host gap {st.median(host) if host else 0:.1f} us "
              f"(p90 {sorted(host)[int(0.9 * len(host))] if host else 0:.1f})")
        per = sorted(((sum(v) / len(steps), n, len(v) / len(steps), st.median(v)) for n, v in by.items()),
                     reverse=True)
        for tot, n, c, med in per[:14]:
            print(f"   {tot:8.1f} us/step  {c:5.1f} calls  median {med:6.1f} us  {n}")


if __name__ == "__main__":
    main(*sys.argv[1:])
