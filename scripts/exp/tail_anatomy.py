"""Per-step kernel anatomy of the LAST steps in a rocprofv3 kernel trace (the
timed replays of a projection script, after its tuning and warm-up): steps
are delimited by a marker kernel that runs once per step (default: the TP
argmax combine).

    python scripts/exp/tail_anatomy.py trace.csv [--steps 10] [--marker car_argmax]
"""
import argparse
import csv
import statistics as st
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="car_argmax")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < a.steps + 1:
        raise SystemExit(f"only {len(marks)} marker launches")
    spans, per = [], defaultdict(list)
    for s0, s1 in zip(marks[-a.steps - 1:-1], marks[-a.steps:]):
        step = rows[s0 + 1:s1 + 1]
        spans.append((step[-1][1] - step[0][0]) / 1e3)
        agg = defaultdict(list)
        for b, e, n in step:
            agg[n].append((e - b) / 1e3)
        for n, v in agg.items():
            per[n].append((len(v), sum(v), st.median(v)))
        launches = len(step)
    print(f"{a.steps} steps: median span {st.median(spans):.1f} us, {launches} launches per step")
    out = []
    for n, v in per.items():
        calls = st.median(x[0] for x in v)
        tot = st.median(x[1] for x in v)
        med = st.median(x[2] for x in v)
        out.append((tot, calls, med, n))
    for tot, calls, med, n in sorted(out, reverse=True):
        print(f"  {tot:9.1f} us/step {calls:6.0f} calls  median {med:7.2f} us  {n[:110]}")


if __name__ == "__main__":
    main()
