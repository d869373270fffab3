"""Per-decode-step anatomy from a rocprofv3 kernel trace.

Graph replays are not reliably attributed to one (queue, stream) pair, so the
steps of an engine are picked out by kernel NAME instead: ``llm`` takes the
Llama-3-8B decode kernels (fused GEMMs with 4-step prefetch groups, D = 128
decode attention, the 4-wide lm_head GEMM), ``stt`` the Whisper decoder's
(2-step groups, D = 64 attention, its lm_head). A step ends at the engine's
lm_head GEMM. Per step: GPU span (first start to last end, so time the other
engine's kernels interleave is included), summed kernel time, and the per-kernel
breakdown (medians over steps)."""
import csv
import re
import statistics as st
import sys

ENGINES = {
    "llm": (re.compile(r"skinny_fused_kernel<\d, \d, 4, |attn_decode_kernel<128|skinny_gemm_kernel<2, 1, 4>"),
            "skinny_gemm_kernel<2, 1, 4>"),
    "stt": (re.compile(r"skinny_fused_kernel<\d, \d, 2, |attn_decode_kernel<64|skinny_gemm_kernel<2, 1, 2>"),
            "skinny_gemm_kernel<2, 1, 2>"),
    # a tensor-parallel rank's graph-replayed decode step alone on the GPU
    # (scripts/config5_projection.py): every kernel, a step ends at the
    # vocab-parallel argmax combine
    "tp": (re.compile(r"."), "car_argmax_kernel"),
}


def main(path, engine="llm"):
    pat, delim = ENGINES[engine]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if pat.search(r["Kernel_Name"]):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    steps, cur = [], []
    for r in rows:
        cur.append(r)
        if delim in r[2]:
            steps.append(cur)
            cur = []
    # decode steps only (tuning sweeps and prefill chunks have other shapes)
    lo, hi = (100, 400) if engine != "tp" else (50, 2000)
    steps = [s for s in steps if lo <= len(s) <= hi]
    if not steps:
        print(f"{engine}: no steps found")
        return
    span = [(s[-1][1] - s[0][0]) / 1e3 for s in steps]
    busy = [sum(r[1] - r[0] for r in s) / 1e3 for s in steps]
    by = {}
    for s in steps:
        for r in s:
            n = r[2].split("(")[0][:60]
            by.setdefault(n, []).append((r[1] - r[0]) / 1e3)
    print(f"{engine}: {len(steps)} steps; median span {st.median(span):.1f} us, "
          f"summed kernel time {st.median(busy):.1f} us, {st.median([len(s) for s in steps]):.0f} launches")
    # host turnaround: last kernel of a step -> first kernel of the next one
    # (sampling read-back, grammar advance, metadata, graph launch)
    gaps = [(b[0][0] - a[-1][1]) / 1e3 for a, b in zip(steps, steps[1:])]
    gaps = [g for g in gaps if 0 <= g < 5000]
    if gaps:
        print(f"   step-to-step gap: median {st.median(gaps):.1f} us, p90 "
              f"{sorted(gaps)[int(0.9 * (len(gaps) - 1))]:.1f} us")
    per = sorted(((sum(v) / len(steps), n, len(v) / len(steps), st.median(v)) for n, v in by.items()),
                 reverse=True)
    for tot, n, c, med in per[:12]:
        print(f"   {tot:8.1f} us/step  {c:5.1f} calls  median {med:6.1f} us  {n}")


if __name__ == "__main__":
    main(*sys.argv[1:])
