"""Per-pass anatomy of the LLM prompt prefill from a rocprofv3 kernel trace.

A Llama prefill pass is recognised by its causal flash-attention kernels
(``attn_prefill2_kernel<128, true>``, one per layer; the Whisper encoder's
are non-causal D = 64). For each pass: GPU span (first to last kernel of the
pass on its queue, so time other engines' kernels interleave is included),
summed kernel time of the pass's own queue inside the span, the idle gaps on
that queue, and the per-kernel breakdown (medians over passes).

  python scripts/prefill_anatomy.py kernel_trace.csv[.gz] [layers]
"""
import csv
import gzip
import statistics as st
import sys


# kernels only the Llama prefill launches (its hipBLASLt GEMMs are shared names)
LLM_PREFILL = ("attn_prefill2_kernel<128, true>", "rope_kv_append", "rmsnorm", "silu_mul",
               "gemm_prefill2_kernel", "slab_rope_append")


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path)


def main(path, layers=32):
    rows = []
    with _open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), (r["Queue_Id"], r["Stream_Id"]),
                         r["Kernel_Name"]))
    rows.sort()
    attn = [i for i, r in enumerate(rows) if "attn_prefill2_kernel<128, true>" in r[3]]
    if not attn:
        print("no LLM prefill passes in the trace")
        return
    # group consecutive causal-attention kernels into passes of `layers`
    passes, cur = [], [attn[0]]
    for i in attn[1:]:
        if len(cur) == layers:
            passes.append(cur)
            cur = []
        cur.append(i)
    if len(cur) == layers:
        passes.append(cur)
    spans, busy, gaps, per = [], [], [], {}
    for p in passes:
        q = rows[p[0]][2]
        # the pass runs from the layer-0 qkv (kernels before the first attention on
        # the same queue back to the previous pass / decode step) to the final norm:
        # approximate with the same-queue kernels between the first and last
        # attention, extended by one layer's share at each end
        lo, hi = rows[p[0]][0], rows[p[-1]][1]
        mine = [r for r in rows[p[0]:p[-1] + 1] if r[2] == q]
        k = sum(r[1] - r[0] for r in mine)
        layer = (hi - lo) / (layers - 1)
        spans.append((hi - lo + layer) / 1e3)
        busy.append(k * layers / (layers - 1) / 1e3)
        g = 0
        for a, b in zip(mine, mine[1:]):
            g += max(0, b[0] - a[1])
        gaps.append(g / 1e3)
        by = {}
        for r in mine:
            if not any(k in r[3] for k in LLM_PREFILL):
                continue          # hipBLASLt (shared with the encoder) and other engines' kernels
            name = r[3].split("(")[0][:90]
            by[name] = by.get(name, 0) + (r[1] - r[0])
        for n, v in by.items():
            per.setdefault(n, []).append(v / 1e3)
    print(f"llm prefill: {len(passes)} passes; median span {st.median(spans):.0f} us, "
          f"summed own-queue kernel time {st.median(busy):.0f} us, "
          f"own-queue idle gaps {st.median(gaps):.0f} us")
    for n, v in sorted(per.items(), key=lambda kv: -st.median(kv[1]))[:14]:
        print(f"  {st.median(v):9.1f} us/pass  {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 32)
