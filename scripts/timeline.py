"""Phase breakdown of a rocprofv3 kernel trace: groups consecutive kernels into
phases (STT encoder / STT decoder / LLM prefill / LLM decode) by kernel family,
reports busy time vs wall span and the idle gaps between kernels."""
import csv
import sys
from collections import defaultdict


def family(name: str) -> str:
    if "skinny_gemm" in name or "slab_" in name or "attn_decode" in name or "masked_argmax" in name \
            or "argmax_unpack" in name:
        return "llm_decode"
    if "attn_fwd_kernel<128" in name or "rmsnorm" in name or "rope_kv_append" in name or \
            "silu_mul" in name:
        return "llm_prefill"
    if "attn_fwd_kernel<64, false, false>" in name or "im2col" in name or "log_mel" in name or \
            "gelu_bias" in name:
        return "stt_encode"
    if "attn_fwd_kernel<64" in name or "layernorm" in name or "attn_combine" in name:
        return "stt_decode"
    return "other"


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    busy = sum(e - s for s, e, _ in rows)
    print(f"span {(t1 - t0) / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms ({100 * busy / (t1 - t0):.1f}%),"
          f" {len(rows)} kernels")
    fam_busy = defaultdict(int)
    fam_gap = defaultdict(int)
    gaps = []
    prev_end = rows[0][0]
    prev_fam = None
    for s, e, n in rows:
        fm = family(n)
        fam_busy[fm] += e - s
        g = s - prev_end
        if g > 0:
            fam_gap[fm] += g
            gaps.append((g, prev_fam, fm))
        prev_end = max(prev_end, e)
        prev_fam = fm
    for fm in sorted(fam_busy, key=lambda k: -fam_busy[k]):
        print(f"  {fm:12s} busy {fam_busy[fm] / 1e6:9.1f} ms   idle-before {fam_gap[fm] / 1e6:9.1f} ms")
    gaps.sort(reverse=True)
    print("largest gaps (ms, prev -> next):")
    for g, a, b in gaps[:15]:
        print(f"  {g / 1e6:8.2f}  {a} -> {b}")
    big = [g for g, _, _ in gaps if g > 100_000]
    print(f"gaps > 0.1 ms: {len(big)} totalling {sum(big) / 1e6:.1f} ms; "
          f"gaps <= 0.1 ms total {sum(g for g, _, _ in gaps if g <= 100_000) / 1e6:.1f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
