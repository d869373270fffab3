"""GPU occupancy over the last ``window`` seconds of a rocprofv3 kernel trace
(the bench's timed region): the fraction of time any kernel runs, and per
engine (LLM decode, Whisper decoder, prefill / encoder / other) the time its
kernels are running, alone or overlapped with the other engines."""
import csv
import gzip
import re
import sys

LLM = re.compile(r"skinny_fused_kernel<\d, \d+, \d, \d, \d, \d(, 0)?>|attn_decode_kernel<128|"
                 r"skinny_gemm_kernel<2, 1, 4>|masked_argmax_kernel<true>|step_fetch|step_publish")


def classify(name: str) -> str:
    if "skinny_fused_kernel<" in name:
        # LLM decode GEMMs stream 4-step groups (U=4) or are the 8B shapes; Whisper uses U=2
        u = re.search(r"skinny_fused_kernel<\d, \d+, (\d),", name)
        return "llm" if u and u.group(1) == "4" else "stt"
    if "attn_decode_kernel<128" in name or "skinny_gemm_kernel<2, 1, 4>" in name or \
            "step_fetch" in name or "step_publish" in name or "masked_argmax_kernel<true>" in name:
        return "llm"
    if "attn_decode_kernel<64" in name or "skinny_gemm_kernel<2, 1, 2>" in name or \
            "masked_argmax_kernel<false>" in name:
        return "stt"
    return "other"


def main(path: str, window: float = 3.0, skip_tail: float = 0.0) -> None:
    op = gzip.open if path.endswith(".gz") else open
    rows = []
    with op(path, "rt") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), classify(r["Kernel_Name"])))
    t_end = max(r[1] for r in rows) - int(skip_tail * 1e9)
    t0 = t_end - int(window * 1e9)
    rows = [r for r in rows if r[0] < t_end]
    ev = []
    for a, b, c in rows:
        if b <= t0:
            continue
        a, b = max(a, t0), min(b, t_end)
        ev.append((a, 1, c))
        ev.append((b, -1, c))
    ev.sort()
    act = {"llm": 0, "stt": 0, "other": 0}
    last = t0
    acc: dict = {}
    for t, d, c in ev:
        key = tuple(k for k in ("llm", "stt", "other") if act[k] > 0)
        acc[key] = acc.get(key, 0) + (t - last)
        act[c] += d
        last = t
    tot = t_end - t0
    print(f"window {window:.1f} s: busy {100 * (1 - acc.get((), 0) / tot):.1f}%")
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print(f"  {'+'.join(k) or 'idle':16s} {100 * v / tot:5.1f}%")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 3.0,
         float(sys.argv[3]) if len(sys.argv) > 3 else 0.0)
