"""Weight-streaming GEMM with in-launch split-K (ops.gemm_ws splits=S) vs the
current prompt-pass pick (ops.proj) on the Llama-3-8B projections, cold weights
(a ring of weight copies larger than the Infinity Cache), us per call.

    python scripts/exp/ws_splitk_bench.py [--ms 300,128,600]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from loqa_hub_amd import ops  # noqa: E402

LLAMA = {"qkv": (6144, 4096, "bf16"), "o": (4096, 4096, "resid"), "gu": (28672, 4096, "swiglu"),
         "down": (4096, 14336, "resid")}


def timeit(fn, n_w, iters=30):
    for i in range(3):
        fn(i % n_w)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n_w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="300,128,600")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for M in map(int, a.ms.split(",")):
        for name, (N, K, epi) in LLAMA.items():
            n_w = max(2, (768 << 20) // (N * K * 2))
            ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(n_w)]
            x = torch.randn(M, K, device=dev).bfloat16()
            res = torch.randn(M, N, device=dev).bfloat16()
            kw = {"residual": res} if epi == "resid" else {}
            row = {"M": M, "shape": name, "proj_us": round(timeit(
                lambda i: ops.proj(x, ws[i], epi=epi, **kw), n_w), 1)}
            for depth in (0, 1):
                if depth == 1 and M > 256:
                    continue
                for S in (1, 2, 3, 4, 6, 8):
                    if K // 64 < 2 * S:
                        continue
                    row[f"ws{depth}_S{S}"] = round(timeit(
                        lambda i: ops.gemm_ws(x, ws[i], epi=epi, depth=depth, splits=S, **kw), n_w), 1)
            print(json.dumps(row), flush=True)
            del ws


if __name__ == "__main__":
    main()
