"""Prefill GEMM (ops.prefill_gemm2, every wave layout) vs hipBLASLt (F.linear) on the Llama-3-8B prefill projections and the Whisper
encoder projections, cold weights (rotated over copies that exceed the
256 MB Infinity Cache), plus relative error vs fp32.

  M=318 python scripts/exp/prefill_gemm2_bench.py
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
M = int(os.environ.get("M", "318"))
MW = int(os.environ.get("MW", "1500"))
SHAPES = [("qkv", M, 6144, 4096, [1, 2, 4]), ("o", M, 4096, 4096, [2, 4, 8]),
          ("gate_up", M, 28672, 4096, [1]), ("down", M, 4096, 14336, [4, 8]),
          ("enc_qkv", MW, 3840, 1280, [1, 2]), ("enc_o", MW, 1280, 1280, [1, 2, 4]),
          ("enc_fc1", MW, 5120, 1280, [1]), ("enc_fc2", MW, 1280, 5120, [2, 4])]
only = os.environ.get("ONLY")


def timeit(fn, nw, n=30):
    for i in range(3):
        fn(i % nw)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(n):
        fn(i % nw)
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / n * 1e3, 1)


for name, m, N, K, splits in SHAPES:
    if only and name not in only.split(","):
        continue
    nw = max(2, min(8, int(1.2e9 // (N * K * 2))))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nw)]
    wps = [ops.shuffle_weight(w) for w in ws]
    x = torch.randn(m, K, device=dev, dtype=torch.bfloat16)
    ref = x.float() @ ws[0].float().t()
    row = {"gemm": name, "M": m, "N": N, "K": K,
           "hipblaslt_us": timeit(lambda i: F.linear(x, ws[i]), nw)}
    tflop = 2 * m * N * K / 1e6
    for lay, (rbw, ft, wm) in ops.PREFILL2_LAYOUTS.items():
        if N % (16 * ft * (4 // wm)):
            continue
        for S in splits:
            if K % (64 * S):
                continue
            epi = "bf16" if S == 1 else "slabs"
            y = ops.prefill_gemm2(x, wps[0], S, epi=epi, layout=lay)
            y = y.float() if S == 1 else y.sum(0)
            err = float((y - ref).norm() / ref.norm())
            us = timeit(lambda i: ops.prefill_gemm2(x, wps[i], S, epi=epi, layout=lay), nw)
            row[f"v2_l{lay}_s{S}_us"] = us
            row[f"v2_l{lay}_s{S}_err"] = round(err, 5)
    best = min((v, k) for k, v in row.items() if k.startswith("v2_") and k.endswith("_us"))
    row["best"] = best[1]
    row["best_tflops"] = round(tflop / best[0], 1)
    row["hipblaslt_tflops"] = round(tflop / row["hipblaslt_us"], 1)
    print(json.dumps(row), flush=True)
    del ws, wps
    torch.cuda.empty_cache()
