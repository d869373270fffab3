"""Prefill projections at M ~ 318 (cold weights): hipBLASLt (F.linear) vs the
weight-streaming prefill GEMM (ops.prefill_gemm) incl. the slab sum, + error
vs fp32."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
M = int(os.environ.get("M", "318"))
res = []
for name, N, K, S in [("qkv", 6144, 4096, 2), ("o", 4096, 4096, 4), ("gate_up", 28672, 4096, 1),
                      ("down", 4096, 14336, 4), ("down_s8", 4096, 14336, 8), ("o_s8", 4096, 4096, 8)]:
    nw = max(2, min(8, int(1.5e9 // (N * K * 2))))
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nw)]
    wps = [ops.shuffle_weight(w) for w in ws]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ref = x.float() @ ws[0].float().t()

    def ours(i):
        if S == 1:
            return ops.prefill_gemm(x, wps[i])
        return ops.prefill_gemm(x, wps[i], S, slabs=True)

    def timeit(fn, n=30):
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
    y = ours(0)
    y = y.float() if S == 1 else y.sum(0)
    err = float((y - ref).norm() / ref.norm())
    res.append({"gemm": name, "M": M, "N": N, "K": K, "S": S, "hipblaslt_us": timeit(lambda i: F.linear(x, ws[i])),
                "ours_us": timeit(ours), "rel_err": round(err, 5)})
    print(json.dumps(res[-1]), flush=True)
    del ws, wps
