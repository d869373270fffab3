"""hipBLASLt (torch.nn.functional.linear) time vs M for the Llama-3-8B
prefill GEMM shapes (cold-ish weights: 4 copies cycled)."""
import json, os, sys, time
import torch
dev = torch.device("cuda")
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
out = {}
for name, (N, K) in shapes.items():
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(4)]
    for M in (300, 318, 320, 384, 512, 636, 640):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        for i in range(4):
            torch.nn.functional.linear(x, ws[i])
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(40):
            torch.nn.functional.linear(x, ws[i % 4])
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) / 40 * 1e3
        out[f"{name}:M{M}"] = [round(us, 1), round(2 * M * N * K / us / 1e6, 1)]
    del ws
print(json.dumps(out))
