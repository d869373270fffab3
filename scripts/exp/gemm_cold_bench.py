"""hipBLASLt (F.linear) on the Llama-3-8B prefill projections with COLD
weights (cycled over copies that outgrow the 256 MB Infinity Cache, as in a
real 32-layer pass) vs hot (one copy re-read), M = prompt tokens."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

dev = torch.device("cuda")
M = int(os.environ.get("M", "318"))
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
res = {}
for name, (N, K) in shapes.items():
    ncp = max(2, -(-(1 << 30) // (N * K * 2)))   # >= 1 GiB of weight copies
    ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(ncp)]
    x = torch.randn(M, K, device=dev).bfloat16()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for mode in ("hot", "cold"):
        for i in range(3):
            torch.nn.functional.linear(x, ws[i % ncp])
        torch.cuda.synchronize()
        n = 4 * ncp
        ev[0].record()
        for i in range(n):
            torch.nn.functional.linear(x, ws[0] if mode == "hot" else ws[i % ncp])
        ev[1].record()
        torch.cuda.synchronize()
        us = ev[0].elapsed_time(ev[1]) / n * 1e3
        res[f"{name}_{mode}"] = round(us, 1)
    print(name, res[f"{name}_hot"], res[f"{name}_cold"], flush=True)
    del ws
print(json.dumps({"M": M, **res}))
