"""Fixed vs streaming cost of the fused decode GEMM: time vs K at fixed N."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench_kernels import gtime  # noqa: E402
dev = torch.device("cuda")
scr = ops.FusedScratch(dev)
for N in (4096, 6144):
    for K in (128, 512, 1024, 2048, 4096):
        ncopy = max(2, -(-(512 << 20) // (N * K * 2)))
        wps = [ops.shuffle_weight(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(ncopy)]
        x = torch.randn(16, K, device=dev, dtype=torch.bfloat16)
        res = torch.randn(16, N, device=dev, dtype=torch.bfloat16)
        out = {"N": N, "K": K, "MB": round(N * K * 2 / 1e6, 1)}
        for S in (1, 2, 4):
            if K % (S * 128):
                continue
            for rt in (1, 2):
                it = iter(range(1 << 30))
                t = gtime(lambda: ops.skinny_fused(x, wps[next(it) % ncopy], "resid", scr, splits=S, rt=rt, wr=1,
                                                   residual=res), inner=max(20, 2 * ncopy))
                out[f"S{S}rt{rt}"] = round(t, 2)
        it = iter(range(1 << 30))
        out["plainS1"] = round(gtime(lambda: ops.skinny_gemm(x, wps[next(it) % ncopy], 1), inner=max(20, 2 * ncopy)), 2)
        print(json.dumps(out), flush=True)
        del wps
x = torch.zeros(16, 4096, device=dev, dtype=torch.bfloat16)
print(json.dumps({"graph_tiny_add_us": round(gtime(lambda: x.add_(1)), 2)}))
