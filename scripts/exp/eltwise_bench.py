"""Elementwise / normalisation kernels of the prefill and encoder passes:
device time per call vs the bytes they move (cold: inputs cycled over copies)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda")
bf = dict(dtype=torch.bfloat16, device=dev)


def dtime(fn, n=40):
    """Per-call device time from a captured graph of n calls (the Python
    wrappers would otherwise set the pace)."""
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(n):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


NC = 8
res = {}
# Whisper encoder: layernorm with residual [1500, 1280]
xs = [torch.randn(1500, 1280, **bf) for _ in range(NC)]
rs = [torch.randn(1500, 1280, **bf) for _ in range(NC)]
w, b = torch.randn(1280, **bf), torch.randn(1280, **bf)
us = dtime(lambda i: ops.layernorm(xs[i % NC], w, b, 1e-5, residual=rs[i % NC]))
res["enc_layernorm_res_1500x1280"] = (round(us, 1), round(1500 * 1280 * 2 * 4 / us / 1e6, 2))
# gelu in place [1500, 5120]
gs = [torch.randn(1500, 5120, **bf) for _ in range(NC)]
us = dtime(lambda i: ops.gelu_bias_(gs[i % NC]))
res["enc_gelu_1500x5120"] = (round(us, 1), round(1500 * 5120 * 2 * 2 / us / 1e6, 2))
# Llama prefill: rmsnorm with residual [318, 4096]
xs = [torch.randn(318, 4096, **bf) for _ in range(NC)]
rs = [torch.randn(318, 4096, **bf) for _ in range(NC)]
w = torch.randn(4096, **bf)
us = dtime(lambda i: ops.rmsnorm(xs[i % NC], w, 1e-5, residual=rs[i % NC]))
res["pf_rmsnorm_res_318x4096"] = (round(us, 1), round(318 * 4096 * 2 * 4 / us / 1e6, 2))
# silu_mul [318, 28672] -> [318, 14336]
ss = [torch.randn(318, 28672, **bf) for _ in range(NC)]
us = dtime(lambda i: ops.silu_mul(ss[i % NC]))
res["pf_silu_mul_318x28672"] = (round(us, 1), round(318 * 28672 * 2 * 1.5 / us / 1e6, 2))
# Whisper-large-v3 log-mel of one / four 30-s windows (f32 MFMA DFT + mel GEMM)
from loqa_hub_amd.ops.reference import MelConstants  # noqa: E402
mc = MelConstants.create(128)
for B in (1, 4):
    au = [torch.randn(B, 480000, device=dev) * 0.1 for _ in range(NC)]
    us = dtime(lambda i: ops.log_mel(au[i % NC], mc), n=8)
    res[f"log_mel_B{B}"] = (round(us, 1), 0.0)
print(json.dumps({k: {"us": v[0], "TBps": v[1]} for k, v in res.items()}))
