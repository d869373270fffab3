"""Prefill / encoder attention (attn_prefill2_kernel): device time per call on the Whisper-large-v3
encoder (1500 frames, 20 heads, D 64) and Llama-3-8B prompt (GQA 32/8, D 128,
causal) shapes, plus max error vs the fp32 reference. LOQA_ATTN_V1=1 selects
the 4-wave kernel."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402
from loqa_hub_amd.ops import reference as ref  # noqa: E402

dev = torch.device("cuda")
cases = {"enc_B1": (1, 1500, 20, 20, 64, False), "enc_B2": (2, 1500, 20, 20, 64, False),
         "enc_B4": (4, 1500, 20, 20, 64, False), "pf_318": (1, 318, 32, 8, 128, True),
         "pf_2x318": (2, 318, 32, 8, 128, True), "pf_1024": (1, 1024, 32, 8, 128, True)}
res = {}
for name, (B, T, H, Hkv, D, causal) in cases.items():
    torch.manual_seed(0)
    q = torch.randn(B * T, H * D, device=dev).bfloat16()
    k = torch.randn(B * T, Hkv * D, device=dev).bfloat16()
    v = torch.randn(B * T, Hkv * D, device=dev).bfloat16()
    cu = torch.arange(0, B + 1, device=dev, dtype=torch.int32) * T
    f = lambda: ops.attention(q, k, v, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=causal,  # noqa: E731
                              max_q=T, cu_k=cu)
    o = f()
    r = ref.attention(q.float().cpu(), k.float().cpu(), v.float().cpu(), cu.cpu(), n_heads=H, n_kv=Hkv,
                      head_dim=D, causal=causal, cu_k=cu.cpu(), scale=D ** -0.5)
    err = float((o.float().cpu() - r.float()).abs().max())
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 20 * 1e3
    fl = 4 * B * T * T * D * H * (0.5 if causal else 1.0)
    res[name] = {"us": round(us, 1), "TF": round(fl / us / 1e6), "max_err": round(err, 4)}
    print(name, res[name], flush=True)
print(json.dumps({"v1": bool(os.environ.get("LOQA_ATTN_V1")), **res}))
