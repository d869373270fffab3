"""Minimal driver for counter profiles of the prefill attention kernel: the
Whisper encoder shape (B sequences x 1500 frames, 20 heads, D 64), 5 calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402

B, T, H, D = int(os.environ.get("B", "4")), 1500, 20, 64
dev = torch.device("cuda")
q = torch.randn(B * T, H * D, device=dev).bfloat16()
k = torch.randn(B * T, H * D, device=dev).bfloat16()
v = torch.randn(B * T, H * D, device=dev).bfloat16()
cu = torch.arange(0, B + 1, device=dev, dtype=torch.int32) * T
for _ in range(5):
    ops.attention(q, k, v, cu, n_heads=H, n_kv=H, head_dim=D, causal=False, max_q=T, cu_k=cu)
torch.cuda.synchronize()
print("ok")
