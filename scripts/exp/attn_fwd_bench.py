"""Prefill / encoder flash attention timing (graph replay): the Whisper-large-v3
encoder self-attention (1500 frames, 20 heads, D 64, B utterances) and a
Llama-3-8B causal prefill (GQA 32/8, D 128)."""
import json, os, sys
import torch
sys.path.insert(0, os.getcwd())
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
bf = dict(dtype=torch.bfloat16, device=dev)
res = {}
for B in (4, 8):
    T, H, D = 1500, 20, 64
    qkv = torch.randn(B * T, 3 * H * D, **bf)
    cu = torch.arange(B + 1, dtype=torch.int32, device=dev) * T

    def run():
        ops.attention(qkv, qkv[:, H * D:], qkv[:, 2 * H * D:], cu, n_heads=H, n_kv=H, head_dim=D,
                      causal=False, max_q=T, cu_k=cu)
    res[f"enc_B{B}_us"] = round(ops.graph_time(run, 16) * 1e3 / 16, 2)
for B, L in ((4, 512), (8, 1024)):
    H, Hkv, D = 32, 8, 128
    q = torch.randn(B * L, H * D, **bf)
    k = torch.randn(B * L, Hkv * D, **bf)
    v = torch.randn(B * L, Hkv * D, **bf)
    cu = torch.arange(B + 1, dtype=torch.int32, device=dev) * L

    def run2():
        ops.attention(q, k, v, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=True, max_q=L, cu_k=cu)
    res[f"llm_prefill_B{B}_L{L}_us"] = round(ops.graph_time(run2, 16) * 1e3 / 16, 2)
print(json.dumps(res), flush=True)
