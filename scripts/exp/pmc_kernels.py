"""Short kernel workload for rocprofv3 --pmc passes (hardware counters per
dispatch): the Llama-3-8B decode GEMMs (M = 16, tuned layouts, cold weights
cycled), the paged decode attention, and the prefill / encoder flash
attention. Each kernel runs 24 times; scripts/pmc_summary.py reduces the
counter CSV to per-kernel MFMA utilisation, LDS bank conflicts and HBM bytes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
bf = dict(dtype=torch.bfloat16, device=dev)
R = 24
scr = ops.FusedScratch(dev)
M = 16
for name, (N, K), mode, kw in (("gate_up", (28672, 4096), "silu", dict(splits=1, rt=2, wr=4, norm=True)),
                               ("down", (4096, 14336), "resid", dict(splits=2, rt=2, wr=1)),
                               ("o", (4096, 4096), "resid", dict(splits=1, rt=1, wr=1))):
    ncopy = max(2, -(-(1 << 30) // (N * K * 2)))
    base = torch.randn(N, K, **bf) * 0.02
    wps = [ops.shuffle_weight(base) for _ in range(ncopy)]
    del base
    x = torch.randn(M, K, **bf)
    if mode == "silu":
        scr.rowsq[: 128 * M].fill_(32.0)
        kw = dict(kw, rowsq_tiles=128)
    else:
        kw = dict(kw, residual=torch.randn(M, N, **bf))
    for i in range(R):
        ops.skinny_fused(x, wps[i % ncopy], mode, scr, **kw)
    torch.cuda.synchronize()
    del wps

# paged decode attention (8B: Hkv 8, G 4, D 128), 6 sequences x 400 keys
B, ctx, Hkv, G, D, blk = 6, 400, 8, 4, 128, 16
nb = B * (ctx // blk + 1)
kc = torch.randn(nb, Hkv, blk, D, **bf)
vc = torch.randn_like(kc)
bt = torch.randperm(nb, device=dev).int().view(B, -1)
q = torch.randn(B, Hkv * G * D, **bf)
cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
ws = ops.AttnWorkspace(dev, 64, Hkv * G, D, 8)
for _ in range(R):
    ops.attention(q, kc, vc, cu, n_heads=Hkv * G, n_kv=Hkv, head_dim=D, causal=True, max_q=1,
                  ctx_lens=cl, block_tables=bt, grouped=True, split_keys=128, num_splits=4, workspace=ws)
torch.cuda.synchronize()

# Whisper-large-v3 encoder self-attention, 4 x 1500 frames, 20 heads, D 64
T, H, D = 1500, 20, 64
qkv = torch.randn(4 * T, 3 * H * D, **bf)
cu = torch.arange(5, dtype=torch.int32, device=dev) * T
for _ in range(R):
    ops.attention(qkv, qkv[:, H * D:], qkv[:, 2 * H * D:], cu, n_heads=H, n_kv=H, head_dim=D,
                  causal=False, max_q=T, cu_k=cu)
torch.cuda.synchronize()
print("pmc workload done", flush=True)
