"""Decode-attention latency vs split count, isolated (graph replay, KV cycled
over per-layer copies so reads are not served from a warm L2).

LLM: Llama-3-8B shapes (Hkv 8, G 4, D 128, paged blk 16), B sequences at ctx.
STT: Whisper-large-v3 cross-attention (H 20, D 64, 1500 contiguous rows)."""
import json, os, sys
import torch
sys.path.insert(0, os.getcwd())
from loqa_hub_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
bf = dict(dtype=torch.bfloat16, device=dev)
res = {}
L = 32

for B, ctx in ((6, 400), (8, 600), (6, 900)):
    Hkv, G, D, blk = 8, 4, 128, 16
    H = Hkv * G
    nb_seq = (ctx + blk - 1) // blk
    nb = B * nb_seq
    kcs = [torch.randn(nb, Hkv, blk, D, **bf) for _ in range(L)]
    vcs = [torch.randn(nb, Hkv, blk, D, **bf) for _ in range(L)]
    bt = torch.randperm(nb, device=dev).int().view(B, nb_seq)
    q = torch.randn(B, H * D, **bf)
    cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
    cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    ws = ops.AttnWorkspace(dev, 64, H, D, 16)
    for sk in (128, 256, 384, 512, 1024):
        ns = -(-ctx // sk)
        it = iter(range(1 << 30))

        def run():
            i = next(it) % L
            ops.attention(q, kcs[i], vcs[i], cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=True, max_q=1,
                          ctx_lens=cl, block_tables=bt, grouped=True, split_keys=sk, num_splits=ns,
                          workspace=ws)
        res[f"llm_B{B}_ctx{ctx}_sk{sk}_ns{ns}_us"] = round(ops.graph_time(run, 64) * 1e3 / 64, 2)

for B in (2, 4):
    H, D, T = 20, 64, 1500
    encs = [torch.randn(B * T, 2 * H * D, **bf) for _ in range(L)]
    q = torch.randn(B, H * D, **bf)
    cu = torch.arange(B + 1, dtype=torch.int32, device=dev)
    starts = torch.arange(B, dtype=torch.int32, device=dev) * T
    lens = torch.full((B,), T, dtype=torch.int32, device=dev)
    ws = ops.AttnWorkspace(dev, 64, H, D, 16)
    for sk in (128, 256, 512, 768, 1536):
        ns = -(-T // sk)
        it = iter(range(1 << 30))

        def run():
            e = encs[next(it) % L]
            ops.attention(q, e, e[:, H * D:], cu, n_heads=H, n_kv=H, head_dim=D, causal=False, max_q=1,
                          cu_k=starts, ctx_lens=lens, grouped=True, split_keys=sk, num_splits=ns, workspace=ws)
        res[f"xattn_B{B}_sk{sk}_ns{ns}_us"] = round(ops.graph_time(run, 64) * 1e3 / 64, 2)
print(json.dumps(res), flush=True)
