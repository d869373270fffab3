"""Mixed prompt-pass attention (``LlamaModel._prompt_attention`` with
``StepMeta.split``): the live decoders' rows on the grouped split-key decode
kernel, the prompt chunk on the flash prefill kernel, each writing its rows of
one output - against the fp32 reference of the whole batch and against the
single prefill launch."""
import numpy as np
import pytest
import torch

from loqa_hub_amd import ops
from loqa_hub_amd.ops import reference as R


def _case(dev, H=32, Hkv=8, D=128, blk=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    qlens = [1, 3, 1, 2, 37]             # 4 live decoders (jump-forward feeds), 1 prompt chunk
    ctx = [190, 75, 300, 33, 120]        # tokens in cache after the pass
    nd = 4
    B = len(qlens)
    max_blocks = max(-(-c // blk) for c in ctx) + 1
    nb = B * max_blocks + 4
    perm = torch.randperm(nb, generator=g)
    bt = perm[:B * max_blocks].view(B, max_blocks).to(torch.int32)
    kc = (torch.randn(nb, Hkv, blk, D, generator=g) * 0.5).to(torch.bfloat16)
    vc = torch.randn(nb, Hkv, blk, D, generator=g).to(torch.bfloat16)
    T = sum(qlens)
    qkv = (torch.randn(T, (H + 2 * Hkv) * D, generator=g) * 0.5).to(torch.bfloat16)
    cu = torch.tensor(np.concatenate([[0], np.cumsum(qlens)]), dtype=torch.int32)
    ctx_t = torch.tensor(ctx, dtype=torch.int32)
    rd = int(cu[nd])
    cu_tail = (cu[nd:] - cu[nd]).to(torch.int32)
    mv = lambda t: t.to(dev)              # noqa: E731
    return dict(H=H, Hkv=Hkv, D=D, nd=nd, rd=rd, qlens=qlens, ctx=ctx, qkv=mv(qkv), kc=mv(kc),
                vc=mv(vc), cu=mv(cu), ctx_t=mv(ctx_t), bt=mv(bt), cu_tail=mv(cu_tail))


def _split(c, ws):
    H, Hkv, D, nd, rd = c["H"], c["Hkv"], c["D"], c["nd"], c["rd"]
    qkv = c["qkv"]
    out = torch.empty(qkv.shape[0], H * D, dtype=torch.bfloat16, device=qkv.device)
    dctx = max(c["ctx"][:nd])
    ns, sk = ops.decode_attn_splits(dctx, nd * Hkv, 128)
    ops.attention(qkv[:rd], c["kc"], c["vc"], c["cu"][:nd + 1], n_heads=H, n_kv=Hkv, head_dim=D,
                  causal=True, max_q=max(c["qlens"][:nd]), ctx_lens=c["ctx_t"][:nd],
                  block_tables=c["bt"][:nd], grouped=True, split_keys=sk, num_splits=ns,
                  workspace=ws, out=out[:rd], max_k=dctx)
    ops.attention(qkv[rd:], c["kc"], c["vc"], c["cu_tail"], n_heads=H, n_kv=Hkv, head_dim=D,
                  causal=True, max_q=max(c["qlens"][nd:]), ctx_lens=c["ctx_t"][nd:],
                  block_tables=c["bt"][nd:], grouped=False, split_keys=256, num_splits=1,
                  workspace=ws, out=out[rd:], max_k=max(c["ctx"]))
    return out


def test_mixed_split_layout_cpu():
    """The two launches cover exactly the batch's rows with the right
    per-sequence metadata (reference attention on the CPU)."""
    c = _case("cpu")
    whole = R.attention(c["qkv"], c["kc"], c["vc"], c["cu"], n_heads=c["H"], n_kv=c["Hkv"],
                        head_dim=c["D"], causal=True, ctx_lens=c["ctx_t"], block_tables=c["bt"])
    got = _split(c, None)
    torch.testing.assert_close(got.float(), whole.float(), rtol=0, atol=0)


@pytest.mark.gpu
def test_mixed_split_attention_gpu():
    dev = torch.device("cuda", 0)
    c = _case(dev)
    ws = ops.AttnWorkspace(dev, 128, c["H"], c["D"], 8)
    got = _split(c, ws)
    one = ops.attention(c["qkv"], c["kc"], c["vc"], c["cu"], n_heads=c["H"], n_kv=c["Hkv"],
                        head_dim=c["D"], causal=True, max_q=max(c["qlens"]), ctx_lens=c["ctx_t"],
                        block_tables=c["bt"], grouped=False, split_keys=256, num_splits=1,
                        workspace=ws, max_k=max(c["ctx"]))
    torch.cuda.synchronize()
    ref = R.attention(c["qkv"].cpu().float(), c["kc"].cpu().float(), c["vc"].cpu().float(),
                      c["cu"].cpu(), n_heads=c["H"], n_kv=c["Hkv"], head_dim=c["D"], causal=True,
                      ctx_lens=c["ctx_t"].cpu(), block_tables=c["bt"].cpu())
    scale = ref.abs().max().item()
    for name, o in (("split", got), ("single", one)):
        err = (o.float().cpu() - ref).abs().max().item()
        assert err < 2e-2 * scale, (name, err, scale)


def test_mixed_split_planning_cpu():
    """``LLMEngine._mixed_split``: the live decoders must lead the pass, fit the
    grouped kernel's query rows and the workspace; otherwise one flash launch."""
    from types import SimpleNamespace
    from loqa_hub_amd.engine.llm_engine import LLMEngine

    def plan(kinds, feeds, max_q=8, ws_tokens=128, ws_counters=4096, on=True):
        cu = np.concatenate([[0], np.cumsum([len(f) for f in feeds])]).astype(np.int32)
        host = {"cu_q": cu, "ctx_lens": np.arange(10, 10 + len(feeds), dtype=np.int32)}
        eng = SimpleNamespace(MIXED_SPLIT=on, max_decode_q=max_q, weights=SimpleNamespace(hkv=8),
                              attn_ws=SimpleNamespace(max_tokens=ws_tokens,
                                                      counters=torch.zeros(ws_counters)))
        return LLMEngine._mixed_split(eng, kinds, feeds, host), host

    sp, host = plan([0, 0, 2], [[1], [2, 3], list(range(40))])
    assert sp == (2, 3, 2, 11) and host["cu_tail"].tolist() == [0, 40]
    assert plan([0, 0, 1], [[1], list(range(9)), [5] * 7])[0] is None        # feed > 8 rows
    assert plan([1, 2], [[1] * 5, [2] * 5])[0] is None                       # no live decoder
    assert plan([0, 0], [[1], [2]])[0] is None                               # nothing to prefill
    assert plan([0, 1], [[1], [2] * 5], ws_tokens=0)[0] is None               # workspace too small
    assert plan([0, 1], [[1], [2] * 5], on=False)[0] is None                  # LOQA_MIXED_SPLIT_ATTN=0
    assert plan([0, 1], [[1], [2] * 5], ws_counters=4)[0] is None             # counters too few
