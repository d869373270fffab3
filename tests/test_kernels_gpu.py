"""Numerics of every HIP kernel against the plain-PyTorch fp32 reference of the
same op (ops/reference.py). Shapes follow SURVEY §2.4."""
import math

import numpy as np
import pytest
import torch

from loqa_hub_amd import ops
from loqa_hub_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


@pytest.mark.parametrize("d,rows", [(4096, 37), (2048, 5), (8192, 3), (384, 64)])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm(d, rows, with_res):
    x = torch.randn(rows, d, device=DEV, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(d, device=DEV)).bfloat16()
    r1 = torch.randn(rows, d, device=DEV, dtype=torch.bfloat16) if with_res else None
    r2 = r1.clone() if with_res else None
    y = ops.rmsnorm(x, w, 1e-5, residual=r1)
    yr = ref.rmsnorm(x, w, 1e-5, residual=r2)
    assert _rel(y, yr) < 1e-2
    if with_res:
        assert torch.equal(r1, r2)


@pytest.mark.parametrize("d", [1280, 384, 512])
def test_layernorm(d):
    x = torch.randn(300, d, device=DEV, dtype=torch.bfloat16) * 3 + 1
    w = torch.randn(d, device=DEV).bfloat16()
    b = torch.randn(d, device=DEV).bfloat16()
    r1 = torch.randn_like(x)
    r2 = r1.clone()
    y = ops.layernorm(x, w, b, 1e-5, residual=r1)
    yr = ref.layernorm(x, w, b, 1e-5, residual=r2)
    assert _rel(y, yr) < 1e-2


@pytest.mark.parametrize("kind,d", [("rms", 4096), ("ln", 1280), ("rms", 384)])
def test_norm_row_gather(kind, d):
    """Norm of gathered rows (the decode step's final norm of its logit rows)
    against index_select + the fp32 reference."""
    x = torch.randn(40, d, device=DEV, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(d, device=DEV)).bfloat16()
    b = torch.randn(d, device=DEV).bfloat16()
    idx = torch.tensor([39, 0, 7, 7, 21], device=DEV, dtype=torch.int64)
    sel = x.index_select(0, idx)
    if kind == "rms":
        y, yr = ops.rmsnorm(x, w, 1e-5, row_idx=idx), ref.rmsnorm(sel, w, 1e-5)
    else:
        y, yr = ops.layernorm(x, w, b, 1e-5, row_idx=idx), ref.layernorm(sel, w, b, 1e-5)
    assert y.shape == (5, d)
    assert _rel(y, yr) < 1e-2


@pytest.mark.parametrize("d,with_pos,sums", [(4096, False, False), (1280, True, True),
                                             (384, True, True)])
def test_embed_stats(d, with_pos, sums):
    """Fused embedding + layer-0 row statistics vs embedding + seed_stats."""
    V, P, rows = 1000, 448, 48
    te = torch.randn(V, d, device=DEV, dtype=torch.bfloat16)
    pe = torch.randn(P, d, device=DEV, dtype=torch.bfloat16) if with_pos else None
    tok = torch.randint(0, V, (rows,), device=DEV, dtype=torch.int32)
    pos = torch.randint(0, P, (rows,), device=DEV, dtype=torch.int32) if with_pos else None
    s1, s2 = ops.FusedScratch(DEV), ops.FusedScratch(DEV)
    out = ops.embed_stats(tok, te, s1, positions=pos, pos_embed=pe, sums=sums)
    xr = te[tok.long()]
    if with_pos:
        xr = (xr.float() + pe[pos.long()].float()).bfloat16()
    assert torch.equal(out, xr)
    s2.seed_stats(xr, sums=sums)
    assert s1.stat_tiles == 1
    torch.testing.assert_close(s1.rowsq[:rows], s2.rowsq[:rows], rtol=1e-5, atol=1e-3)
    if sums:
        torch.testing.assert_close(s1.rowsum[:rows], s2.rowsum[:rows], rtol=1e-4, atol=1e-3)


def test_silu_mul_and_gelu():
    x = torch.randn(77, 2 * 1408, device=DEV, dtype=torch.bfloat16)
    assert _rel(ops.silu_mul(x), ref.silu_mul(x)) < 1e-2
    y = torch.randn(3000, 512, device=DEV, dtype=torch.bfloat16)
    bias = torch.randn(512, device=DEV, dtype=torch.bfloat16)
    pos = torch.randn(1500, 512, device=DEV, dtype=torch.bfloat16)
    y2 = y.clone()
    ops.gelu_bias_(y, bias, pos)
    ref.gelu_bias_(y2, bias, pos)
    assert _rel(y, y2) < 1e-2


@pytest.mark.parametrize("H,Hkv", [(8, 2), (32, 8), (72, 8)])
def test_rope_kv_append(H, Hkv):
    """(8, 2) / (32, 8): the batched-load kernel; (72, 8): the per-group loop
    (more groups than 8 per thread)."""
    D, blk, T = 128, 16, 21
    qkv = torch.randn(T, (H + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 500, (T,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(D, 1024, 500000.0, device=DEV)
    slots = torch.randperm(8 * blk, device=DEV)[:T].to(torch.int32)
    slots[3] = -1
    kc1 = torch.zeros(8, Hkv, blk, D, device=DEV, dtype=torch.bfloat16)
    vc1 = torch.zeros_like(kc1)
    kc2, vc2 = kc1.clone(), vc1.clone()
    q1, q2 = qkv.clone(), qkv.clone()
    ops.rope_kv_append(q1, pos, cs, kc1, vc1, slots, H, Hkv, D)
    ref.rope_kv_append(q2, pos, cs, kc2, vc2, slots, H, Hkv, D)
    assert _rel(q1, q2) < 1e-2
    assert _rel(kc1, kc2) < 1e-2
    assert torch.equal(vc1, vc2)


def _paged(kv_tokens, blk, n_blocks):
    """Scatter per-seq contiguous K [L, Hkv, D] into a random paged layout."""
    Hkv, D = kv_tokens[0].shape[1:]
    cache = torch.zeros(n_blocks, Hkv, blk, D, device=DEV, dtype=torch.bfloat16)
    perm = torch.randperm(n_blocks).tolist()
    tables = []
    for kt in kv_tokens:
        nb = (kt.shape[0] + blk - 1) // blk
        tab = [perm.pop() for _ in range(nb)]
        for i in range(kt.shape[0]):
            cache[tab[i // blk], :, i % blk] = kt[i]
        tables.append(tab)
    mb = max(len(t) for t in tables)
    bt = torch.zeros(len(tables), mb, dtype=torch.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = torch.tensor(t)
    return cache, bt.to(DEV)


@pytest.mark.parametrize("D,H,Hkv", [(64, 4, 4), (128, 8, 2)])
@pytest.mark.parametrize("causal", [False, True])
def test_attention_prefill_contiguous(D, H, Hkv, causal):
    lens = [1500, 37, 200]
    T = sum(lens)
    q = torch.randn(T, H * D, device=DEV, dtype=torch.bfloat16)
    kv = torch.randn(T, 2 * Hkv * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int32, device=DEV)
    k, v = kv[:, : Hkv * D], kv[:, Hkv * D:]
    o = ops.attention(q, k, v, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=causal, max_q=max(lens), cu_k=cu)
    orf = ref.attention(q, k, v, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=causal, cu_k=cu)
    assert _rel(o, orf) < 2e-2


@pytest.mark.parametrize("G", [1, 4])
@pytest.mark.parametrize("D", [64, 128])
def test_attention_prefill_paged_with_prefix(G, D):
    """Paged causal prefill behind a cached prefix; D = 64 runs the 64-rows-
    per-wave variant (partial 256-row tile, causal bound per row group)."""
    Hkv = 2
    H = Hkv * G
    blk = 16
    ctx = [400, 90, 33]
    ql = [380, 90, 1]          # seq 0 has a 20-token cached prefix
    ks = [torch.randn(c, Hkv, D, device=DEV, dtype=torch.bfloat16) for c in ctx]
    vs = [torch.randn(c, Hkv, D, device=DEV, dtype=torch.bfloat16) for c in ctx]
    kc, bt = _paged(ks, blk, 64)
    torch.manual_seed(1)
    vc, _ = _paged(vs, blk, 64)
    # same layout for V: rebuild with the same tables
    vc = torch.zeros_like(kc)
    for b, vt in enumerate(vs):
        for i in range(vt.shape[0]):
            vc[int(bt[b, i // blk]), :, i % blk] = vt[i]
    q = torch.randn(sum(ql), H * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(np.cumsum(ql)), dtype=torch.int32, device=DEV)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    o = ops.attention(q, kc, vc, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=True, max_q=max(ql),
                      ctx_lens=cl, block_tables=bt)
    orf = ref.attention(q, kc, vc, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=True, ctx_lens=cl,
                        block_tables=bt)
    assert _rel(o, orf) < 2e-2


# decode-attention kernel forms: (8-wave min keys, prefetch min keys) -> the
# 4-wave kernel, the 8-wave single-pass one, and the prefetching variants
ATTN_FORMS = {"w4": (0, 0), "w8": (256, 0), "w4pf": (0, 64), "w8pf": (256, 64)}


@pytest.fixture(params=sorted(ATTN_FORMS))
def attn_form(request, monkeypatch):
    w8, pf = ATTN_FORMS[request.param]
    monkeypatch.setattr(ops, "ATTN8_MIN_KEYS", w8)
    monkeypatch.setattr(ops, "ATTN_PF_MIN_KEYS", pf)
    return request.param


@pytest.mark.parametrize("split_keys", [128, 256, 512])
@pytest.mark.parametrize("qlens,G,splits", [([1, 1, 1, 1], 4, 4), ([3, 1, 7, 2], 4, 2),
                                            ([1, 1], 1, 1), ([16, 5], 8, 3)])
def test_attention_grouped_paged(qlens, G, splits, split_keys, attn_form):
    """Paged GQA decode attention; split_keys 128 / 256 / 512 run the 4- and
    8-wave kernels (one pass, several passes, one split or several), with and
    without the next-tile prefetch."""
    D, Hkv, blk = 128, 2, 16
    H = Hkv * G
    ctx = [700, 65, 300, 1][: len(qlens)]
    ctx = [max(c, q) for c, q in zip(ctx, qlens)]
    ks = [torch.randn(c, Hkv, D, device=DEV, dtype=torch.bfloat16) for c in ctx]
    kc, bt = _paged(ks, blk, 128)
    vc = torch.randn_like(kc)
    q = torch.randn(sum(qlens), H * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(np.cumsum(qlens)), dtype=torch.int32, device=DEV)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    ws = ops.AttnWorkspace(DEV, 64, H, D, 8)

    def run():
        return ops.attention(q, kc, vc, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=True,
                             max_q=max(qlens), ctx_lens=cl, block_tables=bt, grouped=True,
                             split_keys=split_keys,
                             num_splits=max(splits, math.ceil(max(ctx) / split_keys)), workspace=ws)
    o = run()
    orf = ref.attention(q, kc, vc, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=True, ctx_lens=cl,
                        block_tables=bt)
    assert _rel(o, orf) < 2e-2
    # the in-launch split combine leaves its tickets reset: a replay is bitwise equal
    assert torch.equal(run(), o)
    assert int(ws.counters.abs().sum()) == 0


@pytest.mark.parametrize("split_keys", [128, 256, 512, 1536])
def test_attention_grouped_cross_starts(split_keys, attn_form):
    """Whisper cross-attention: subset of utterances addressed by start/len
    (4 / 8 / 16-wave workgroups, 12 / 6 / 3 / 1 splits)."""
    D, H, T = 64, 6, 1500
    enc = torch.randn(4 * T, 2 * H * D, device=DEV, dtype=torch.bfloat16)
    live = [0, 2, 3]
    q = torch.randn(len(live), H * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.arange(len(live) + 1, dtype=torch.int32, device=DEV)
    starts = torch.tensor([i * T for i in live], dtype=torch.int32, device=DEV)
    lens = torch.full((len(live),), T, dtype=torch.int32, device=DEV)
    ws = ops.AttnWorkspace(DEV, 64, H, D, 12)
    o = ops.attention(q, enc, enc[:, H * D:], cu, n_heads=H, n_kv=H, head_dim=D, causal=False, max_q=1,
                      cu_k=starts, ctx_lens=lens, grouped=True, split_keys=split_keys,
                      num_splits=-(-T // split_keys), workspace=ws)
    orf = ref.attention(q, enc, enc[:, H * D:], cu, n_heads=H, n_kv=H, head_dim=D, causal=False,
                        cu_k=starts, ctx_lens=lens)
    assert _rel(o, orf) < 2e-2


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_masked_argmax(dtype):
    B, V = 6, 128256
    logits = torch.randn(B, V, device=DEV).to(dtype)
    bits = torch.rand(3, V, device=DEV) < 0.01
    bits[2] = False
    bits[2, 12345] = True
    mask = ref.pack_mask(bits)
    rows = torch.tensor([0, 1, 2, 0, 1, 2], dtype=torch.int32, device=DEV)
    a = ops.masked_argmax(logits, mask, rows)
    b = ref.masked_argmax(logits, mask, rows)
    assert torch.equal(a.cpu(), b.cpu())
    assert int(a[2]) == 12345
    assert torch.equal(ops.masked_argmax(logits).cpu(), logits.float().argmax(-1).int().cpu())


def test_pcm16_sumsq():
    segs = [np.random.randint(-32768, 32767, n).astype(np.int16) for n in (16000, 1, 70001)]
    cat = torch.from_numpy(np.concatenate(segs)).to(DEV)
    off = torch.tensor([0, 16000, 16001, 86002], dtype=torch.int64, device=DEV)
    f, ss = ops.pcm16_to_f32_sumsq(cat, off)
    fr, ssr = ref.pcm16_to_f32_sumsq(cat.cpu(), off.cpu())
    assert torch.allclose(f.cpu(), fr)
    assert torch.allclose(ss.cpu(), ssr, rtol=1e-4)


@pytest.mark.parametrize("n_mels", [80, 128])
def test_log_mel(n_mels):
    c = ref.MelConstants.create(n_mels)
    t = np.arange(480000) / 16000
    a = np.stack([0.3 * np.sin(2 * np.pi * 440 * t) * (t < 3), 0.1 * np.random.randn(480000)])
    audio = torch.from_numpy(a.astype(np.float32)).to(DEV)
    m = ops.log_mel(audio, c).float()
    mr = ref.log_mel(audio, c)
    assert m.shape == mr.shape == (2, n_mels, 3000)
    assert float((m - mr).abs().max()) < 0.05


def test_im2col():
    x = torch.randn(2, 80, 3000, device=DEV, dtype=torch.bfloat16)
    a = ops.im2col_k3(x, (80 * 3000, 3000, 1), 2, 80, 3000, 1)
    b = ref.im2col_k3(x, (80 * 3000, 3000, 1), 2, 80, 3000, 1)
    assert torch.equal(a, b)
    y = torch.randn(2, 3000, 64, device=DEV, dtype=torch.bfloat16)
    a = ops.im2col_k3(y, (3000 * 64, 1, 64), 2, 64, 3000, 2)
    b = ref.im2col_k3(y, (3000 * 64, 1, 64), 2, 64, 3000, 2)
    assert torch.equal(a, b)


@pytest.mark.parametrize("Mpad,N,K", [(16, 6144, 4096), (32, 4096, 14336), (64, 1280, 1280),
                                      (128, 2560, 2048), (16, 128256, 4096)])
def test_skinny_gemm(Mpad, N, K):
    x = torch.randn(Mpad, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    wp = ops.shuffle_weight(w)
    assert torch.equal(wp.cpu(), ref.shuffle_weight(w.cpu()))
    part = ops.skinny_gemm(x, wp)
    want = x.float() @ w.float().t()
    assert part.shape[1:] == (Mpad, N)
    assert _rel(part.sum(0), want) < 1e-3


def test_slab_consumers():
    Mpad, d, H, Hkv, D, F = 32, 512, 4, 2, 128, 1024
    part = torch.randn(4, Mpad, d, device=DEV)
    res1 = torch.randn(Mpad, d, device=DEV, dtype=torch.bfloat16)
    res2 = res1.clone()
    w = torch.randn(d, device=DEV).bfloat16()
    y1 = ops.slab_rmsnorm(part, res1, w, 1e-5)
    y2 = ref.slab_rmsnorm(part, res2, w, 1e-5)
    assert _rel(y1, y2) < 1e-2 and torch.equal(res1, res2)
    idx = torch.tensor([3, 1, 0] + [0] * 13, dtype=torch.int64, device=DEV)
    z1 = ops.slab_rmsnorm(part, res1, w, 1e-5, row_idx=idx, write_residual=False)
    z2 = ref.slab_rmsnorm(part, res2, w, 1e-5, row_idx=idx, write_residual=False)
    assert _rel(z1, z2) < 1e-2
    qkv = torch.randn(2, Mpad, (H + 2 * Hkv) * D, device=DEV)
    pos = torch.arange(Mpad, dtype=torch.int32, device=DEV)
    cs = ref.rope_cos_sin(D, 256, 10000.0, device=DEV)
    slots = torch.arange(Mpad, dtype=torch.int32, device=DEV)
    slots[-5:] = -1
    kc1 = torch.zeros(4, Hkv, 16, D, device=DEV, dtype=torch.bfloat16)
    vc1, kc2, vc2 = torch.zeros_like(kc1), torch.zeros_like(kc1), torch.zeros_like(kc1)
    q1 = ops.slab_rope_append(qkv, pos, cs, kc1, vc1, slots, H, Hkv, D)
    q2 = ref.slab_rope_append(qkv, pos, cs, kc2, vc2, slots, H, Hkv, D)
    assert _rel(q1, q2) < 1e-2 and _rel(kc1, kc2) < 1e-2 and _rel(vc1, vc2) < 1e-2
    gu = torch.randn(3, Mpad, 2 * F, device=DEV)
    assert _rel(ops.slab_silu_mul(gu), ref.slab_silu_mul(gu)) < 1e-2
    assert _rel(ops.slab_reduce(gu), gu.sum(0)) < 1e-5


def test_whisper_slab_consumers():
    """LayerNorm / bias+GELU / biased KV-append consumers and the embed kernel."""
    Mpad, d, H, D = 16, 1280, 20, 64
    part = torch.randn(5, Mpad, d, device=DEV)
    bias = torch.randn(d, device=DEV).bfloat16()
    res1 = torch.randn(Mpad, d, device=DEV, dtype=torch.bfloat16)
    res2 = res1.clone()
    w, b = torch.randn(d, device=DEV).bfloat16(), torch.randn(d, device=DEV).bfloat16()
    y1 = ops.slab_layernorm(part, res1, w, b, 1e-5, bias=bias)
    y2 = ref.slab_layernorm(part, res2, w, b, 1e-5, bias=bias)
    assert _rel(y1, y2) < 1e-2 and _rel(res1, res2) < 1e-3
    idx = torch.tensor([4, 2] + [0] * 14, dtype=torch.int64, device=DEV)
    z1 = ops.slab_layernorm(part, res1, w, b, 1e-5, bias=bias, row_idx=idx, write_residual=False)
    z2 = ref.slab_layernorm(part, res2, w, b, 1e-5, bias=bias, row_idx=idx, write_residual=False)
    assert _rel(z1, z2) < 1e-2
    f = torch.randn(2, Mpad, 5120, device=DEV)
    fb = torch.randn(5120, device=DEV).bfloat16()
    assert _rel(ops.slab_bias_act(f, fb, "gelu"), ref.slab_bias_act(f, fb, "gelu")) < 1e-2
    assert _rel(ops.slab_bias_act(f, fb), ref.slab_bias_act(f, fb)) < 1e-2
    qkv = torch.randn(2, Mpad, 3 * H * D, device=DEV)
    qb = torch.randn(3 * H * D, device=DEV).bfloat16()
    pos = torch.arange(Mpad, dtype=torch.int32, device=DEV)
    slots = torch.arange(Mpad, dtype=torch.int32, device=DEV)
    slots[-3:] = -1
    kc1 = torch.zeros(2, H, 16, D, device=DEV, dtype=torch.bfloat16)
    vc1, kc2, vc2 = torch.zeros_like(kc1), torch.zeros_like(kc1), torch.zeros_like(kc1)
    q1 = ops.slab_rope_append(qkv, pos, None, kc1, vc1, slots, H, H, D, bias=qb)
    q2 = ref.slab_rope_append(qkv, pos, None, kc2, vc2, slots, H, H, D, bias=qb)
    assert _rel(q1, q2) < 1e-2 and _rel(kc1, kc2) < 1e-2 and _rel(vc1, vc2) < 1e-2
    te = torch.randn(1000, d, device=DEV).bfloat16()
    pe = torch.randn(448, d, device=DEV).bfloat16()
    tk = torch.randint(0, 1000, (Mpad,), dtype=torch.int32, device=DEV)
    e = ops.embed_pos(tk, pos, te, pe)
    assert torch.equal(e, (te[tk.long()].float() + pe[pos.long()].float()).bfloat16())


@pytest.mark.parametrize("qlens", [[1, 1, 1], [4, 4, 4]])
def test_attn_decode_contiguous_cross(qlens):
    """Split-key decode kernel on contiguous encoder rows (non-causal)."""
    D, H, T = 64, 20, 1500
    enc = torch.randn(4 * T, 2 * H * D, device=DEV, dtype=torch.bfloat16)
    live = [3, 0, 2]
    cu = torch.tensor(np.concatenate([[0], np.cumsum(qlens)]), dtype=torch.int32, device=DEV)
    q = torch.randn(16, H * D, device=DEV, dtype=torch.bfloat16)
    starts = torch.tensor([i * T for i in live], dtype=torch.int32, device=DEV)
    lens = torch.full((3,), T, dtype=torch.int32, device=DEV)
    ws = ops.AttnWorkspace(DEV, 64, H, D, 12)
    o = ops.attention(q, enc, enc[:, H * D:], cu, n_heads=H, n_kv=H, head_dim=D, causal=False,
                      max_q=max(qlens), cu_k=starts, ctx_lens=lens, grouped=True, split_keys=128,
                      num_splits=12, workspace=ws)
    n = int(cu[-1])
    orf = ref.attention(q[:n], enc, enc[:, H * D:], cu, n_heads=H, n_kv=H, head_dim=D,
                        causal=False, cu_k=starts, ctx_lens=lens)
    assert _rel(o[:n], orf) < 2e-2


def test_llama_decode_fast_path_matches_generic():
    """forward_decode (skinny GEMM + slab ops) == forward (hipBLASLt + generic ops)."""
    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    eng = LLMEngine(llama_config("test-tiny"), DEV, max_seqs=4, use_graphs=False)
    tok = torch.randint(10, 4000, (2, 40)).tolist()
    outs = []
    for decode in (True, False):
        pool = eng.kv.pool
        for sid in (1, 2):
            pool.add_seq(sid + (10 if decode else 20), [])
        seqs = []
        from loqa_hub_amd.engine.llm_engine import GenRequest
        for i, sid in enumerate((1, 2)):
            r = GenRequest([], [])
            r.seq_id = sid + (10 if decode else 20)
            seqs.append(r)
        feeds = [t[:5] for t in tok]
        max_q, max_ctx, host = eng._meta(seqs, feeds, decode, 2, ops.mpad_for(10) if decode else None)
        host["mask_rows"] = np.zeros(2, np.int32)
        dev = eng._to_device(host)
        meta = eng._build_meta(dev, max_q, max_ctx, decode)
        if decode:
            lg = eng.model.forward_decode(meta, eng.kv.k, eng.kv.v, eng.attn_ws)[:2]
        else:
            lg = eng.model.logits(eng.model.forward(meta, eng.kv.k, eng.kv.v, eng.attn_ws))
        outs.append(lg.float())
    assert _rel(outs[0], outs[1]) < 3e-2


# ------------------------------------------------------------------ VITS kernels
@pytest.mark.parametrize("Cin,Cout,K,dil,act,pre", [
    (192, 192, 5, 1, None, None), (64, 32, 7, 3, "relu", 0.1), (512, 256, 3, 1, "tanh", None),
    (32, 1, 7, 1, "tanh", 0.01), (192, 384, 5, 1, "gated", None),
    (128, 128, 11, 5, None, 0.1), (256, 256, 7, 3, None, 0.1)])
def test_conv1d_mfma(Cin, Cout, K, dil, act, pre):
    """Stride-1 convs run the LDS-staged kernel (64- or 32-channel chunks by
    the 64 KiB budget: the K = 11, dil = 5 case takes 32) vs the fp32 torch
    reference."""
    B, T = 2, 300
    w = torch.randn(Cout, Cin, K, device=DEV) * (Cin * K) ** -0.5
    b = torch.randn(Cout, device=DEV) * 0.1
    cw = ops.ConvWeight(w, b, gated=act == "gated")
    x = torch.randn(B, T, Cin, device=DEV).bfloat16()
    res = torch.randn(B, T, cw.out_channels, device=DEV).bfloat16()
    lens = torch.tensor([T, 211], dtype=torch.int32, device=DEV)
    y = ops.conv1d(x, cw, dil=dil, pre_slope=pre, act=act, res=res, alpha=0.5, lens=lens)
    yr = ref.conv1d(x, w, b, dil=dil, pad=dil * (K - 1) // 2, pre_slope=pre, act=act, res=res,
                    alpha=0.5, lens=lens)
    assert _rel(y, yr) < 1e-2


def test_conv1d_accumulate_inplace_and_pcm16():
    B, T, C = 1, 513, 64
    cw = ops.ConvWeight(torch.randn(C, C, 3, device=DEV) * 0.1, torch.zeros(C, device=DEV))
    x = torch.randn(B, T, C, device=DEV).bfloat16()
    acc = torch.randn(B, T, C, device=DEV).bfloat16()
    expect = ref.conv1d(x, cw.w, cw.bias, pad=1, alpha=1 / 3, acc=acc)
    out = ops.conv1d(x, cw, alpha=1 / 3, acc=acc, out=acc)
    assert out.data_ptr() == acc.data_ptr() and _rel(acc, expect) < 1e-2
    post = ops.ConvWeight(torch.randn(1, C, 7, device=DEV) * 0.05, None)
    pcm = ops.conv1d(x, post, pre_slope=0.01, act="tanh", pcm16=True)
    pr = ref.conv1d(x, post.w, None, pad=3, pre_slope=0.01, act="tanh")
    assert pcm.dtype == torch.int16
    assert (pcm.float() - (pr.clamp(-1, 1) * 32767).round()).abs().max() <= 400


@pytest.mark.parametrize("Cin,Cout,K,s", [(512, 256, 16, 8), (64, 32, 4, 2)])
def test_conv_transpose_polyphase(Cin, Cout, K, s):
    w = torch.randn(Cin, Cout, K, device=DEV) * (Cin * K / s) ** -0.5
    b = torch.randn(Cout, device=DEV) * 0.1
    ct = ops.ConvTransposeWeight(w, b, s, (K - s) // 2)
    x = torch.randn(2, 57, Cin, device=DEV).bfloat16()
    y = ops.conv_transpose1d(x, ct, pre_slope=0.1)
    yr = ref.conv_transpose1d(x, w, b, stride=s, padding=(K - s) // 2, pre_slope=0.1)
    assert y.shape == yr.shape and _rel(y, yr) < 1e-2


def test_relpos_attention_and_expand():
    B, T, H, D, W = 2, 77, 2, 96, 4
    qkv = torch.randn(B, T, 3 * H * D, device=DEV).bfloat16()
    ek = torch.randn(2 * W + 1, D, device=DEV).bfloat16() * 0.1
    ev = torch.randn(2 * W + 1, D, device=DEV).bfloat16() * 0.1
    lens = torch.tensor([T, 50], dtype=torch.int32, device=DEV)
    o = ops.relpos_attention(qkv, ek, ev, lens, H, D, W)
    orf = ref.relpos_attention(qkv, ek, ev, lens, H, D, W, 1 / math.sqrt(D))
    assert _rel(o, orf) < 1e-2
    stats = torch.randn(B, T, 2 * 64, device=DEV).bfloat16() * 0.5
    dur = torch.randint(1, 6, (B, T), device=DEV, dtype=torch.int32)
    dur[1, 50:] = 0
    cum = torch.cumsum(dur, 1, dtype=torch.int32)
    flen = cum[:, -1].contiguous()
    F = int(flen.max())
    z = ops.expand_sample(stats, cum, flen, F, 0.0)
    assert _rel(z, ref.expand_sample(stats, cum, flen, F, 0.0)) < 1e-2
    zn = ops.expand_sample(torch.zeros_like(stats), cum, flen, F, 1.0, seed=7)[0].float()
    assert abs(zn.mean().item()) < 0.05 and abs(zn.std().item() - 1.0) < 0.05
    # frame-padded launch (graph bucket) with the seed read on the device: the
    # same latent on the valid frames, zeros past them
    zs = ops.expand_sample(stats, cum, flen, F, 0.667, seed=11)
    sd = torch.tensor([11], dtype=torch.int32, device=DEV)
    zp = ops.expand_sample(stats, cum, flen, F + 96, 0.667, seed=0, seed_dev=sd)
    assert torch.equal(zp[:, :F], zs) and not zp[:, F:].any()


@pytest.mark.parametrize("D,H,Hkv,lens,causal", [
    (128, 32, 8, [1100, 3, 640, 1], True),      # long GQA prefill, decode-like rows
    (64, 20, 20, [1500, 1500, 1500], False),     # Whisper encoder, batch 3
    (64, 6, 6, [65, 127, 129, 64], False),       # tile-boundary lengths (odd/one tile per half)
])
def test_attention_prefill2_shapes(D, H, Hkv, lens, causal):
    """Split-KV prefill attention: key-tile counts odd / even / one (the second
    wave group idle), lengths at the 64-key tile and 128-row boundaries."""
    T = sum(lens)
    q = torch.randn(T, H * D, device=DEV, dtype=torch.bfloat16)
    kv = torch.randn(T, 2 * Hkv * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int32, device=DEV)
    k, v = kv[:, : Hkv * D], kv[:, Hkv * D:]
    o = ops.attention(q, k, v, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=causal, max_q=max(lens), cu_k=cu)
    orf = ref.attention(q, k, v, cu, n_heads=H, n_kv=Hkv, head_dim=D, causal=causal, cu_k=cu)
    assert _rel(o, orf) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("layout", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("M,N,K,S,epi", [(318, 256, 512, 1, "bf16"), (100, 384, 1024, 4, "slabs"),
                                         (1, 128, 256, 2, "slabs"), (481, 512, 640, 1, "swiglu"),
                                         (161, 256, 256, 1, "swiglu")])
def test_prefill_gemm2(layout, M, N, K, S, epi):
    """Prefill GEMM v2 (2 x 2 waves, csrc/kernels/gemm_prefill.hip) vs fp32:
    bf16 output, f32 split-K slabs, and the SwiGLU pair-tile epilogue."""
    from loqa_hub_amd import ops
    from loqa_hub_amd.ops import reference as R
    rbw, ft, wm = ops.PREFILL2_LAYOUTS[layout]
    if N % (16 * ft * (4 // wm)):
        pytest.skip("N not a multiple of the layout's feature block")
    g = torch.Generator(device="cuda").manual_seed(M + N + layout)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    if epi == "swiglu":
        w = w[R.perm_gate_up(N // 2).cuda()].contiguous()
    out = ops.prefill_gemm2(x, ops.shuffle_weight(w), S, epi=epi, layout=layout)
    ref = x.float() @ w.float().t()
    if epi == "slabs":
        assert out.shape == (S, M, N)
        assert float((out.sum(0) - ref).norm() / ref.norm()) < 1e-5
    elif epi == "swiglu":
        assert out.shape == (M, N // 2)
        r = R.swiglu_pairs(ref)
        assert float((out.float() - r).norm() / r.norm()) < 1e-2
    else:
        assert float((out.float() - ref).norm() / ref.norm()) < 5e-3
