"""The fused qkv GEMM + decode attention launch (gemm_skinny.hip ATTD mode,
``ops.skinny_fused(attn=...)``): the GEMM's workgroups turn into attention
workers once their tiles are in. It must match the two-launch path (qkv
GEMM, then attn_decode) BIT FOR BIT - same q rows, same cache appends, same
attention output - on the Llama-3-8B (GQA 32/8, D 128, RMSNorm, RoPE) and
Whisper large-v3 decoder (MHA 20/20, D 64, LayerNorm, no RoPE) shapes, for
every tile layout the tuner can pick, and leave its hand-off words zeroed
(graph replays)."""
import pytest
import torch

from loqa_hub_amd import ops
from loqa_hub_amd.ops import reference as ref

SHAPES = {
    # name: H, Hkv, D, K (d_model), norm
    "llama": (32, 8, 128, 4096, "rms"),
    "whisper": (20, 20, 64, 1280, "ln"),
}


def _layout(Mpad, max_q, g, blk=16):
    """Sequences of one decode step: q lengths, prior contexts, block tables."""
    B = max(1, Mpad // max_q - (1 if Mpad // max_q > 2 else 0))   # some padded rows
    qlens = [max_q if b % 3 else max(1, max_q // 2) for b in range(B)]
    prior = [int(x) for x in torch.randint(1, 700, (B,), generator=g)]
    prior[0] = 1                       # a sequence at its first decoded token
    ctx = [p + q for p, q in zip(prior, qlens)]
    max_blocks = max(-(-c // blk) for c in ctx) + 1
    nb = B * max_blocks + 16
    blocks = torch.randperm(nb, generator=g)[: B * max_blocks].view(B, max_blocks).int()
    return B, qlens, prior, ctx, blocks, nb


def test_decode_layout_builder_cpu():
    for Mpad in (16, 32, 64):
        for max_q in (1, 4):
            B, qlens, prior, ctx, blocks, nb = _layout(Mpad, max_q, torch.Generator().manual_seed(1))
            assert sum(qlens) <= Mpad and blocks.shape[0] == B and int(blocks.max()) < nb
            assert all(-(-c // 16) <= blocks.shape[1] for c in ctx)


def _case(shape, Mpad, max_q, seed=0, blk=16):
    H, Hkv, D, K, norm = SHAPES[shape]
    g = torch.Generator().manual_seed(seed)
    dev = torch.device("cuda", 0)
    N = (H + 2 * Hkv) * D
    w = (torch.randn(N, K, generator=g) * 0.02).bfloat16()
    nw = (torch.rand(K, generator=g) + 0.5).bfloat16()
    perm = ref.perm_rope_qkv(H, Hkv, D)
    if norm == "rms":
        lin = ops.FusedLinear(w.to(dev), norm="rms", norm_w=nw.to(dev), perm=perm.to(dev))
    else:
        nb_ = (torch.randn(K, generator=g) * 0.1).bfloat16()
        bias = (torch.randn(N, generator=g) * 0.1).bfloat16()
        lin = ops.FusedLinear(w.to(dev), norm="ln", norm_w=nw.to(dev), norm_b=nb_.to(dev),
                              bias=bias.to(dev), perm=perm.to(dev))
    B, qlens, prior, ctx, blocks, nb = _layout(Mpad, max_q, g, blk)
    T = sum(qlens)
    assert T <= Mpad and (H // Hkv) * max_q <= 32
    kc = (torch.randn(nb, Hkv, blk, D, generator=g) * 0.5).bfloat16()
    vc = (torch.randn(nb, Hkv, blk, D, generator=g) * 0.5).bfloat16()
    pos, slots = [], []
    for b in range(B):
        for i in range(qlens[b]):
            p = prior[b] + i
            pos.append(p)
            slots.append(int(blocks[b, p // blk]) * blk + p % blk)
    pos += [0] * (Mpad - T)
    slots += [-1] * (Mpad - T)
    x = torch.randn(Mpad, K, generator=g).bfloat16()
    cu = [0]
    for q in qlens:
        cu.append(cu[-1] + q)
    c = dict(
        H=H, Hkv=Hkv, D=D, K=K, N=N, lin=lin, x=x.to(dev), kc=kc.to(dev), vc=vc.to(dev),
        pos=torch.tensor(pos, dtype=torch.int32, device=dev),
        slots=torch.tensor(slots, dtype=torch.int32, device=dev),
        cu_q=torch.tensor(cu, dtype=torch.int32, device=dev),
        ctx=torch.tensor(ctx, dtype=torch.int32, device=dev), bt=blocks.to(dev),
        max_q=max_q, max_ctx=max(ctx), B=B,
        cs=ref.rope_cos_sin(D, 2048, 500000.0).to(dev) if norm == "rms" else None)
    return c


def _run(c, fuse, *, S, rt, wr, ws, scr, out=None):
    ops.FUSE_QKV_ATTN = fuse
    kc, vc = c["kc"].clone(), c["vc"].clone()
    q = torch.empty(c["x"].shape[0], c["H"] * c["D"], dtype=torch.bfloat16, device=c["x"].device)
    ns, sk = ops.decode_attn_splits(c["max_ctx"], c["B"] * c["Hkv"], 128)
    scr.seed_stats(c["x"])
    a = ops.skinny_fused(
        c["x"], c["lin"], "rope", scr, splits=S, rt=rt, wr=wr, xl=0, eps=1e-5, rowsq_tiles=1,
        positions=c["pos"], cos_sin=c["cs"], q_out=q, k_cache=kc, v_cache=vc, slots=c["slots"],
        n_heads=c["H"], n_kv=c["Hkv"], head_dim=c["D"],
        attn=dict(cu_q=c["cu_q"], ctx_lens=c["ctx"], block_tables=c["bt"], max_q=c["max_q"],
                  split_keys=sk, num_splits=ns, workspace=ws, max_k=c["max_ctx"], out=out))
    torch.cuda.synchronize()
    T = int(c["cu_q"][-1])
    return q[:T].clone(), kc, vc, a[:T].clone()


@pytest.fixture
def restore_flag():
    old = ops.FUSE_QKV_ATTN
    yield
    ops.FUSE_QKV_ATTN = old


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["llama", "whisper"])
@pytest.mark.parametrize("Mpad", [16, 32, 64])
@pytest.mark.parametrize("rt,wr,S", [(1, 1, 1), (2, 1, 1), (2, 1, 2), (1, 4, 1), (2, 4, 1)])
@pytest.mark.parametrize("max_q", [1, 4])
def test_fused_qkv_attention_bitwise_gpu(restore_flag, shape, Mpad, rt, wr, S, max_q):
    c = _case(shape, Mpad, max_q, seed=Mpad * 7 + max_q)
    dev = c["x"].device
    if wr == 4 and c["N"] % (64 * rt):
        pytest.skip("4 waves along rows need N % (64 rt) == 0")
    if (c["N"] // (16 * rt * wr)) * S > torch.cuda.get_device_properties(dev).multi_processor_count:
        pytest.skip("grid larger than the CU count: not a fused-launch layout")
    ws = ops.AttnWorkspace(dev, 64, c["H"], c["D"], 64)
    scr = ops.FusedScratch(dev)
    ops.FUSE_QKV_ATTN = True
    ns, sk = ops.decode_attn_splits(c["max_ctx"], c["B"] * c["Hkv"], 128)
    plan = ops._attd_plan(c["x"], c["lin"], scr, S, rt, wr, 0, torch.empty(Mpad, c["H"] * c["D"],
                          dtype=torch.bfloat16, device=dev), c["kc"], c["H"], c["Hkv"], c["D"],
                          dict(cu_q=c["cu_q"], ctx_lens=c["ctx"], block_tables=c["bt"],
                               max_q=c["max_q"], split_keys=sk, num_splits=ns, workspace=ws),
                          None)
    assert plan is not None, "the fused launch must be the path under test"
    base = _run(c, False, S=S, rt=rt, wr=wr, ws=ws, scr=scr)
    fused = _run(c, True, S=S, rt=rt, wr=wr, ws=ws, scr=scr)
    for name, a, b in zip(("q", "k_cache", "v_cache", "attn"), fused, base):
        assert torch.equal(a, b), (name, float((a.float() - b.float()).abs().max()))
    # hand-off words back at zero (ready / work / exit) and no spin timeout
    assert int(ws.sync.abs().sum()) == 0, ws.sync[:80].tolist()
    assert int(ws.counters.abs().sum()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["llama", "whisper"])
def test_fused_qkv_attention_graph_replay_gpu(restore_flag, shape):
    """Captured once, replayed: every replay reproduces the eager two-launch
    result (the last workgroup out re-arms the hand-off words)."""
    c = _case(shape, 32, 1, seed=11)
    dev = c["x"].device
    ws = ops.AttnWorkspace(dev, 64, c["H"], c["D"], 64)
    scr = ops.FusedScratch(dev)
    base = _run(c, False, S=1, rt=2, wr=1, ws=ws, scr=scr)
    ops.FUSE_QKV_ATTN = True
    kc, vc = c["kc"].clone(), c["vc"].clone()
    q = torch.empty(32, c["H"] * c["D"], dtype=torch.bfloat16, device=dev)
    out = torch.empty(32, c["H"] * c["D"], dtype=torch.bfloat16, device=dev)
    ns, sk = ops.decode_attn_splits(c["max_ctx"], c["B"] * c["Hkv"], 128)
    scr.seed_stats(c["x"])
    kw = dict(splits=1, rt=2, wr=1, xl=0, eps=1e-5, rowsq_tiles=1, positions=c["pos"],
              cos_sin=c["cs"], q_out=q, k_cache=kc, v_cache=vc, slots=c["slots"], n_heads=c["H"],
              n_kv=c["Hkv"], head_dim=c["D"],
              attn=dict(cu_q=c["cu_q"], ctx_lens=c["ctx"], block_tables=c["bt"],
                        max_q=c["max_q"], split_keys=sk, num_splits=ns, workspace=ws, out=out))
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        ops.skinny_fused(c["x"], c["lin"], "rope", scr, **kw)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        ops.skinny_fused(c["x"], c["lin"], "rope", scr, **kw)
    T = int(c["cu_q"][-1])
    for _ in range(3):
        out.zero_()
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(out[:T], base[3])
        assert torch.equal(q[:T], base[0])
        assert int(ws.sync.abs().sum()) == 0


def test_fused_qkv_attention_cpu_falls_back():
    """On the CPU (and whenever the fused launch is unsupported) ``attn=``
    runs the GEMM and then :func:`ops.attention`."""
    torch.manual_seed(0)
    H, Hkv, D, K = 4, 2, 64, 256
    N = (H + 2 * Hkv) * D
    w = (torch.randn(N, K) * 0.05).bfloat16()
    nw = (torch.rand(K) + 0.5).bfloat16()
    lin = ops.FusedLinear(w, norm="rms", norm_w=nw, perm=ref.perm_rope_qkv(H, Hkv, D))
    scr = ops.FusedScratch("cpu", max_tiles=64, max_rows=16)
    x = torch.randn(16, K).bfloat16()
    scr.seed_stats(x)
    kc = torch.zeros(8, Hkv, 16, D).bfloat16()
    vc = torch.zeros_like(kc)
    bt = torch.tensor([[0, 1], [2, 3]], dtype=torch.int32)
    slots = torch.tensor([0, 32] + [-1] * 14, dtype=torch.int32)
    pos = torch.zeros(16, dtype=torch.int32)
    cu = torch.tensor([0, 1, 2], dtype=torch.int32)
    ctx = torch.tensor([1, 1], dtype=torch.int32)
    cs = ref.rope_cos_sin(D, 64, 10000.0)
    q = torch.empty(16, H * D).bfloat16()
    ws = ops.AttnWorkspace("cpu", 16, H, D, 4)
    a = ops.skinny_fused(x, lin, "rope", scr, eps=1e-5, rowsq_tiles=1, positions=pos, cos_sin=cs,
                         q_out=q, k_cache=kc, v_cache=vc, slots=slots, n_heads=H, n_kv=Hkv,
                         head_dim=D,
                         attn=dict(cu_q=cu, ctx_lens=ctx, block_tables=bt, max_q=1,
                                   split_keys=128, num_splits=1, workspace=ws))
    # one key per sequence: attention returns that token's own v row per head
    G = H // Hkv
    for b, slot in enumerate((0, 32)):
        blkid, off = slot // 16, slot % 16
        for h in range(H):
            v = vc[blkid, h // G, off].float()
            assert torch.allclose(a[b, h * D:(h + 1) * D].float(), v, atol=1e-2)


def _xcase(Mpad, max_q, seed=0, n_audio=1500):
    """Whisper large-v3 cross-attention step: q projection (LayerNorm
    prologue + bias) of the decoder rows, K / V = per-utterance encoder rows."""
    H, D, K = 20, 64, 1280
    g = torch.Generator().manual_seed(seed)
    dev = torch.device("cuda", 0)
    w = (torch.randn(K, K, generator=g) * 0.02).bfloat16()
    nw = (torch.rand(K, generator=g) + 0.5).bfloat16()
    nb_ = (torch.randn(K, generator=g) * 0.1).bfloat16()
    bias = (torch.randn(K, generator=g) * 0.1).bfloat16()
    lin = ops.FusedLinear(w.to(dev), norm="ln", norm_w=nw.to(dev), norm_b=nb_.to(dev),
                          bias=bias.to(dev))
    B = max(1, Mpad // max_q - (1 if Mpad // max_q > 2 else 0))
    qlens = [max_q if b % 3 else max(1, max_q // 2) for b in range(B)]
    cu = [0]
    for q in qlens:
        cu.append(cu[-1] + q)
    gd = torch.Generator(device=dev).manual_seed(seed)
    kv = (torch.randn(B * n_audio, 2 * K, generator=gd, device=dev) * 0.5).bfloat16()
    return dict(H=H, D=D, K=K, lin=lin, x=torch.randn(Mpad, K, generator=g).bfloat16().to(dev),
                kv=kv, cu_q=torch.tensor(cu, dtype=torch.int32, device=dev),
                starts=torch.arange(B, dtype=torch.int32, device=dev) * n_audio,
                lens=torch.full((B,), n_audio, dtype=torch.int32, device=dev), max_q=max_q, B=B)


def _xrun(c, fuse, *, S, rt, wr, ws, scr, split_keys=512):
    ops.FUSE_QKV_ATTN = fuse
    Mpad = c["x"].shape[0]
    out = torch.empty(Mpad, c["K"], dtype=torch.bfloat16, device=c["x"].device)
    ns = -(-1500 // split_keys)
    scr.seed_stats(c["x"])
    a = ops.skinny_fused(
        c["x"], c["lin"], "act", scr, splits=S, rt=rt, wr=wr, xl=0, eps=1e-5, rowsq_tiles=1,
        out=out, n_heads=c["H"], n_kv=c["H"], head_dim=c["D"],
        attn=dict(cu_q=c["cu_q"], ctx_lens=c["lens"], kv_start=c["starts"], k=c["kv"],
                  v=c["kv"][:, c["K"]:], max_q=c["max_q"], split_keys=split_keys, num_splits=ns,
                  workspace=ws))
    torch.cuda.synchronize()
    T = int(c["cu_q"][-1])
    return out[:T].clone(), a[:T].clone()


@pytest.mark.gpu
@pytest.mark.parametrize("Mpad", [16, 32, 64])
@pytest.mark.parametrize("rt,wr,S", [(1, 1, 1), (2, 1, 1), (1, 1, 2), (1, 4, 1), (2, 4, 1)])
@pytest.mark.parametrize("max_q", [1, 4])
def test_fused_xq_cross_attention_bitwise_gpu(restore_flag, Mpad, rt, wr, S, max_q):
    """The Whisper cross-attention hand-off (act mode: q projection ->
    attention over the encoder rows) equals the two launches bit for bit."""
    c = _xcase(Mpad, max_q, seed=Mpad + max_q)
    dev = c["x"].device
    ws = ops.AttnWorkspace(dev, 64, c["H"], c["D"], 64)
    scr = ops.FusedScratch(dev)
    ops.FUSE_QKV_ATTN = True
    plan = ops._attd_plan(c["x"], c["lin"], scr, S, rt, wr, 0,
                          torch.empty(Mpad, c["K"], dtype=torch.bfloat16, device=dev), c["kv"],
                          c["H"], c["H"], c["D"],
                          dict(cu_q=c["cu_q"], ctx_lens=c["lens"], kv_start=c["starts"],
                               k=c["kv"], v=c["kv"][:, c["K"]:], max_q=c["max_q"],
                               split_keys=512, num_splits=3, workspace=ws), None, "act", "none")
    assert plan is not None, "the fused launch must be the path under test"
    base = _xrun(c, False, S=S, rt=rt, wr=wr, ws=ws, scr=scr)
    fused = _xrun(c, True, S=S, rt=rt, wr=wr, ws=ws, scr=scr)
    for name, a, b in zip(("xq", "attn"), fused, base):
        assert torch.equal(a, b), (name, float((a.float() - b.float()).abs().max()))
    assert int(ws.sync.abs().sum()) == 0, ws.sync[:80].tolist()
    assert int(ws.counters.abs().sum()) == 0
