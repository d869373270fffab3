"""Fused-epilogue decode GEMMs (RMSNorm prologue; RoPE+KV-append / residual +
row-sumsq / SwiGLU epilogues; in-launch split-K reduce) against the unfused
skinny-GEMM + slab-consumer path, on the CPU (reference semantics of the
weight permutations) and on the GPU (the HIP kernels)."""
import pytest
import torch

from loqa_hub_amd import ops


def _decode_logits(eng, fused: bool, seq_base: int, tok, Mpad: int):
    from loqa_hub_amd.engine.llm_engine import GenRequest
    pool = eng.kv.pool
    seqs = []
    for i in range(len(tok)):
        r = GenRequest([], [])
        r.seq_id = seq_base + i
        pool.add_seq(r.seq_id, [])
        seqs.append(r)
    outs = []
    feeds = [t[:5] for t in tok]
    for step in range(3):  # a 5-token step then single-token steps (cache grows)
        max_q, max_ctx, host = eng._meta(seqs, feeds, True, len(tok), Mpad)
        dev = eng._to_device(host)
        meta = eng._build_meta(dev, max_q, max_ctx, True)
        if fused:
            lg = eng.model.forward_decode_fused(meta, eng.kv.k, eng.kv.v, eng.attn_ws, eng.scratch)
        else:
            lg = eng.model.forward_decode(meta, eng.kv.k, eng.kv.v, eng.attn_ws)
        outs.append(lg[: len(tok)].float().cpu())
        feeds = [[t[5 + step]] for t in tok]
    return outs


def _compare(device, splits=None, Mpad=16):
    from loqa_hub_amd.engine.llm_engine import LLMEngine
    from loqa_hub_amd.models.configs import llama_config
    eng = LLMEngine(llama_config("test-tiny"), device, max_seqs=8, use_graphs=False)
    if splits is not None:  # force split-K (exercises the in-launch reducer)
        for key in list(ops._SPLITS):
            del ops._SPLITS[key]
        d = eng.cfg.d_model
        for N, K in ((eng.weights.h * 64 + 2 * eng.weights.hkv * 64, d), (d, eng.weights.h * 64),
                     (2 * eng.weights.f, d), (d, eng.weights.f)):
            for mp in (16, 32, 64):
                s = max(x for x in ops.SPLIT_CANDIDATES if x <= splits and K % (x * 128) == 0)
                ops._SPLITS[(N, K, mp)] = s
        saved = dict(ops._FSPLITS)
        ops._FSPLITS.clear()
    g = torch.Generator().manual_seed(3)
    tok = torch.randint(10, 4000, (3, 12), generator=g).tolist()
    a = _decode_logits(eng, True, 100, tok, Mpad)
    b = _decode_logits(eng, False, 200, tok, Mpad)
    for x, y in zip(a, b):
        rel = float((x - y).norm() / (y.norm() + 1e-12))
        assert rel < 2e-2, rel
    ops._SPLITS.clear()
    if splits is not None:
        ops._FSPLITS.update(saved)


def test_fused_decode_matches_unfused_cpu():
    _compare("cpu")


def test_permutations_are_bijections():
    from loqa_hub_amd.ops import reference as ref
    p = ref.perm_rope_qkv(32, 8, 128)
    assert sorted(p.tolist()) == list(range((32 + 16) * 128))
    g = ref.perm_gate_up(14336)
    assert sorted(g.tolist()) == list(range(2 * 14336))


@pytest.mark.gpu
@pytest.mark.parametrize("splits,Mpad", [(None, 16), (1, 16), (2, 16), (None, 64), (2, 64)])
def test_fused_decode_matches_unfused_gpu(splits, Mpad):
    _compare("cuda", splits, Mpad)


@pytest.mark.gpu
def test_fused_resid_rowsq_and_silu_gpu():
    """Kernel-level: residual epilogue + row sum-of-squares, then the RMSNorm
    prologue of a SwiGLU GEMM, against the reference chain."""
    from loqa_hub_amd.ops import reference as ref
    dev = "cuda"
    torch.manual_seed(0)
    Mpad, d, F = 16, 1024, 2048
    scr = ops.FusedScratch(dev)
    x = torch.randn(Mpad, 512, device=dev).bfloat16()
    wo = ops.shuffle_weight((torch.randn(d, 512, device=dev) * 0.05).bfloat16())
    res1 = torch.randn(Mpad, d, device=dev).bfloat16()
    res2 = res1.clone()
    for S in (1, 4):
        ops.skinny_fused(x, wo, "resid", scr, splits=S, residual=res1)
        part = ops.skinny_gemm(x, wo, S)
        ops.slab_rmsnorm(part, res2, torch.ones(d, device=dev).bfloat16(), 1e-5)
        assert torch.equal(res1, res2)
    sq = scr.rowsq[: (d // 32) * Mpad].view(d // 32, Mpad).sum(0)
    assert torch.allclose(sq, res1.float().pow(2).sum(1), rtol=1e-3)
    wgu = (torch.randn(2 * F, d, device=dev) * 0.03).bfloat16()
    wn = torch.rand(d, device=dev).bfloat16() + 0.5
    wp = ops.shuffle_weight(ops.fold_norm(wgu, wn)[ref.perm_gate_up(F).to(dev)].contiguous())
    for S in (1, 2):
        a = ops.skinny_fused(res1, wp, "silu", scr, splits=S, norm=True, eps=1e-5,
                             rowsq_tiles=d // 32)
        h = ref.rmsnorm(res1, wn, 1e-5)
        expect = ref.silu_mul((h.float() @ wgu.float().t()).bfloat16())
        assert float((a.float() - expect.float()).norm() / expect.float().norm()) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["resid", "silu", "act", "rope"])
@pytest.mark.parametrize("Mpad,rt", [(16, 1), (16, 2), (32, 1), (32, 2), (64, 1), (64, 2), (64, 4)])
def test_fused_rows_per_wave_layout_gpu(mode, Mpad, rt):
    """Every (rt, wr) layout of the fused GEMM against the fp32 CPU reference of
    the same call: 16-row pair tiles (SwiGLU / RoPE partners exchanged across
    lanes l, l ^ 32) and 4-waves-along-rows tiles."""
    from loqa_hub_amd.ops import reference as ref
    torch.manual_seed(3)
    K = 1024
    H, Hkv, D = 8, 2, 64
    N = {"resid": 512, "silu": 1024, "act": 512, "rope": (H + 2 * Hkv) * D}[mode]
    x = torch.randn(Mpad, K).bfloat16()
    w = (torch.randn(N, K) * 0.03).bfloat16()
    if mode == "silu":
        w = w[ref.perm_gate_up(N // 2)].contiguous()
    elif mode == "rope":
        w = w[ref.perm_rope_qkv(H, Hkv, D)].contiguous()
    res0 = torch.randn(Mpad, N).bfloat16()
    cs = ref.rope_cos_sin(D, 256, 10000.0)

    def run(dev, wr):
        wp = ops.shuffle_weight(w.to(dev))
        scr = ops.FusedScratch(dev)
        kw = dict(splits=1, wr=wr, rt=rt)
        xd = x.to(dev)
        if mode == "resid":
            res = res0.clone().to(dev)
            ops.skinny_fused(xd, wp, "resid", scr, residual=res, **kw)
            return [res.float().cpu(), scr.rowsq[: (N // (16 * rt)) * Mpad].float().cpu()]
        if mode == "rope":
            kc = torch.zeros(4, Hkv, 16, D, device=dev).bfloat16()
            vc = torch.zeros_like(kc)
            pos = (torch.arange(Mpad, dtype=torch.int32) * 3 + 5).to(dev)
            slots = torch.arange(Mpad, dtype=torch.int32, device=dev)
            q = torch.empty(Mpad, H * D, device=dev).bfloat16()
            ops.skinny_fused(xd, wp, "rope", scr, positions=pos, cos_sin=cs.to(dev), q_out=q,
                             k_cache=kc, v_cache=vc, slots=slots, n_heads=H, n_kv=Hkv,
                             head_dim=D, **kw)
            return [q.float().cpu(), kc.float().cpu(), vc.float().cpu()]
        return [ops.skinny_fused(xd, wp, mode, scr, **kw).float().cpu()]

    expect = run("cpu", 1)
    for wr in (1, 4):
        got = run("cuda", wr)
        for a, b in zip(got, expect):
            rel = float((a - b).norm() / b.norm().clamp_min(1e-6))
            assert rel < 1e-2, (wr, rel)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["resid", "silu", "act", "rope"])
@pytest.mark.parametrize("Mpad,rt,S", [(32, 1, 1), (32, 2, 2), (32, 2, 4), (64, 1, 1), (64, 2, 2),
                                       (128, 1, 1), (128, 1, 2), (128, 2, 1), (128, 2, 4)])
@pytest.mark.parametrize("norm", [None, "rms"])
def test_fused_xl_layout_gpu(mode, Mpad, rt, S, norm):
    """The x-through-LDS (XL) layout of the fused GEMM (Mpad 32 / 64 / 128, 4 waves
    along rows, per-wave split-K tickets) against the fp32 CPU reference of
    the same call, with and without the RMSNorm prologue."""
    from loqa_hub_amd.ops import reference as ref
    if norm and mode == "resid":
        pytest.skip("no residual GEMM takes a norm prologue (it would rewrite the statistics it reads)")
    torch.manual_seed(5)
    K = 1024
    H, Hkv, D = 8, 2, 64
    N = {"resid": 512, "silu": 1024, "act": 512, "rope": (H + 2 * Hkv) * D}[mode]
    x = torch.randn(Mpad, K).bfloat16()
    w = (torch.randn(N, K) * 0.03).bfloat16()
    if mode == "silu":
        w = w[ref.perm_gate_up(N // 2)].contiguous()
    elif mode == "rope":
        w = w[ref.perm_rope_qkv(H, Hkv, D)].contiguous()
    res0 = torch.randn(Mpad, N).bfloat16()
    cs = ref.rope_cos_sin(D, 512, 10000.0)
    tiles = 4
    rowsq = torch.rand(tiles * Mpad) * 300 + 50

    def run(dev):
        wp = ops.shuffle_weight(w.to(dev))
        scr = ops.FusedScratch(dev)
        kw = dict(splits=S, wr=4, rt=rt, xl=1)
        if norm:
            scr.rowsq[: tiles * Mpad].copy_(rowsq.to(dev))
            kw.update(norm=norm, rowsq_tiles=tiles)
        xd = x.to(dev)
        if mode == "resid":
            res = res0.clone().to(dev)
            ops.skinny_fused(xd, wp, "resid", scr, residual=res, **kw)
            return [res.float().cpu(), scr.rowsq[: (N // (16 * rt)) * Mpad].float().cpu()]
        if mode == "rope":
            kc = torch.zeros(Mpad // 16, Hkv, 16, D, device=dev).bfloat16()
            vc = torch.zeros_like(kc)
            pos = (torch.arange(Mpad, dtype=torch.int32) * 3 + 5).to(dev)
            slots = torch.arange(Mpad, dtype=torch.int32, device=dev)
            q = torch.empty(Mpad, H * D, device=dev).bfloat16()
            ops.skinny_fused(xd, wp, "rope", scr, positions=pos, cos_sin=cs.to(dev), q_out=q,
                             k_cache=kc, v_cache=vc, slots=slots, n_heads=H, n_kv=Hkv,
                             head_dim=D, **kw)
            return [q.float().cpu(), kc.float().cpu(), vc.float().cpu()]
        return [ops.skinny_fused(xd, wp, mode, scr, **kw).float().cpu()]

    expect = run("cpu")
    got = run("cuda")
    for a, b in zip(got, expect):
        rel = float((a - b).norm() / b.norm().clamp_min(1e-6))
        assert rel < 1e-2, rel


def _ln_case(dev, S=None, Mpad=16, rt=2, xl=None):
    """LayerNorm-prologue GEMM (folded weight / shift / bias) with a GELU
    epilogue, against layernorm -> linear -> gelu in fp32."""
    torch.manual_seed(1)
    K, N = 512, 768
    x = (torch.randn(Mpad, K, device=dev) * 2 + 0.5).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    g = (torch.rand(K, device=dev) + 0.5).bfloat16()
    b = (torch.randn(K, device=dev) * 0.1).bfloat16()
    bias = (torch.randn(N, device=dev) * 0.1).bfloat16()
    lin = ops.FusedLinear(w, norm="ln", norm_w=g, norm_b=b, bias=bias)
    scr = ops.FusedScratch(dev)
    scr.seed_stats(x)
    y = ops.skinny_fused(x, lin, "act", scr, splits=S, act="gelu", eps=1e-5, rowsq_tiles=1, rt=rt,
                         xl=xl)
    h = torch.nn.functional.layer_norm(x.float(), (K,), g.float(), b.float(), 1e-5)
    expect = torch.nn.functional.gelu(h @ w.float().t() + bias.float())
    rel = float((y.float() - expect).norm() / expect.norm())
    assert rel < 2e-2, rel
    # residual epilogue with row sums feeds the next LayerNorm prologue
    res = x.clone()
    a = (torch.randn(Mpad, N, device=dev) * 0.5).bfloat16()
    wo = (torch.randn(K, N, device=dev) * 0.05).bfloat16()
    ops.skinny_fused(a, ops.FusedLinear(wo, bias=bias[:K]), "resid", scr,
                     splits=S, residual=res, row_sums=True, rt=rt, xl=xl)
    tiles = K // (16 * rt)
    assert scr.stat_tiles == tiles
    sm = scr.rowsum[: tiles * Mpad].view(tiles, Mpad).sum(0)
    sq = scr.rowsq[: tiles * Mpad].view(tiles, Mpad).sum(0)
    assert torch.allclose(sm, res.float().sum(1), rtol=1e-3, atol=1e-2)
    assert torch.allclose(sq, res.float().pow(2).sum(1), rtol=1e-3)


def test_fused_layernorm_act_cpu():
    _ln_case("cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("S,Mpad,rt", [(1, 16, 2), (2, 16, 2), (1, 64, 2), (2, 32, 2),
                                       (1, 16, 1), (2, 32, 1), (2, 64, 1)])
def test_fused_layernorm_act_gpu(S, Mpad, rt):
    _ln_case("cuda", S, Mpad, rt)


@pytest.mark.gpu
@pytest.mark.parametrize("S,Mpad,rt", [(1, 128, 1), (2, 128, 2), (1, 64, 1), (1, 32, 2)])
def test_fused_layernorm_act_xl_gpu(S, Mpad, rt):
    _ln_case("cuda", S, Mpad, rt, xl=1)


@pytest.mark.gpu
def test_whisper_fused_decode_matches_fast_gpu():
    """Whisper decoder step: fused-epilogue path vs the skinny-GEMM + slab path."""
    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.engine.synthetic import make_batch
    from loqa_hub_amd.models.configs import whisper_config
    from loqa_hub_amd.models.whisper import decode_step_fast, decode_step_fused
    cfg = whisper_config("test-whisper")
    utts = make_batch(1, 3, [1, 2, 3])
    eng = STTEngine(cfg, torch.device("cuda"), seed=3, max_batch=4, use_graphs=False)
    outs = {}
    for mode in ("fused", "fast"):
        reqs = [STTRequest(u.pcm) for u in utts]
        audio, _ = eng.upload(reqs)
        eng.cross_kv(eng.model.encode(audio))
        for i, r in enumerate(reqs):
            r.seq_id = eng._next
            r.slot = i
            r.feed = list(eng.sot)
            eng._next += 1
            eng.kv.pool.add_seq(r.seq_id, [])
        res = []
        for step in range(3):
            max_q, host = eng._host_meta(reqs, 4, 16)
            dev = eng._dev(host)
            args = (eng.model, dev["tokens"], dev["positions"], dev["slots"], dev["cu_q"],
                    dev["ctx_lens"], dev["block_tables"], max_q, eng.kv.k, eng.kv.v, eng.xkv,
                    dev["enc_starts"], dev["enc_lens"], dev["logit_idx"], eng.ws)
            if mode == "fused":
                lg = decode_step_fused(*args, eng.scratch, eng.self_splits)
            else:
                lg = decode_step_fast(*args, eng.self_splits)
            res.append(lg[:3, : cfg.vocab_size].float().cpu())
            for i, r in enumerate(reqs):
                r.feed = [11 + step + i]
        outs[mode] = res
    for a, b in zip(outs["fused"], outs["fast"]):
        rel = float((a - b).norm() / b.norm())
        assert rel < 2e-2, rel


def test_fused_scratch_holds_70b_mpad128():
    """Row statistics for the largest decode GEMM at the largest Mpad: the 70B
    gate|up (N = 57344) at Mpad 128 with 16-row tiles (config 5's tuner runs
    it)."""
    scr = ops.FusedScratch(torch.device("cpu"))
    ntiles = 57344 // 16
    assert ntiles <= scr.counters.numel() and ntiles * 128 <= scr.rowsq.numel()
