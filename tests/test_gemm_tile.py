"""LDS-tiled MFMA GEMM (csrc/kernels/gemm_tile.hip): the GPU kernel against the
fp32 torch reference of the same op, every layout and epilogue, and the
implicit-im2col conv stem against torch's conv1d."""
import pytest
import torch

from loqa_hub_amd import ops


def test_conv_k3_reference_matches_torch_conv1d():
    torch.manual_seed(0)
    B, cin, tin, cout = 2, 64, 37, 128
    x = torch.randn(B, cin, tin)
    w = torch.randn(cout, cin, 3) * 0.1
    wt = ops.conv_k3_weight(w.reshape(cout, cin * 3).bfloat16(), cin)
    xt = x.transpose(1, 2).reshape(B * tin, cin).bfloat16()
    for stride in (1, 2):
        ref = torch.nn.functional.conv1d(x.bfloat16().float(), w.bfloat16().float(), padding=1,
                                         stride=stride)
        y = ops.gemm_tile(xt, wt, conv=(B, stride)).float()
        r = ref.transpose(1, 2).reshape(-1, cout)
        assert y.shape == r.shape
        assert (y - r).abs().max().item() < 2e-2 * r.abs().max().item()


def test_gemm_tile_cpu_epilogues():
    torch.manual_seed(1)
    x = torch.randn(70, 128).bfloat16()
    w = torch.randn(256, 128).bfloat16()
    part = ops.gemm_tile(x, w, epi="slabs", splits=2)
    full = x.float() @ w.float().t()
    assert torch.allclose(part.sum(0), full, atol=1e-3, rtol=1e-3)
    sw = ops.gemm_tile(x, w, epi="swiglu").float()
    g, u = full[:, :128].bfloat16().float(), full[:, 128:].bfloat16().float()
    assert torch.allclose(sw, (g * torch.sigmoid(g) * u).bfloat16().float(), atol=5e-2, rtol=2e-2)


def _rel(a, b):
    return (a.float().cpu() - b.float().cpu()).abs().max().item() / max(b.float().abs().max().item(), 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", list(range(10)))
def test_gemm_tile_gpu_matches_fp32(layout):
    dev = torch.device("cuda", 0)
    torch.manual_seed(layout)
    for M, N, K in ((300, 512, 256), (1500, 768, 1280), (64, 256, 192)):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        b = torch.randn(N, device=dev) * 0.1
        pos = torch.randn(7, N, device=dev).bfloat16()
        y = ops.gemm_tile(x, w, bias=b, act="gelu", pos=pos, layout=layout)
        r = ops._gt_ref(x.cpu(), w.cpu(), b.cpu(), "gelu", pos.cpu(), "bf16", 1)
        assert _rel(y, r) < 1e-2, (layout, M, N, K)
        if K % 128 == 0:
            p = ops.gemm_tile(x, w, epi="slabs", splits=2, layout=layout)
            rp = ops._gt_ref(x.cpu(), w.cpu(), None, None, None, "slabs", 2)
            assert _rel(p, rp) < 1e-3, (layout, M, N, K)
        s = ops.gemm_tile(x, w, epi="swiglu", layout=layout)
        rs = ops._gt_ref(x.cpu(), w.cpu(), None, None, None, "swiglu", 1)
        assert _rel(s, rs) < 2e-2, (layout, M, N, K)


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1, 2])
def test_gemm_tile_conv_stem_gpu(stride):
    dev = torch.device("cuda", 0)
    torch.manual_seed(stride)
    B, cin, tin, cout = 2, 128, 300, 256
    x = torch.randn(B, cin, tin, device=dev)
    w = torch.randn(cout, cin, 3, device=dev) * 0.05
    b = torch.randn(cout, device=dev) * 0.1
    xt = x.transpose(1, 2).reshape(B * tin, cin).contiguous().bfloat16()
    wt = ops.conv_k3_weight(w.reshape(cout, cin * 3).bfloat16(), cin)
    for layout in (0, 2):
        y = ops.gemm_tile(xt, wt, bias=b, act="gelu", conv=(B, stride), layout=layout)
        ref = torch.nn.functional.conv1d(x.bfloat16().float(), w.bfloat16().float(), b, padding=1,
                                         stride=stride)
        ref = torch.nn.functional.gelu(ref.transpose(1, 2).reshape(-1, cout))
        assert _rel(y, ref) < 2e-2, layout


@pytest.mark.gpu
def test_whisper_encoder_tiled_stem_matches_library_path(monkeypatch):
    """The encoder with the conv stem and fc2 on the tiled GEMM (128 mels, as
    large-v3) against the im2col + hipBLASLt path on the same weights."""
    from loqa_hub_amd.models import whisper as wm
    from loqa_hub_amd.models.configs import whisper_config

    dev = torch.device("cuda", 0)
    cfg = whisper_config("test-whisper", n_mels=128, enc_layers=3)
    w = wm.WhisperWeights(cfg, dev, seed=3)
    model = wm.WhisperModel(w)
    g = torch.Generator(device=dev).manual_seed(5)
    audio = (torch.rand(2, 480000, device=dev, generator=g) - 0.5) * 0.2
    monkeypatch.setattr(wm, "ENC_TILE", 1)
    a = model.encode(audio)
    monkeypatch.setattr(wm, "ENC_TILE", 0)
    b = model.encode(audio)
    assert a.shape == b.shape == (2 * 1500, cfg.d_model)
    assert torch.isfinite(a.float()).all()
    err = (a.float() - b.float()).abs()
    assert err.max().item() < 0.05 * b.float().abs().max().item(), err.max().item()
    assert err.mean().item() < 0.01 * b.float().abs().mean().item() + 1e-3


@pytest.mark.gpu
def test_cross_kv_one_launch_matches_per_layer(monkeypatch):
    """Cross-attention K|V of all decoder layers as one tiled GEMM over the
    layer-concatenated weights against one hipBLASLt GEMM per layer: the
    K|V buffers agree to bf16 rounding and the greedy transcripts match."""
    import numpy as np

    from loqa_hub_amd.engine.stt_engine import STTEngine, STTRequest
    from loqa_hub_amd.models import whisper as wm
    from loqa_hub_amd.models.configs import whisper_config

    rng = np.random.default_rng(5)
    pcms = [(rng.standard_normal(n) * 3000).astype(np.int16) for n in (16000, 40000)]
    outs, kvs = [], []
    for flag in (1, 0):
        monkeypatch.setattr(wm, "XKV_TILE", flag)
        e = STTEngine(whisper_config("whisper-tiny"), "cuda", seed=4, max_batch=4)
        assert (e.xkv_all is not None) == bool(flag)
        reqs = [STTRequest(p, max_new_tokens=10) for p in pcms]
        e.transcribe(reqs)
        outs.append([r.tokens for r in reqs])
        kvs.append(torch.stack([x[:2 * 1500].float() for x in e.xkv]).cpu())
    err = (kvs[0] - kvs[1]).abs().max().item()
    assert err <= 2e-2 * kvs[1].abs().max().item(), err
    assert outs[0] == outs[1]


@pytest.mark.gpu
def test_encoder_graph_replay_matches_eager():
    """The captured encoder (one graph replay per batch) against the eager
    encoder on the same inputs, for two different inputs through one graph."""
    from loqa_hub_amd.engine.stt_engine import STTEngine
    from loqa_hub_amd.models.configs import whisper_config

    e = STTEngine(whisper_config("whisper-tiny"), "cuda", seed=6, max_batch=4)
    e._enc_graph(2)
    g = torch.Generator(device="cuda").manual_seed(9)
    for _ in range(2):
        audio = (torch.rand(2, 480000, device="cuda", generator=g) - 0.5) * 0.3
        ref = e.model.encode(audio).float()
        out = e.encode(audio).float()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
