"""Split-K tiled MFMA GEMM with the in-launch reduction (csrc/kernels/gemm_sk.hip)
against the fp32 torch reference of the same op: every layout, K-chunk count
and epilogue (bf16 + bias, SwiGLU, residual add), ragged M, and the bitwise
determinism of the last-arriver reduction."""
import pytest
import torch

from loqa_hub_amd import ops


def _rel(a, b):
    return (a.float().cpu() - b.float().cpu()).abs().max().item() / max(b.float().abs().max().item(), 1e-6)


def test_gemm_sk_cpu_reference_and_plan():
    torch.manual_seed(0)
    x = torch.randn(33, 128).bfloat16()
    w = torch.randn(256, 128).bfloat16()
    y = ops.gemm_sk(x, w)
    assert _rel(y, x.float() @ w.float().t()) < 1e-2
    res = torch.randn(33, 256).bfloat16()
    r0 = res.clone()
    out = ops.gemm_sk(x, w, epi="resid", residual=res)
    assert out is res and _rel(res, r0.float() + x.float() @ w.float().t()) < 1e-2
    sw = ops.gemm_sk(x, w, epi="swiglu")
    assert sw.shape == (33, 128)
    # the planner always returns a tileable layout
    for M, N, K in ((295, 6144, 4096), (295, 4096, 14336), (420, 28672, 4096), (1500, 3840, 1280),
                    (3000, 5120, 1280), (64, 4096, 4096)):
        for epi in ("bf16", "swiglu", "resid"):
            lay, s = ops.gemm_sk_plan(M, N, K, epi)
            bn = ops.SK_LAYOUTS[lay][0]
            assert N % bn == 0 and 1 <= s <= K // 64


@pytest.mark.gpu
@pytest.mark.parametrize("layout", sorted(ops.SK_LAYOUTS))
def test_gemm_sk_gpu_matches_fp32(layout):
    dev = torch.device("cuda", 0)
    torch.manual_seed(layout)
    bn, bm = ops.SK_LAYOUTS[layout][:2]
    for M, K in ((bm * 2 + 37, 512), (17, 256), (300, 1024)):
        N = bn * 3
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        b = torch.randn(N, device=dev) * 0.1
        for S in (1, 2, 3, 5):
            if S > K // 64:
                continue
            y = ops.gemm_sk(x, w, bias=b, layout=layout, splits=S)
            r = ops._sk_ref(x.cpu(), w.cpu(), "bf16", b.cpu(), None)
            assert _rel(y, r) < 1e-2, (layout, M, K, S)
            res = torch.randn(M, N, device=dev).bfloat16()
            rr = ops._sk_ref(x.cpu(), w.cpu(), "resid", None, res.cpu())
            ops.gemm_sk(x, w, epi="resid", residual=res, layout=layout, splits=S)
            assert _rel(res, rr) < 1e-2, (layout, M, K, S, "resid")
            sw = ops.gemm_sk(x, w, epi="swiglu", layout=layout, splits=S)
            rs = ops._sk_ref(x.cpu(), w.cpu(), "swiglu", None, None)
            assert _rel(sw, rs) < 2e-2, (layout, M, K, S, "swiglu")


@pytest.mark.gpu
def test_gemm_sk_split_reduction_is_deterministic():
    """The last arriver sums the K chunks in fixed order: repeated launches give
    bitwise-identical outputs although the arrival order varies."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    x = torch.randn(301, 4096, device=dev).bfloat16()
    w = (torch.randn(4096, 4096, device=dev) * 0.02).bfloat16()
    ref = ops.gemm_sk(x, w, layout=1, splits=6)
    for _ in range(5):
        assert torch.equal(ops.gemm_sk(x, w, layout=1, splits=6), ref)
    assert _rel(ref, ops._sk_ref(x.cpu(), w.cpu(), "bf16", None, None)) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["test-whisper", "whisper-large-v3"])
def test_whisper_encoder_sk_matches_library_path(monkeypatch, name):
    """Every encoder projection on the split-K tiled GEMM (qkv + bias, o +
    bias into the residual, fc1 + bias + GELU, fc2 + bias into the residual)
    against the hipBLASLt / slab path on the same weights."""
    from loqa_hub_amd.models import whisper as wm
    from loqa_hub_amd.models.configs import whisper_config

    dev = torch.device("cuda", 0)
    cfg = whisper_config(name, n_mels=128, enc_layers=3)
    w = wm.WhisperWeights(cfg, dev, seed=3)
    model = wm.WhisperModel(w)
    g = torch.Generator(device=dev).manual_seed(5)
    audio = (torch.rand(2, 480000, device=dev, generator=g) - 0.5) * 0.2
    monkeypatch.setattr(wm, "ENC_SK", 1)
    a = model.encode(audio)
    monkeypatch.setattr(wm, "ENC_SK", 0)
    b = model.encode(audio)
    assert a.shape == b.shape == (2 * 1500, cfg.d_model)
    assert torch.isfinite(a.float()).all()
    err = (a.float() - b.float()).abs()
    assert err.max().item() < 0.05 * b.float().abs().max().item(), err.max().item()
    assert err.mean().item() < 0.01 * b.float().abs().mean().item() + 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [0, 1])
def test_gemm_ws_gpu_matches_fp32(depth):
    """Row-resident weight-streaming GEMM: every row-block size, ragged M,
    every epilogue, against the fp32 reference."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(10 + depth)
    for M, N, K in ((300, 384, 512), (17, 256, 128), (385, 128, 256), (1000, 256, 192), (64, 512, 64)):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        b = torch.randn(N, device=dev) * 0.1
        y = ops.gemm_ws(x, w, bias=b, act="gelu", depth=depth)
        assert _rel(y, ops._sk_ref(x.cpu(), w.cpu(), "bf16", b.cpu(), None, "gelu")) < 1e-2, (M, N, K)
        res = torch.randn(M, N, device=dev).bfloat16()
        rr = ops._sk_ref(x.cpu(), w.cpu(), "resid", b.cpu(), res.cpu())
        ops.gemm_ws(x, w, epi="resid", residual=res, bias=b, depth=depth)
        assert _rel(res, rr) < 1e-2, (M, N, K, "resid")
        sw = ops.gemm_ws(x, w, epi="swiglu", depth=depth)
        assert _rel(sw, ops._sk_ref(x.cpu(), w.cpu(), "swiglu", None, None)) < 2e-2, (M, N, K, "swiglu")
    # explicit row blocks, every size the kernel takes
    x = torch.randn(700, 256, device=dev).bfloat16()
    w = (torch.randn(256, 256, device=dev) * 0.05).bfloat16()
    ref = ops._sk_ref(x.cpu(), w.cpu(), "bf16", None, None)
    for bm in (64, 128, 192, 256) + ((320, 384) if depth == 0 else ()):
        assert _rel(ops.gemm_ws(x, w, depth=depth, bm=bm), ref) < 1e-2, bm


@pytest.mark.gpu
@pytest.mark.parametrize("depth", [0, 1])
def test_gemm_ws_splitk_gpu_matches_fp32(depth):
    """Weight-streaming GEMM with the K range split over workgroups and summed
    in-launch: every epilogue, ragged M, uneven K chunks, against the fp32
    reference; the split result does not depend on which chunk lands last
    (two launches bitwise equal); counters left zero for the next launch."""
    dev = torch.device("cuda", 0)
    torch.manual_seed(20 + depth)
    for M, N, K, S in ((300, 384, 1024, 4), (17, 256, 640, 3), (300, 256, 14336 // 8, 7),
                       (129, 128, 512, 8), (64, 512, 256, 2)):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        b = torch.randn(N, device=dev) * 0.1
        y = ops.gemm_ws(x, w, bias=b, act="gelu", depth=depth, splits=S)
        assert _rel(y, ops._sk_ref(x.cpu(), w.cpu(), "bf16", b.cpu(), None, "gelu")) < 1e-2, (M, N, K, S)
        assert torch.equal(y, ops.gemm_ws(x, w, bias=b, act="gelu", depth=depth, splits=S))
        res = torch.randn(M, N, device=dev).bfloat16()
        rr = ops._sk_ref(x.cpu(), w.cpu(), "resid", b.cpu(), res.cpu())
        ops.gemm_ws(x, w, epi="resid", residual=res, bias=b, depth=depth, splits=S)
        assert _rel(res, rr) < 1e-2, (M, N, K, S, "resid")
        sw = ops.gemm_ws(x, w, epi="swiglu", depth=depth, splits=S)
        assert _rel(sw, ops._sk_ref(x.cpu(), w.cpu(), "swiglu", None, None)) < 2e-2, (M, N, K, S)
    torch.cuda.synchronize()
    for (_, st), (_, cnt) in ops._SK_WS.items():
        assert int(cnt.abs().sum()) == 0
