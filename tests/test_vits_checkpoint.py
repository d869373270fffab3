"""Hugging Face VITS / MMS-TTS checkpoints through ``models/loader.load_vits``:
component parity against transformers' ``VitsModel`` (the oracle, fp32, run on
the CPU here) on a small random checkpoint written with ``save_pretrained``.

Compared piecewise, since the two sample differently: the text encoder
(hidden states and prior statistics), the stochastic duration predictor
(log durations from the same hidden states and the same noise), and the
reverse flow + HiFi-GAN vocoder (waveform from the same prior latents).
Our weights are bf16 on the conv path, so tolerances are bf16-sized; the
duration predictor runs fp32 and is held to fp32 tolerances."""
import json

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")

from loqa_hub_amd.models.loader import load_vits          # noqa: E402
from loqa_hub_amd.models.vits import VitsModel, text_to_ids  # noqa: E402

VOCAB = {c: i for i, c in enumerate("_ abcdefghijklmnopqrstuvwxyz.,'?!-")}


def _hf_model(sdp: bool = True, seed: int = 0, speakers: int = 1):
    from transformers import VitsConfig, VitsModel as HFVits
    torch.manual_seed(seed)
    extra = {"num_speakers": speakers, "speaker_embedding_size": 16} if speakers > 1 else {}
    cfg = VitsConfig(**extra,
        vocab_size=len(VOCAB), hidden_size=32, num_hidden_layers=2, num_attention_heads=2,
        window_size=4, ffn_dim=64, ffn_kernel_size=3, flow_size=32, spectrogram_bins=33,
        prior_encoder_num_flows=2, prior_encoder_num_wavenet_layers=2,
        posterior_encoder_num_wavenet_layers=1, upsample_initial_channel=256,
        upsample_rates=[8, 8, 2, 2], upsample_kernel_sizes=[16, 16, 4, 4],
        resblock_kernel_sizes=[3, 7, 11], resblock_dilation_sizes=[[1, 3, 5]] * 3,
        duration_predictor_num_flows=2, depth_separable_num_layers=2,
        use_stochastic_duration_prediction=sdp, noise_scale=0.667, noise_scale_duration=0.8,
        sampling_rate=16000)
    m = HFVits(cfg).eval()
    with torch.no_grad():
        # the zero-initialised parts (affine flow, biases, coupling post convs)
        # get values, so every path of the port is exercised
        for name, p in m.named_parameters():
            if name.startswith("posterior_encoder") or "post_" in name:
                continue
            if "cond" in name or "embed_speaker" in name:
                p.normal_(0.0, 0.3 if "embed_speaker" in name else 0.1)
            elif name.endswith(("translate", "log_scale")):
                p.normal_(0.0, 0.3)
            elif name.endswith(".bias"):
                p.normal_(0.0, 0.05)
            elif "flow.flows" in name and "conv_post" in name:
                p.normal_(0.0, 0.05)
            elif "norm" in name and name.endswith("weight"):
                p.normal_(1.0, 0.1)
    return m


DEVICES = ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)]


@pytest.fixture(scope="module")
def ckpt_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("mms_tts")
    m = _hf_model()
    m.save_pretrained(str(d), safe_serialization=True)
    (d / "vocab.json").write_text(json.dumps(VOCAB))
    return m, d


@pytest.fixture(scope="module", params=DEVICES)
def ckpt(request, ckpt_dir):
    """(HF model on the CPU, our config, our weights on the device, vocab, dir):
    the GPU variant runs the HIP conv / attention kernels against the same
    fp32 CPU oracle."""
    m, d = ckpt_dir
    cfg, w, vocab = load_vits(str(d), request.param)
    return m, cfg, w, vocab, d


def _ids(vocab, texts):
    ids = [text_to_ids(t, 0, vocab) for t in texts]
    T = max(map(len, ids))
    arr = torch.zeros(len(ids), T, dtype=torch.int64)
    for b, i in enumerate(ids):
        arr[b, :len(i)] = torch.tensor(i)
    return arr, torch.tensor([len(i) for i in ids], dtype=torch.int32)


def _close(a, b, rtol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item()
    assert err <= rtol * max(scale, 1e-6), (err, scale)


def test_config_and_vocab(ckpt):
    _, cfg, w, vocab, _ = ckpt
    assert cfg.sdp and cfg.hidden == 32 and cfg.sample_rate == 16000
    assert cfg.upsample_kernels == (16, 16, 4, 4) and vocab == VOCAB
    assert w.sdp is not None and w.dp is None and len(w.sdp["flows"]) == 3
    assert text_to_ids("Hi!", 0, vocab) == [0, VOCAB["h"], 0, VOCAB["i"], 0, VOCAB["!"], 0]
    assert text_to_ids("h#i", 0, vocab) == [0, VOCAB["h"], 0, VOCAB["i"], 0]   # unknowns dropped


def _dev(w):
    return w.emb.device


def test_text_encoder_parity(ckpt):
    m, cfg, w, vocab, _ = ckpt
    ids, lens = _ids(vocab, ["turn on the kitchen lights", "hello there"])
    mask = (torch.arange(ids.shape[1])[None] < lens[:, None].long())
    with torch.no_grad():
        out = m.text_encoder(input_ids=ids, padding_mask=mask[..., None].float(),
                             attention_mask=mask.long())
        stats, x = VitsModel(w).encode_text(ids.to(_dev(w)), lens.to(_dev(w)))
        stats, x = stats.cpu(), x.cpu()
    C = cfg.inter_channels
    mk = mask[..., None]
    _close(x.float() * mk, out.last_hidden_state * mk, 0.05)
    _close(stats[..., :C].float() * mk, out.prior_means * mk, 0.05)
    _close(stats[..., C:].float() * mk, out.prior_log_variances * mk, 0.05)


def test_stochastic_duration_predictor_parity(ckpt):
    m, cfg, w, vocab, _ = ckpt
    ids, lens = _ids(vocab, ["what is the weather", "play music in the living room"])
    B, T = ids.shape
    mask = (torch.arange(T)[None] < lens[:, None].long())
    with torch.no_grad():
        h = m.text_encoder(input_ids=ids, padding_mask=mask[..., None].float(),
                           attention_mask=mask.long()).last_hidden_state
        torch.manual_seed(7)
        ref = m.duration_predictor(h.transpose(1, 2), mask[:, None].float(), reverse=True,
                                   noise_scale=0.8)[:, 0]
        torch.manual_seed(7)
        noise = torch.randn(B, 2, T) * 0.8
        dv = _dev(w)
        ours = VitsModel(w)._sdp.log_durations(h.to(dv), mask.to(dv), noise.to(dv)).cpu()
    torch.testing.assert_close(ours * mask, ref * mask, rtol=1e-4, atol=1e-4)
    # the spline actually moved the values (not an identity pass-through)
    assert (ref * mask).abs().max() > 0.05


def test_flow_and_vocoder_parity(ckpt):
    m, cfg, w, _, _ = ckpt
    torch.manual_seed(3)
    B, F, C = 2, 40, cfg.inter_channels
    flen = torch.tensor([40, 29], dtype=torch.int32)
    fmask = (torch.arange(F)[None] < flen[:, None].long())
    z = torch.randn(B, F, C) * fmask[..., None]
    model = VitsModel(w)
    hop = model.hop
    with torch.no_grad():
        lat = m.flow(z.transpose(1, 2), fmask[:, None].float(), None, reverse=True)
        ref = m.decoder(lat * fmask[:, None].float(), None)[:, 0]            # [B, F * hop]
        dv = _dev(w)
        zz = model.flow_reverse(z.to(torch.bfloat16).to(dv).contiguous(), flen.to(dv))
        _close(zz.float().cpu() * fmask[..., None], lat.transpose(1, 2) * fmask[..., None], 0.05)
        pcm = model.decode(zz, (flen * hop).to(torch.int32).to(dv)).float().cpu() / 32767.0
    for b in range(B):
        n = int(flen[b]) * hop
        a, r = pcm[b, :n], ref[b, :n]
        corr = torch.corrcoef(torch.stack([a, r]))[0, 1].item()
        rel = ((a - r).norm() / r.norm()).item()
        # bf16 through ~40 convs, then a saturating tanh: RMS, not max, error
        assert corr > 0.995 and rel < 0.05, (corr, rel)


def test_engine_serves_checkpoint(ckpt):
    """The served path: the engine loads the directory itself; on the GPU the
    stochastic predictor (its noise draw included) runs inside the captured
    text-phase graph, replayed for a second batch of the same bucket."""
    from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
    _, cfg, w, _, d = ckpt
    dv = _dev(w)
    eng = VitsTTSEngine(None, dv, checkpoint=str(d), use_graphs=dv.type == "cuda")
    assert eng.cfg.sample_rate == 16000 and eng.vocab == VOCAB
    hop = eng.model.hop
    for texts in (["turn on the lights", "ok"], ["dim the hallway", "yes please"]):
        pcm = eng.synthesize_batch(texts)
        assert all(len(p) > 0 and len(p) % hop == 0 for p in pcm)
        assert np.abs(pcm[0].astype(np.int32)).max() > 0
    if dv.type == "cuda":
        assert eng.stats["graph_replays"] == 2 and eng.stats["graph_captures"] >= 2


def test_deterministic_predictor_checkpoint(tmp_path):
    m = _hf_model(sdp=False, seed=1)
    m.save_pretrained(str(tmp_path), safe_serialization=True)
    cfg, w, vocab = load_vits(str(tmp_path), "cpu")
    assert not cfg.sdp and w.sdp is None and vocab is None
    ids, lens = _ids({c: i for i, c in enumerate("_ abcdefghijklmnopqrstuvwxyz.,'?!-")},
                     ["good morning"])
    mask = (torch.arange(ids.shape[1])[None] < lens[:, None].long())
    with torch.no_grad():
        h = m.text_encoder(input_ids=ids, padding_mask=mask[..., None].float(),
                           attention_mask=mask.long()).last_hidden_state
        ref = m.duration_predictor(h.transpose(1, 2), mask[:, None].float())[:, 0]
        model = VitsModel(w)
        _, x = model.encode_text(ids, lens)
        dur = model.durations(x, lens)
    want = torch.ceil(torch.exp(ref) * mask)
    # bf16 hidden states: a ceil may land one frame either side
    assert (dur.float() - want).abs().max() <= 1


# ------------------------------------------------------------ multi-speaker
@pytest.fixture(scope="module")
def ckpt_ms_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("vits_ms")
    m = _hf_model(seed=2, speakers=3)
    m.save_pretrained(str(d), safe_serialization=True)
    (d / "vocab.json").write_text(json.dumps(VOCAB))
    return m, d


@pytest.fixture(scope="module", params=DEVICES)
def ckpt_ms(request, ckpt_ms_dir):
    m, d = ckpt_ms_dir
    cfg, w, vocab = load_vits(str(d), request.param)
    return m, cfg, w, vocab, d


def test_multi_speaker_duration_parity(ckpt_ms):
    """Speaker-conditioned stochastic duration predictor vs the oracle."""
    m, cfg, w, vocab, _ = ckpt_ms
    assert cfg.n_speakers == 3 and cfg.speaker_dim == 16 and w.spk is not None
    ids, lens = _ids(vocab, ["what is the weather", "lights off"])
    B, T = ids.shape
    mask = (torch.arange(T)[None] < lens[:, None].long())
    spk = torch.tensor([2, 1])
    with torch.no_grad():
        h = m.text_encoder(input_ids=ids, padding_mask=mask[..., None].float(),
                           attention_mask=mask.long()).last_hidden_state
        g = m.embed_speaker(spk).unsqueeze(-1)
        torch.manual_seed(11)
        ref = m.duration_predictor(h.transpose(1, 2), mask[:, None].float(), global_conditioning=g,
                                   reverse=True, noise_scale=0.8)[:, 0]
        torch.manual_seed(11)
        noise = torch.randn(B, 2, T) * 0.8
        dv = _dev(w)
        model = VitsModel(w)
        gv = model.speaker_vec(spk.to(dv))
        ours = model._sdp.log_durations(h.to(dv), mask.to(dv), noise.to(dv),
                                        model._proj("dp", gv)).cpu()
        # the speaker moves the durations (a conditioning actually applied)
        torch.manual_seed(11)
        ref0 = m.duration_predictor(h.transpose(1, 2), mask[:, None].float(),
                                    global_conditioning=m.embed_speaker(torch.tensor([0, 0])).unsqueeze(-1),
                                    reverse=True, noise_scale=0.8)[:, 0]
    torch.testing.assert_close(ours * mask, ref * mask, rtol=1e-4, atol=1e-4)
    assert ((ref - ref0) * mask).abs().max() > 1e-3


def test_multi_speaker_flow_and_vocoder_parity(ckpt_ms):
    m, cfg, w, _, _ = ckpt_ms
    torch.manual_seed(5)
    B, F, C = 2, 36, cfg.inter_channels
    flen = torch.tensor([36, 36], dtype=torch.int32)
    fmask = torch.ones(B, F, dtype=torch.bool)
    z = torch.randn(B, F, C)
    spk = torch.tensor([0, 2])
    model = VitsModel(w)
    hop = model.hop
    dv = _dev(w)
    with torch.no_grad():
        g = m.embed_speaker(spk).unsqueeze(-1)
        lat = m.flow(z.transpose(1, 2), fmask[:, None].float(), g, reverse=True)
        ref = m.decoder(lat, g)[:, 0]
        gv = model.speaker_vec(spk.to(dv))
        zz = model.flow_reverse(z.to(torch.bfloat16).to(dv).contiguous(), flen.to(dv), gv)
        _close(zz.float().cpu(), lat.transpose(1, 2), 0.05)
        pcm = model.decode(zz, (flen * hop).to(torch.int32).to(dv), gv).float().cpu() / 32767.0
    for b in range(B):
        a, r = pcm[b], ref[b]
        corr = torch.corrcoef(torch.stack([a, r]))[0, 1].item()
        rel = ((a - r).norm() / r.norm()).item()
        assert corr > 0.995 and rel < 0.05, (b, corr, rel)


def test_multi_speaker_engine_voices(ckpt_ms):
    """Voices map to speakers; one batch mixes speakers (graph replay on the
    GPU), and a speaker's audio does not depend on its batch neighbours'."""
    from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
    _, cfg, w, _, d = ckpt_ms
    dv = _dev(w)
    eng = VitsTTSEngine(None, dv, checkpoint=str(d), use_graphs=dv.type == "cuda")
    name = eng.cfg.name
    assert eng.voices() == [f"{name}:0", f"{name}:1", f"{name}:2"]
    assert eng.speaker_id(f"{name}:2") == 2 and eng.speaker_id("1") == 1
    assert eng.speaker_id("af_bella") == 0 and eng.speaker_id("") == 0 and eng.speaker_id("9") == 0
    eng.model.noise_scale = 0.0            # deterministic: compare rows across batches
    eng.model.noise_scale_duration = 0.0
    mixed = eng.synthesize_batch(["turn on the lights", "turn on the lights"], speakers=[0, 2])
    alone = eng.synthesize_batch(["turn on the lights"], speakers=[2])
    assert len(mixed[1]) == len(alone[0])
    # the batch's frame padding differs (its longest row), and the vocoder's
    # receptive field reaches a few frames into it: compare away from the end
    k = int(0.8 * len(alone[0]))
    a, b = mixed[1][:k].astype(np.float64), alone[0][:k].astype(np.float64)
    assert np.corrcoef(a, b)[0, 1] > 0.999
    assert not np.array_equal(mixed[0], mixed[1])      # different speakers, different audio


# ------------------------------------------------------------- full size
@pytest.mark.gpu
def test_mms_size_checkpoint_gpu(tmp_path):
    """A checkpoint of the public MMS-TTS shape (transformers' VitsConfig
    defaults: hidden 192, 6 layers, 4 flows, 512-channel HiFi-GAN at 16 kHz,
    stochastic duration predictor), random weights: the loader, the duration
    predictor and the flow + vocoder through the HIP kernels against the fp32
    oracle, and the served engine's graph replays."""
    from transformers import VitsConfig, VitsModel as HFVits
    from loqa_hub_amd.engine.tts_engine import VitsTTSEngine
    torch.manual_seed(0)
    m = HFVits(VitsConfig()).eval()
    m.save_pretrained(str(tmp_path), safe_serialization=True)
    vocab = {c: i for i, c in enumerate("_ '-abcdefghijklmnopqrstuvwxyz0123456")}
    (tmp_path / "vocab.json").write_text(json.dumps(vocab))
    dev = torch.device("cuda", 0)
    cfg, w, voc = load_vits(str(tmp_path), dev)
    assert cfg.hidden == 192 and cfg.sample_rate == 16000 and cfg.sdp
    model = VitsModel(w)
    ids, lens = _ids(voc, ["turn on the kitchen lights please", "good night"])
    B, T = ids.shape
    mask = (torch.arange(T)[None] < lens[:, None].long())
    with torch.no_grad():
        h = m.text_encoder(input_ids=ids, padding_mask=mask[..., None].float(),
                           attention_mask=mask.long()).last_hidden_state
        torch.manual_seed(3)
        ref = m.duration_predictor(h.transpose(1, 2), mask[:, None].float(), reverse=True,
                                   noise_scale=0.8)[:, 0]
        torch.manual_seed(3)
        noise = torch.randn(B, 2, T) * 0.8
        ours = model._sdp.log_durations(h.to(dev), mask.to(dev), noise.to(dev)).cpu()
        torch.testing.assert_close(ours * mask, ref * mask, rtol=1e-3, atol=1e-3)
        F = 48
        flen = torch.tensor([F, F], dtype=torch.int32)
        z = torch.randn(B, F, cfg.inter_channels)
        lat = m.flow(z.transpose(1, 2), torch.ones(B, 1, F), None, reverse=True)
        wav = m.decoder(lat, None)[:, 0]
        zz = model.flow_reverse(z.to(torch.bfloat16).to(dev).contiguous(), flen.to(dev))
        pcm = model.decode(zz, (flen * model.hop).to(torch.int32).to(dev)).float().cpu() / 32767.0
    for b in range(B):
        corr = torch.corrcoef(torch.stack([pcm[b], wav[b]]))[0, 1].item()
        rel = ((pcm[b] - wav[b]).norm() / wav[b].norm()).item()
        assert corr > 0.99 and rel < 0.1, (b, corr, rel)
    eng = VitsTTSEngine(None, dev, checkpoint=str(tmp_path))
    for texts in (["turn on the lights", "done"], ["play some music", "ok then"]):
        out = eng.synthesize_batch(texts)
        assert all(len(p) > 0 and len(p) % model.hop == 0 for p in out)
    assert eng.stats["graph_replays"] == 2
