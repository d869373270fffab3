"""Model configurations for the on-GPU STT -> intent -> TTS pipeline.

Dimensions are public model-card facts. Weights are always
seeded random-init (no network, no checkpoints); ``loqa_hub_amd.engine.weights``
can also map safetensors files when they exist locally.
"""
from __future__ import annotations

from dataclasses import dataclass, replace


@dataclass(frozen=True)
class LlamaConfig:
    name: str
    d_model: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    ffn_dim: int
    vocab_size: int
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    tie_embeddings: bool = False
    max_positions: int = 8192
    # Llama-3.1-style RoPE frequency scaling: (factor, low_freq_factor,
    # high_freq_factor, original_max_positions), or None
    rope_scaling: tuple | None = None

    @property
    def qkv_dim(self) -> int:
        return (self.n_heads + 2 * self.n_kv_heads) * self.head_dim

    def n_params(self) -> int:
        d, f = self.d_model, self.ffn_dim
        per = d * self.qkv_dim + self.n_heads * self.head_dim * d + 3 * d * f + 2 * d
        emb = self.vocab_size * d * (1 if self.tie_embeddings else 2)
        return self.n_layers * per + emb + d


LLAMA_CONFIGS = {
    "tinyllama": LlamaConfig("tinyllama-1.1b", 2048, 22, 32, 4, 64, 5632, 32000, rope_theta=10000.0),
    "llama3.2-1b": LlamaConfig("llama-3.2-1b", 2048, 16, 32, 8, 64, 8192, 128256, tie_embeddings=True,
                               rope_scaling=(32.0, 1.0, 4.0, 8192)),
    "llama3.2-3b": LlamaConfig("llama-3.2-3b", 3072, 28, 24, 8, 128, 8192, 128256, tie_embeddings=True,
                               rope_scaling=(32.0, 1.0, 4.0, 8192)),
    "llama3-8b": LlamaConfig("llama-3-8b", 4096, 32, 32, 8, 128, 14336, 128256),
    "llama3-70b": LlamaConfig("llama-3-70b", 8192, 80, 64, 8, 128, 28672, 128256),
    # small shapes for CPU tests / smoke
    "test-tiny": LlamaConfig("test-tiny", 256, 2, 4, 2, 64, 512, 4096, tie_embeddings=True,
                             max_positions=2048),
}


@dataclass(frozen=True)
class WhisperConfig:
    name: str
    n_mels: int
    d_model: int
    enc_layers: int
    dec_layers: int
    n_heads: int
    vocab_size: int
    n_audio_ctx: int = 1500
    n_text_ctx: int = 448

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    @property
    def ffn_dim(self) -> int:
        return 4 * self.d_model


WHISPER_CONFIGS = {
    "whisper-tiny": WhisperConfig("whisper-tiny", 80, 384, 4, 4, 6, 51865),
    "whisper-base": WhisperConfig("whisper-base", 80, 512, 6, 6, 8, 51865),
    "whisper-small": WhisperConfig("whisper-small", 80, 768, 12, 12, 12, 51865),
    "whisper-large-v3": WhisperConfig("whisper-large-v3", 128, 1280, 32, 32, 20, 51866),
    "test-whisper": WhisperConfig("test-whisper", 80, 128, 2, 2, 2, 4096, n_audio_ctx=1500),
}


@dataclass(frozen=True)
class VitsConfig:
    """VITS (text encoder + stochastic duration + flow + HiFi-GAN) at the public
    'vits-ljs' sizes; sample rate 22.05 kHz, hop 256."""
    name: str
    n_symbols: int = 178
    hidden: int = 192
    filter_channels: int = 768
    n_heads: int = 2
    enc_layers: int = 6
    kernel_size: int = 3
    flow_layers: int = 4
    wn_layers: int = 4
    inter_channels: int = 192
    upsample_rates: tuple = (8, 8, 2, 2)
    upsample_initial: int = 512
    resblock_kernels: tuple = (3, 7, 11)
    resblock_dilations: tuple = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    sample_rate: int = 22050
    window: int = 4
    # checkpoints (public VITS / MMS-TTS): the stochastic duration predictor
    # and the sampling constants of the published models
    sdp: bool = False
    sdp_filter: int = 192
    sdp_flows: int = 4
    sdp_bins: int = 10
    sdp_tail: float = 5.0
    sdp_kernel: int = 3
    noise_scale: float = 0.667
    noise_scale_duration: float = 0.8
    speaking_rate: float = 1.0
    upsample_kernels: tuple = ()          # () -> 2r for r > 2, else 4
    leaky_slope: float = 0.1
    # multi-speaker checkpoints (VCTK-style): a speaker embedding conditions
    # the duration predictor, every flow WaveNet layer and the vocoder input
    n_speakers: int = 1
    speaker_dim: int = 0


VITS_CONFIGS = {
    "vits-ljs": VitsConfig("vits-ljs"),
    "test-vits": VitsConfig("test-vits", hidden=64, filter_channels=128, enc_layers=2, flow_layers=2,
                            wn_layers=2, inter_channels=64, upsample_initial=256),
}


def llama_config(name: str, **over) -> LlamaConfig:
    c = LLAMA_CONFIGS[name]
    return replace(c, **over) if over else c


def whisper_config(name: str, **over) -> WhisperConfig:
    c = WHISPER_CONFIGS[name]
    return replace(c, **over) if over else c


def vits_config(name: str, **over) -> VitsConfig:
    c = VITS_CONFIGS[name]
    return replace(c, **over) if over else c


# --------------------------------------------------------------------------
# A checkpoint's own config.json (Hugging Face naming): any Llama-family or
# Whisper checkpoint, not only the named sizes above
def llama_config_from_hf(d: dict, name: str = "checkpoint") -> LlamaConfig:
    H = int(d["num_attention_heads"])
    D = int(d.get("head_dim") or int(d["hidden_size"]) // H)
    rs = d.get("rope_scaling") or None
    scaling = None
    if rs:
        kind = rs.get("rope_type", rs.get("type"))
        if kind != "llama3":
            raise ValueError(f"{name}: rope_scaling type {kind!r} is not supported")
        scaling = (float(rs["factor"]), float(rs.get("low_freq_factor", 1.0)),
                   float(rs.get("high_freq_factor", 4.0)),
                   int(rs.get("original_max_position_embeddings", 8192)))
    return LlamaConfig(name, int(d["hidden_size"]), int(d["num_hidden_layers"]), H,
                       int(d.get("num_key_value_heads", H)), D, int(d["intermediate_size"]),
                       int(d["vocab_size"]), rope_theta=float(d.get("rope_theta", 10000.0)),
                       norm_eps=float(d.get("rms_norm_eps", 1e-5)),
                       tie_embeddings=bool(d.get("tie_word_embeddings", False)),
                       max_positions=min(int(d.get("max_position_embeddings", 8192)), 8192),
                       rope_scaling=scaling)


def whisper_config_from_hf(d: dict, name: str = "checkpoint") -> WhisperConfig:
    c = WhisperConfig(name, int(d["num_mel_bins"]), int(d["d_model"]), int(d["encoder_layers"]),
                      int(d["decoder_layers"]), int(d["encoder_attention_heads"]),
                      int(d["vocab_size"]), n_audio_ctx=int(d.get("max_source_positions", 1500)),
                      n_text_ctx=int(d.get("max_target_positions", 448)))
    if int(d.get("encoder_ffn_dim", c.ffn_dim)) != c.ffn_dim:
        raise ValueError(f"{name}: encoder_ffn_dim {d['encoder_ffn_dim']} != 4 * d_model")
    return c


def vits_config_from_hf(d: dict, name: str = "checkpoint") -> VitsConfig:
    """A Hugging Face VITS / MMS-TTS config.json (``VitsConfig`` field names)."""
    return VitsConfig(
        name, n_symbols=d["vocab_size"], hidden=d["hidden_size"], filter_channels=d["ffn_dim"],
        n_heads=d["num_attention_heads"], enc_layers=d["num_hidden_layers"],
        kernel_size=d.get("ffn_kernel_size", 3), flow_layers=d.get("prior_encoder_num_flows", 4),
        wn_layers=d.get("prior_encoder_num_wavenet_layers", 4), inter_channels=d["flow_size"],
        upsample_rates=tuple(d["upsample_rates"]), upsample_initial=d["upsample_initial_channel"],
        resblock_kernels=tuple(d["resblock_kernel_sizes"]),
        resblock_dilations=tuple(tuple(x) for x in d["resblock_dilation_sizes"]),
        sample_rate=d.get("sampling_rate", 16000), window=d.get("window_size", 4),
        sdp=bool(d.get("use_stochastic_duration_prediction", True)),
        sdp_filter=d.get("duration_predictor_filter_channels", 256),
        sdp_flows=d.get("duration_predictor_num_flows", 4),
        sdp_bins=d.get("duration_predictor_flow_bins", 10),
        sdp_tail=float(d.get("duration_predictor_tail_bound", 5.0)),
        sdp_kernel=d.get("duration_predictor_kernel_size", 3),
        noise_scale=float(d.get("noise_scale", 0.667)),
        noise_scale_duration=float(d.get("noise_scale_duration", 0.8)),
        speaking_rate=float(d.get("speaking_rate", 1.0)),
        upsample_kernels=tuple(d.get("upsample_kernel_sizes", ())),
        leaky_slope=float(d.get("leaky_relu_slope", 0.1)),
        n_speakers=int(d.get("num_speakers", 1)),
        speaker_dim=int(d.get("speaker_embedding_size", 0)) if d.get("num_speakers", 1) > 1 else 0)


def checkpoint_config(path: str):
    """The config.json dict in (or beside) a checkpoint, or None."""
    import json
    import os
    if not path:
        return None
    d = path if os.path.isdir(path) else os.path.dirname(os.path.abspath(path))
    f = os.path.join(d, "config.json")
    if not os.path.isfile(f):
        return None
    with open(f, encoding="utf-8") as fh:
        return json.load(fh)
