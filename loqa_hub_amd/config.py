"""Typed configuration loaded from the environment.

Same variable names and defaults as the reference (``internal/config/config.go``:
Load :113-174, validate :177-211; helpers :214-255 silently fall back to the
default on a parse error). Differences, all additive:

* ONE config object: ``OLLAMA_URL``/``OLLAMA_MODEL``, ``NATS_URL``, ``DB_PATH``
  and ``LOG_*`` are read here instead of ad hoc in each component;
* documented aliases are accepted (``LOQA_HUB_PORT``, ``DB_PATH``,
  ``STREAMING_VISUAL_FEEDBACK_DELAY``, ``ARBITRATION_WINDOW_DURATION``,
  ``MAX_CONCURRENT_RELAYS``) - the reference's own names win when both are set;
* GPU keys for the on-device pipeline (``HUB_*``) and arbitration scope.

Durations use Go syntax (``300ms``, ``1h30m``, ``2s``).
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field

_DUR_RE = re.compile(r"([0-9]*\.?[0-9]+)(ns|us|µs|ms|s|m|h)")
_UNIT = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_go_duration(s: str) -> float:
    """Go time.ParseDuration subset -> seconds. Raises ValueError."""
    s = s.strip()
    if s in ("0", "+0", "-0"):
        return 0.0
    sign = 1.0
    if s[:1] in "+-":
        sign = -1.0 if s[0] == "-" else 1.0
        s = s[1:]
    if not s:
        raise ValueError("empty duration")
    pos, total = 0, 0.0
    for m in _DUR_RE.finditer(s):
        if m.start() != pos:
            raise ValueError(f"invalid duration {s!r}")
        total += float(m.group(1)) * _UNIT[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise ValueError(f"invalid duration {s!r}")
    return sign * total


def format_go_duration(sec: float) -> str:
    if sec == 0:
        return "0s"
    if abs(sec) < 1:
        ms = sec * 1e3
        return f"{ms:g}ms"
    h, rem = divmod(sec, 3600)
    m, s = divmod(rem, 60)
    out = ""
    if h:
        out += f"{int(h)}h"
    if h or m:
        out += f"{int(m)}m"
    return out + f"{s:g}s"


def _get(env, *keys):
    for k in keys:
        v = env.get(k, "")
        if v != "":
            return v
    return ""


def env_str(env, default: str, *keys) -> str:
    v = _get(env, *keys)
    return v if v != "" else default


_INT_RE = re.compile(r"^[+-]?[0-9]+$")


def env_int(env, default: int, *keys) -> int:
    v = _get(env, *keys)
    return int(v, 10) if _INT_RE.match(v) else default


def env_float(env, default: float, *keys) -> float:
    v = _get(env, *keys)
    try:
        return float(v) if v != "" else default
    except ValueError:
        return default


_TRUE = {"1", "t", "T", "true", "TRUE", "True"}
_FALSE = {"0", "f", "F", "false", "FALSE", "False"}


def env_bool(env, default: bool, *keys) -> bool:
    v = _get(env, *keys)
    if v in _TRUE:
        return True
    if v in _FALSE:
        return False
    return default


def env_duration(env, default: float, *keys) -> float:
    v = _get(env, *keys)
    try:
        return parse_go_duration(v) if v != "" else default
    except ValueError:
        return default


@dataclass
class ServerConfig:
    host: str = "0.0.0.0"
    port: int = 8080
    grpc_port: int = 50051
    db_path: str = "./data/loqa-hub.db"
    read_timeout: float = 30.0
    write_timeout: float = 30.0


@dataclass
class STTConfig:
    url: str = "http://stt:8000"
    language: str = "en"
    temperature: float = 0.0
    max_tokens: int = 224


@dataclass
class TTSConfig:
    url: str = "http://localhost:8880/v1"
    voice: str = "af_bella"
    speed: float = 1.0
    response_format: str = "wav"
    normalize: bool = True
    max_concurrent: int = 10
    timeout: float = 10.0
    fallback_enabled: bool = True


@dataclass
class StreamingConfig:
    enabled: bool = False
    ollama_url: str = "http://ollama:11434"
    model: str = "llama3.2:3b"
    max_buffer_time: float = 2.0
    max_tokens_per_phrase: int = 50
    audio_concurrency: int = 3
    visual_feedback_delay: float = 0.050
    interrupt_timeout: float = 0.500
    fallback_enabled: bool = True
    metrics_enabled: bool = True


@dataclass
class LoggingConfig:
    level: str = "info"
    format: str = "json"


@dataclass
class NATSConfig:
    url: str = "nats://localhost:4222"
    subject: str = "loqa.commands"
    max_reconnect: int = 10
    reconnect_wait: float = 2.0


@dataclass
class PrivacyConfig:
    data_retention: float = 30 * 24 * 3600.0
    zero_persistence: bool = False
    auto_cleanup_enabled: bool = True
    cleanup_interval: float = 24 * 3600.0


@dataclass
class OllamaConfig:
    """The service-level parser endpoint (reference: env-only in
    audio_service.go:204-212; default http://localhost:11434)."""
    url: str = "http://localhost:11434"
    model: str = "llama3.2:3b"


@dataclass
class GPUConfig:
    """On-device pipeline (SURVEY §5.6 'New')."""
    num_gpus: int = 0                 # 0 = all visible
    dp: int = 0                       # 0 = num_gpus
    tp: int = 1
    stt_model: str = "whisper-base"
    llm_model: str = "tinyllama"
    tts_model: str = "vits-ljs"
    dtype: str = "bf16"
    max_batch: int = 64
    kv_block: int = 16
    max_seq_len: int = 1024
    llm_backend: str = "gpu"          # gpu | ollama
    stt_backend: str = "gpu"          # gpu | http
    tts_backend: str = "gpu"          # gpu | http | none
    use_graphs: bool = True
    seed: int = 0
    tp_fallback_model: str = "llama3-8b"   # a failed TP group degrades to this ("none": off)
    # the fallback's weights (+ tokenizer in / beside it); required when
    # llm_checkpoint is set (no silent swap to a random-init model)
    tp_fallback_checkpoint: str = ""
    stt_checkpoint: str = ""          # safetensors file/dir (HF naming); "" = seeded random init
    llm_checkpoint: str = ""
    tts_checkpoint: str = ""          # HF VITS / MMS-TTS dir; "" = the random-init HUB_TTS_MODEL
    # what a TTS_FORMAT the GPU voice cannot encode (mp3, opus, aac, flac) gets:
    # "wav" = WAV, labelled wav, logged + counted; "error" = the synthesis fails
    tts_format_policy: str = "wav"
    # tokenizer.json of a checkpoint ("": the one in / beside the checkpoint;
    # no checkpoint: the synthetic tokenizer of the random-init weights)
    stt_tokenizer: str = ""
    llm_tokenizer: str = ""

    def llm_config(self):
        """The intent model's shape: the checkpoint's own config.json when it
        has one (any Llama-family checkpoint), else the named ``HUB_LLM_MODEL``."""
        from .models.configs import checkpoint_config, llama_config, llama_config_from_hf
        d = checkpoint_config(self.llm_checkpoint)
        return llama_config_from_hf(d, self.llm_model) if d else llama_config(self.llm_model)

    def tp_fallback_config(self):
        """Shape of the TP failover engine: its checkpoint's config.json, else
        ``HUB_TP_FALLBACK_MODEL``."""
        from .models.configs import checkpoint_config, llama_config, llama_config_from_hf
        d = checkpoint_config(self.tp_fallback_checkpoint)
        return llama_config_from_hf(d, self.tp_fallback_model) if d else \
            llama_config(self.tp_fallback_model)

    def stt_config(self):
        """As ``llm_config`` for the Whisper checkpoint / ``HUB_STT_MODEL``."""
        from .models.configs import checkpoint_config, whisper_config, whisper_config_from_hf
        d = checkpoint_config(self.stt_checkpoint)
        return whisper_config_from_hf(d, self.stt_model) if d else whisper_config(self.stt_model)

    def tokenizer(self, which: str, vocab_size: int):
        """The tokenizer for ``which`` ("stt" / "llm"): an explicit
        ``HUB_*_TOKENIZER``, else the checkpoint's own file, else None."""
        from .engine.tokenizer import find_tokenizer, load_tokenizer
        explicit = getattr(self, f"{which}_tokenizer")
        if explicit:
            return load_tokenizer(explicit, vocab_size)
        ckpt = getattr(self, f"{which}_checkpoint")
        return load_tokenizer(ckpt, vocab_size) if find_tokenizer(ckpt) else None


@dataclass
class ArbitrationConfig:
    window: float = 0.300
    scope: str = "global"             # global | per_relay_group
    max_concurrent_relays: int = 0    # 0 = unlimited
    end_of_speech_wait: float = 5.0
    bridge_timeout: float = 2.0
    confirmation_enabled: bool = False
    relay_groups: dict = field(default_factory=dict)  # relay id -> room/group
    # per_relay_group scope: a relay whose group (static ARBITRATION_RELAY_GROUPS
    # map) has no other member cannot collide, so it wins at once instead of
    # waiting out the window ("Single relay: No additional latency (bypass
    # arbitration)", reference docs/COLLISION_DETECTION.md:203; the reference's
    # code always waits, audio_service.go:443,494-502, hence opt-in)
    single_relay_bypass: bool = False


@dataclass
class Config:
    server: ServerConfig = field(default_factory=ServerConfig)
    stt: STTConfig = field(default_factory=STTConfig)
    tts: TTSConfig = field(default_factory=TTSConfig)
    streaming: StreamingConfig = field(default_factory=StreamingConfig)
    logging: LoggingConfig = field(default_factory=LoggingConfig)
    nats: NATSConfig = field(default_factory=NATSConfig)
    privacy: PrivacyConfig = field(default_factory=PrivacyConfig)
    ollama: OllamaConfig = field(default_factory=OllamaConfig)
    gpu: GPUConfig = field(default_factory=GPUConfig)
    arbitration: ArbitrationConfig = field(default_factory=ArbitrationConfig)

    def validate(self) -> None:
        if self.server.port <= 0 or self.server.port > 65535:
            raise ConfigError(f"invalid server port: {self.server.port}")
        if self.server.grpc_port <= 0 or self.server.grpc_port > 65535:
            raise ConfigError(f"invalid gRPC port: {self.server.grpc_port}")
        if self.stt.url == "":
            raise ConfigError("STT URL must be provided")
        if self.tts.url == "":
            raise ConfigError("TTS URL must be provided")
        if self.tts.max_concurrent <= 0:
            raise ConfigError(f"TTS max concurrent must be positive: {self.tts.max_concurrent}")
        if self.tts.speed <= 0:
            raise ConfigError(f"TTS speed must be positive: {self.tts.speed:f}")
        if self.privacy.data_retention < 0:
            raise ConfigError("data retention duration cannot be negative: "
                              f"{format_go_duration(self.privacy.data_retention)}")
        if self.privacy.cleanup_interval <= 0:
            raise ConfigError("cleanup interval must be positive: "
                              f"{format_go_duration(self.privacy.cleanup_interval)}")
        if self.arbitration.scope not in ("global", "per_relay_group"):
            raise ConfigError(f"invalid ARBITRATION_SCOPE: {self.arbitration.scope}")
        if self.gpu.tp < 1:
            raise ConfigError(f"HUB_TP must be >= 1: {self.gpu.tp}")


def parse_relay_groups(s: str) -> dict:
    """"relay-1=kitchen,relay-2=kitchen" -> {relay id: group}."""
    out = {}
    for part in filter(None, (p.strip() for p in s.split(","))):
        k, sep, v = part.partition("=")
        if sep and k.strip() and v.strip():
            out[k.strip()] = v.strip()
    return out


class ConfigError(ValueError):
    pass


def load(env=None) -> Config:
    """Build the configuration from ``env`` (default ``os.environ``) and
    validate it; raises ``ConfigError`` ("invalid configuration: ...")."""
    e = os.environ if env is None else env
    c = Config(
        server=ServerConfig(
            host=env_str(e, "0.0.0.0", "LOQA_HOST"),
            port=env_int(e, 8080, "LOQA_PORT", "LOQA_HUB_PORT"),
            grpc_port=env_int(e, 50051, "LOQA_GRPC_PORT"),
            db_path=env_str(e, "./data/loqa-hub.db", "LOQA_DB_PATH", "DB_PATH"),
            read_timeout=env_duration(e, 30.0, "LOQA_READ_TIMEOUT"),
            write_timeout=env_duration(e, 30.0, "LOQA_WRITE_TIMEOUT"),
        ),
        stt=STTConfig(
            url=env_str(e, "http://stt:8000", "STT_URL"),
            language=env_str(e, "en", "STT_LANGUAGE"),
            temperature=env_float(e, 0.0, "STT_TEMPERATURE"),
            max_tokens=env_int(e, 224, "STT_MAX_TOKENS"),
        ),
        tts=TTSConfig(
            url=env_str(e, "http://localhost:8880/v1", "TTS_URL"),
            voice=env_str(e, "af_bella", "TTS_VOICE"),
            speed=env_float(e, 1.0, "TTS_SPEED"),
            response_format=env_str(e, "wav", "TTS_FORMAT"),
            normalize=env_bool(e, True, "TTS_NORMALIZE"),
            max_concurrent=env_int(e, 10, "TTS_MAX_CONCURRENT"),
            timeout=env_duration(e, 10.0, "TTS_TIMEOUT"),
            fallback_enabled=env_bool(e, True, "TTS_FALLBACK_ENABLED"),
        ),
        streaming=StreamingConfig(
            enabled=env_bool(e, False, "STREAMING_ENABLED"),
            ollama_url=env_str(e, "http://ollama:11434", "OLLAMA_URL", "STREAMING_OLLAMA_URL"),
            model=env_str(e, "llama3.2:3b", "STREAMING_MODEL"),
            max_buffer_time=env_duration(e, 2.0, "STREAMING_MAX_BUFFER_TIME"),
            max_tokens_per_phrase=env_int(e, 50, "STREAMING_MAX_TOKENS_PER_PHRASE"),
            audio_concurrency=env_int(e, 3, "STREAMING_AUDIO_CONCURRENCY"),
            visual_feedback_delay=env_duration(e, 0.050, "STREAMING_VISUAL_DELAY",
                                               "STREAMING_VISUAL_FEEDBACK_DELAY"),
            interrupt_timeout=env_duration(e, 0.500, "STREAMING_INTERRUPT_TIMEOUT"),
            fallback_enabled=env_bool(e, True, "STREAMING_FALLBACK_ENABLED"),
            metrics_enabled=env_bool(e, True, "STREAMING_METRICS_ENABLED"),
        ),
        logging=LoggingConfig(
            level=env_str(e, "info", "LOG_LEVEL"),
            format=env_str(e, "json", "LOG_FORMAT"),
        ),
        nats=NATSConfig(
            url=env_str(e, "nats://localhost:4222", "NATS_URL"),
            subject=env_str(e, "loqa.commands", "NATS_SUBJECT"),
            max_reconnect=env_int(e, 10, "NATS_MAX_RECONNECT"),
            reconnect_wait=env_duration(e, 2.0, "NATS_RECONNECT_WAIT"),
        ),
        privacy=PrivacyConfig(
            data_retention=env_duration(e, 30 * 24 * 3600.0, "LOQA_DATA_RETENTION"),
            zero_persistence=env_bool(e, False, "LOQA_ZERO_PERSISTENCE"),
            auto_cleanup_enabled=env_bool(e, True, "LOQA_AUTO_CLEANUP"),
            cleanup_interval=env_duration(e, 24 * 3600.0, "LOQA_CLEANUP_INTERVAL"),
        ),
        ollama=OllamaConfig(
            url=env_str(e, "http://localhost:11434", "OLLAMA_URL"),
            model=env_str(e, "llama3.2:3b", "OLLAMA_MODEL"),
        ),
        gpu=GPUConfig(
            num_gpus=env_int(e, 0, "HUB_NUM_GPUS"),
            dp=env_int(e, 0, "HUB_DP"),
            tp=env_int(e, 1, "HUB_TP"),
            stt_model=env_str(e, "whisper-base", "HUB_STT_MODEL"),
            llm_model=env_str(e, "tinyllama", "HUB_LLM_MODEL"),
            tts_model=env_str(e, "vits-ljs", "HUB_TTS_MODEL"),
            dtype=env_str(e, "bf16", "HUB_DTYPE"),
            max_batch=env_int(e, 64, "HUB_MAX_BATCH"),
            kv_block=env_int(e, 16, "HUB_KV_BLOCK"),
            max_seq_len=env_int(e, 1024, "HUB_MAX_SEQ_LEN"),
            llm_backend=env_str(e, "gpu", "HUB_LLM_BACKEND"),
            stt_backend=env_str(e, "gpu", "HUB_STT_BACKEND"),
            tts_backend=env_str(e, "gpu", "HUB_TTS_BACKEND"),
            use_graphs=env_bool(e, True, "HUB_USE_GRAPHS"),
            seed=env_int(e, 0, "HUB_SEED"),
            tp_fallback_model=env_str(e, "llama3-8b", "HUB_TP_FALLBACK_MODEL"),
            tp_fallback_checkpoint=env_str(e, "", "HUB_TP_FALLBACK_CHECKPOINT"),
            stt_checkpoint=env_str(e, "", "HUB_STT_CHECKPOINT"),
            llm_checkpoint=env_str(e, "", "HUB_LLM_CHECKPOINT"),
            tts_checkpoint=env_str(e, "", "HUB_TTS_CHECKPOINT"),
            tts_format_policy=env_str(e, "wav", "HUB_TTS_FORMAT_POLICY"),
            stt_tokenizer=env_str(e, "", "HUB_STT_TOKENIZER"),
            llm_tokenizer=env_str(e, "", "HUB_LLM_TOKENIZER"),
        ),
        arbitration=ArbitrationConfig(
            window=env_duration(e, 0.300, "ARBITRATION_WINDOW_DURATION"),
            scope=env_str(e, "global", "ARBITRATION_SCOPE"),
            max_concurrent_relays=env_int(e, 0, "MAX_CONCURRENT_RELAYS"),
            end_of_speech_wait=env_duration(e, 5.0, "ARBITRATION_EOS_WAIT"),
            bridge_timeout=env_duration(e, 2.0, "BRIDGE_TIMEOUT"),
            confirmation_enabled=env_bool(e, False, "CONFIRMATION_ENABLED"),
            relay_groups=parse_relay_groups(env_str(e, "", "ARBITRATION_RELAY_GROUPS")),
            single_relay_bypass=env_bool(e, False, "ARBITRATION_SINGLE_RELAY_BYPASS"),
        ),
    )
    try:
        c.validate()
    except ConfigError as err:
        raise ConfigError(f"invalid configuration: {err}") from err
    return c
