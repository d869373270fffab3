"""On-GPU text-to-speech engine (VITS) behind the ``TextToSpeech`` contract
(``internal/llm/tts.go``), replacing the external OpenAI-compatible TTS.

Concurrent ``synthesize`` calls (the progressive pipeline's phrase workers of
every live session) are micro-batched into one padded VITS forward; each
result is returned as a WAV (PCM16 mono, the voice's sample rate) or raw PCM.
``speed`` maps to the duration length scale (1 / speed), as in the reference's
request body.

``response_format`` (``openai_tts_client.go:39-46``; the status manager asks
for ``mp3``, ``status_manager.go:441-462``): ``wav`` and ``pcm`` are produced
as asked. No compressed-audio encoder ships in this image, so ``mp3``,
``opus``, ``aac`` and ``flac`` follow ``format_policy``: ``"wav"`` (default)
returns WAV, logs the downgrade once per format and counts it in
``stats["format_downgrades"]``; ``"error"`` raises
:class:`UnsupportedAudioFormat`. Either way ``TTSResult.format`` names the
container the bytes are really in, and the hub labels the audio with it.
"""
from __future__ import annotations

import asyncio
import io
import logging
import struct
import threading
import time

import numpy as np
import torch

from ..llm.tts import TTSOptions, TTSResult
from ..models.configs import VitsConfig
from ..models.vits import VitsGraphRunner, VitsModel, VitsWeights, text_to_ids
from ..utils.faults import faults

log = logging.getLogger("loqa.tts")

SUPPORTED_FORMATS = ("wav", "pcm")
_CONTENT_TYPES = {"wav": "audio/wav", "pcm": "audio/pcm"}


class UnsupportedAudioFormat(ValueError):
    """A response_format the on-GPU TTS cannot encode (format_policy "error")."""


def pcm16_to_wav(pcm: np.ndarray, sample_rate: int) -> bytes:
    data = np.ascontiguousarray(pcm, dtype="<i2").tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, sample_rate, sample_rate * 2, 2, 16)
    return hdr + b"data" + struct.pack("<I", len(data)) + data


class VitsTTSEngine:
    def __init__(self, cfg: VitsConfig | None, device, *, seed: int = 0, batch_window: float = 0.003,
                 max_batch: int = 32, use_graphs: bool = True, checkpoint: str | None = None,
                 format_policy: str = "wav"):
        """``checkpoint``: a Hugging Face VITS / MMS-TTS directory (config.json,
        safetensors, vocab.json; models/loader.py ``load_vits``) — its config
        and vocabulary replace ``cfg`` and the character table; None: the
        random-init voice of ``cfg``. ``format_policy``: what an unsupported
        response_format gets - "wav" (a logged, counted downgrade) or "error"."""
        if format_policy not in ("wav", "error"):
            raise ValueError(f"format_policy must be 'wav' or 'error', not {format_policy!r}")
        self.format_policy = format_policy
        self._downgrade_logged: set[str] = set()
        self.device = torch.device(device)
        self.vocab = None
        if checkpoint:
            from ..models.loader import load_vits
            cfg, weights, self.vocab = load_vits(checkpoint, self.device)
        else:
            weights = VitsWeights(cfg, self.device, seed=seed)
        self.cfg = cfg
        self.model = VitsModel(weights)
        # bucketed HIP-graph replay (models/vits.py VitsGraphRunner), built
        # lazily on the placed TTS stream
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self._runner: VitsGraphRunner | None = None
        self.batch_window = batch_window
        self.max_batch = max_batch
        self._pending: list[tuple[str, float, int, asyncio.Future]] = []
        self._flusher: asyncio.Task | None = None
        self._gpu_lock = threading.Lock()
        self._stream = None            # the placed TTS stream (utils/streams.py), created lazily
        self._seed = seed
        self.stats = {"batches": 0, "phrases": 0, "samples": 0, "gpu_s": 0.0, "launch_s": 0.0,
                      "format_downgrades": 0}

    # ---------------------------------------------------------------- batch
    # ---------------------------------------------------------------- voices
    def voices(self) -> list[str]:
        """Voice names: the model name (one speaker), else ``name:<id>`` per
        speaker of a multi-speaker checkpoint."""
        n = self.model.n_speakers
        return [self.cfg.name] if n == 1 else [f"{self.cfg.name}:{i}" for i in range(n)]

    def speaker_id(self, voice: str | None) -> int:
        """Speaker of a voice name (``name:<id>``, ``<id>`` or a listed name);
        anything else (the reference's default ``af_bella``, "") -> speaker 0."""
        n = self.model.n_speakers
        if n == 1 or not voice:
            return 0
        v = voice.rsplit(":", 1)[-1]
        if v.isdigit() and int(v) < n:
            return int(v)
        return 0

    def synthesize_batch(self, texts: list[str], speeds: list[float] | None = None,
                         speakers: list[int] | None = None) -> list[np.ndarray]:
        """Synchronous batched synthesis -> PCM16 arrays (``speakers``: speaker
        ids per text, multi-speaker voices)."""
        speeds = speeds or [1.0] * len(texts)
        ids = [text_to_ids(t, self.cfg.n_symbols, self.vocab) for t in texts]
        T = max(len(i) for i in ids)
        arr = np.zeros((len(ids), T), np.int64)
        for b, i in enumerate(ids):
            arr[b, :len(i)] = i
        lens = torch.tensor([len(i) for i in ids], dtype=torch.int32, device=self.device)
        # one length scale per batch (the engine groups by speed upstream)
        ls = 1.0 / max(1e-3, float(np.mean(speeds)))
        with self._gpu_lock, torch.inference_mode(), self._stream_ctx():
            t0 = time.perf_counter()
            self._seed += 1
            if self.use_graphs and self._runner is None:
                self._runner = VitsGraphRunner(self.model, self.device)
            synth = self._runner.synthesize if self._runner is not None else self.model.synthesize
            spk = None
            if self.model.n_speakers > 1:
                spk = torch.tensor(speakers or [0] * len(texts), dtype=torch.int64, device=self.device)
            pcm, n = synth(torch.from_numpy(arr).to(self.device), lens, seed=self._seed,
                           length_scale=ls, speakers=spk)
            t1 = time.perf_counter()
            pcm, n = pcm.cpu().numpy(), n.cpu().numpy()
            t2 = time.perf_counter()
            self.stats["gpu_s"] += t2 - t0       # launch to result on the host
            self.stats["launch_s"] += t1 - t0    # host side: launches + the frame-count sync
        self.stats["batches"] += 1
        if self._runner is not None:
            self.stats.update({f"graph_{k}": v for k, v in self._runner.stats.items()})
        self.stats["phrases"] += len(texts)
        self.stats["samples"] += int(n.sum())
        return [pcm[b, : int(n[b])].copy() for b in range(len(texts))]

    # phrase lengths (characters) and batch sizes the warm-up synthesizes: the
    # HIP-graph buckets (batch, symbols, frames) a served reply stream hits
    WARMUP_CHARS = (6, 12, 24, 40, 64, 96, 140)
    WARMUP_BATCHES = (1, 2, 4)

    def warmup_graphs(self) -> int:
        """Capture the graph buckets of typical reply phrases before serving
        (a capture costs an eager run plus the capture itself: taken lazily, the
        first minutes of serving pay them inside the replies). Returns the
        number of captures made. No-op without graphs."""
        if not self.use_graphs:
            return 0
        base = "turning on the kitchen lights and the living room music now "
        seed = self._seed
        for B in self.WARMUP_BATCHES:
            for n in self.WARMUP_CHARS:
                text = (base * (n // len(base) + 1))[:n]
                self.synthesize_batch([text] * B)
        self._seed = seed                 # the served replies' noise seeds as without warm-up
        caps = self._runner.stats["captures"] if self._runner is not None else 0
        for k in ("batches", "phrases", "samples", "gpu_s", "launch_s"):
            self.stats[k] = 0 if k in ("batches", "phrases", "samples") else 0.0
        self.stats["warmup_captures"] = caps
        return caps

    def _stream_ctx(self):
        """VITS runs on its own explicitly placed pool stream (a fixed hardware
        queue beside the decoders, docs/PERF.md "Stream placement"), never on
        whatever stream the executor thread happens to default to."""
        import contextlib
        if self.device.type != "cuda":
            return contextlib.nullcontext()
        if self._stream is None:
            from ..utils.streams import init_pools, placed_stream
            init_pools(self.device)
            self._stream = placed_stream(self.device, "tts")
        return torch.cuda.stream(self._stream)

    # ------------------------------------------------------ TextToSpeech API
    def output_format(self, requested: str | None) -> str:
        """The container a request for ``requested`` gets (see module doc)."""
        fmt = (requested or "wav").lower()
        if fmt in SUPPORTED_FORMATS:
            return fmt
        if self.format_policy == "error":
            raise UnsupportedAudioFormat(
                f"on-GPU TTS cannot encode {fmt!r} (supported: {', '.join(SUPPORTED_FORMATS)})")
        self.stats["format_downgrades"] += 1
        if fmt not in self._downgrade_logged:
            self._downgrade_logged.add(fmt)
            log.warning("TTS response_format %r is not available on the GPU backend (no %s "
                        "encoder); returning WAV and labelling the audio 'wav'", fmt, fmt)
        return "wav"

    async def synthesize(self, text: str, options: TTSOptions | None = None) -> TTSResult:
        if not text:
            raise ValueError("text cannot be empty")
        faults().check("tts_error")
        # decided before any GPU work: an "error" policy rejects at once
        fmt = self.output_format(options.response_format if options else None)
        speed = options.speed if options and options.speed > 0 else 1.0
        spk = self.speaker_id(options.voice if options else None)
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._pending.append((text, speed, spk, fut))
        if len(self._pending) >= self.max_batch or self._flusher is None or self._flusher.done():
            self._flusher = loop.create_task(self._flush())
        pcm = await fut
        if fmt == "pcm":
            data = pcm.astype("<i2").tobytes()
        else:
            data = pcm16_to_wav(pcm, self.cfg.sample_rate)
        return TTSResult(data, _CONTENT_TYPES[fmt], len(data), self.cfg.sample_rate, format=fmt)

    async def _flush(self) -> None:
        await asyncio.sleep(self.batch_window)
        while self._pending:
            batch, self._pending = self._pending[: self.max_batch], self._pending[self.max_batch:]
            try:
                outs = await asyncio.get_running_loop().run_in_executor(
                    None, self.synthesize_batch, [t for t, _, _, _ in batch],
                    [s for _, s, _, _ in batch], [k for _, _, k, _ in batch])
            except Exception as e:  # noqa: BLE001
                for *_, f in batch:
                    if not f.done():
                        f.set_exception(e)
                continue
            for (_, _, _, f), pcm in zip(batch, outs):
                if not f.done():
                    f.set_result(pcm)

    async def get_available_voices(self) -> list[str]:
        return self.voices()

    async def close(self) -> None:
        return None


def wav_info(data: bytes) -> tuple[int, int]:
    """(sample_rate, n_samples) of a PCM16 WAV produced by ``pcm16_to_wav``."""
    f = io.BytesIO(data)
    f.seek(24)
    sr = struct.unpack("<I", f.read(4))[0]
    f.seek(40)
    n = struct.unpack("<I", f.read(4))[0] // 2
    return sr, n
