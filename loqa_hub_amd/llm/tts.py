"""Text-to-speech contract (``internal/llm/tts.go``) and the OpenAI-compatible
TTS client (``internal/llm/openai_tts_client.go``).

``TextToSpeech`` is implemented by ``OpenAITTSClient`` (external service, the
reference path) and by the on-GPU VITS engine (``engine/tts_engine.py``).

Client behaviour kept: ``GET {url}/audio/voices`` connection test at creation
(:292-316); ``POST {url}/audio/speech`` with ``{model:"tts-1", input, voice,
response_format, speed, normalization_options?}`` where
``normalization_options = {"normalize": false}`` only when normalisation is
off (:39-46, :142-158); a concurrency semaphore of ``max_concurrent`` with a 5 s
acquire timeout ("TTS synthesis queue full", :106-112); voice list cached for
1 h (:227-283).
"""
from __future__ import annotations

import asyncio
import json
import time
from dataclasses import dataclass
from typing import Protocol

from .http import AiohttpClient, HTTPClient
from ..utils.faults import faults


@dataclass
class TTSOptions:
    voice: str = ""
    speed: float = 0.0
    response_format: str = ""
    normalize: bool = True


@dataclass
class TTSResult:
    audio: bytes
    content_type: str
    length: int
    sample_rate: int = 0
    # the container the bytes are actually in ("wav", "pcm", "mp3", ...): what
    # a consumer labels the audio with (gRPC AudioResponse.audio_format, the
    # NATS audio message), which can differ from the requested response_format
    # when the backend cannot produce that one (engine/tts_engine.py)
    format: str = ""


class TextToSpeech(Protocol):
    async def synthesize(self, text: str, options: TTSOptions | None = None) -> TTSResult: ...

    async def get_available_voices(self) -> list[str]: ...

    async def close(self) -> None: ...


class OpenAITTSClient:
    QUEUE_WAIT_S = 5.0
    VOICE_CACHE_S = 3600.0

    def __init__(self, cfg, *, client: HTTPClient | None = None):
        if not cfg.url:
            raise ValueError("TTS URL cannot be empty")
        self.cfg = cfg
        self.base_url = cfg.url.rstrip("/")
        self.client = client or AiohttpClient()
        self._sem = asyncio.Semaphore(max(1, int(cfg.max_concurrent)))
        self._voices: list[str] = []
        self._voices_t = 0.0

    @classmethod
    async def create(cls, cfg, *, client: HTTPClient | None = None) -> "OpenAITTSClient":
        c = cls(cfg, client=client)
        try:
            await c.test_connection()
        except Exception as e:
            raise ConnectionError(f"failed to connect to TTS service: {e}") from e
        return c

    async def test_connection(self) -> None:
        r = await self.client.request("GET", self.base_url + "/audio/voices", timeout=5.0)
        if r.status != 200:
            raise ConnectionError(f"TTS service returned status {r.status}")

    def build_request(self, text: str, options: TTSOptions | None) -> dict:
        voice, speed = self.cfg.voice, self.cfg.speed
        fmt, normalize = self.cfg.response_format, self.cfg.normalize
        if options is not None:
            voice = options.voice or voice
            speed = options.speed if options.speed > 0 else speed
            fmt = options.response_format or fmt
            normalize = options.normalize
        req = {"model": "tts-1", "input": text, "voice": voice, "response_format": fmt}
        if speed:
            req["speed"] = speed
        if not normalize:
            req["normalization_options"] = {"normalize": False}
        return req

    async def synthesize(self, text: str, options: TTSOptions | None = None) -> TTSResult:
        if not text:
            raise ValueError("text cannot be empty")
        faults().check("tts_error")
        try:
            await asyncio.wait_for(self._sem.acquire(), self.QUEUE_WAIT_S)
        except asyncio.TimeoutError:
            raise RuntimeError("TTS synthesis queue full, request timed out") from None
        try:
            body = json.dumps(self.build_request(text, options)).encode()
            try:
                r = await self.client.request(
                    "POST", self.base_url + "/audio/speech", body=body,
                    headers={"Content-Type": "application/json", "Accept": "audio/*"},
                    timeout=self.cfg.timeout)
            except Exception as e:
                raise ConnectionError(f"TTS HTTP request failed: {e}") from e
            if r.status != 200:
                raise RuntimeError(f"TTS request failed with status {r.status}: "
                                   f"{r.body.decode(errors='replace')}")
            ctype = r.headers.get("Content-Type", "")
            fmt = (options.response_format if options and options.response_format
                   else self.cfg.response_format)
            return TTSResult(r.body, ctype, len(r.body), format=fmt)
        finally:
            self._sem.release()

    async def get_available_voices(self) -> list[str]:
        if self._voices and time.monotonic() - self._voices_t < self.VOICE_CACHE_S:
            return list(self._voices)
        r = await self.client.request("GET", self.base_url + "/audio/voices",
                                      headers={"Accept": "application/json"}, timeout=10.0)
        if r.status != 200:
            raise RuntimeError(f"voices request failed with status {r.status}")
        try:
            voices = list(json.loads(r.body).get("voices") or [])
        except ValueError as e:
            raise ValueError(f"failed to decode voices response: {e}") from e
        self._voices, self._voices_t = voices, time.monotonic()
        return list(voices)

    async def close(self) -> None:
        close = getattr(self.client, "close", None)
        if close is not None:
            await close()
