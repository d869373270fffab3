"""OpenAI-compatible STT REST client (``internal/llm/stt_client.go``).

The reference path for BASELINE config 1 (external STT service); the MI355X
path is the on-GPU Whisper engine (engine/stt_engine.py). Kept behaviour:
``/health`` check at construction (:89-105), ``POST /v1/audio/transcriptions``
multipart with ``file=audio.wav`` (32-bit IEEE-float mono WAV, :365-398),
``model=tiny``, ``language``, ``temperature=0.0``, ``response_format=json``
(:136-149), ``{"text": ...}`` response, then wake-word post-processing
(:401-513, shared with the GPU path via ``transcriber.py``). The WAV body is
built with one vectorised ``tobytes`` instead of a per-sample append
(SURVEY §3.7 #10).
"""
from __future__ import annotations

import json
import logging
import struct
import time
import uuid

import numpy as np

from .http import AiohttpClient, HTTPClient
from .transcriber import TranscriptionResult, post_process_transcription

log = logging.getLogger("loqa.stt")


def float32_to_wav(samples: np.ndarray, sample_rate: int) -> bytes:
    data = np.ascontiguousarray(samples, dtype="<f4").tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 3, 1, sample_rate, sample_rate * 4, 4, 32)
    hdr += b"data" + struct.pack("<I", len(data))
    return hdr + data


def multipart_body(fields: list[tuple[str, str]], file_field: str, filename: str,
                   file_bytes: bytes, file_type: str = "application/octet-stream"
                   ) -> tuple[bytes, str]:
    boundary = uuid.uuid4().hex
    parts = [(f'--{boundary}\r\nContent-Disposition: form-data; name="{file_field}"; '
              f'filename="{filename}"\r\nContent-Type: {file_type}\r\n\r\n').encode(),
             file_bytes, b"\r\n"]
    for k, v in fields:
        parts.append((f'--{boundary}\r\nContent-Disposition: form-data; name="{k}"\r\n\r\n'
                      f"{v}\r\n").encode())
    parts.append(f"--{boundary}--\r\n".encode())
    return b"".join(parts), f"multipart/form-data; boundary={boundary}"


class STTClient:
    def __init__(self, base_url: str = "", language: str = "en", *,
                 client: HTTPClient | None = None, timeout: float = 30.0):
        self.base_url = (base_url or "http://localhost:8000").rstrip("/")
        self.language = language or "en"
        self.client = client or AiohttpClient()
        self.timeout = timeout

    @classmethod
    async def create(cls, base_url: str = "", language: str = "en", *,
                     enable_health_check: bool = True, client: HTTPClient | None = None
                     ) -> "STTClient":
        c = cls(base_url, language, client=client)
        if enable_health_check:
            try:
                await c.health_check()
            except Exception as e:
                raise ConnectionError(f"STT service health check failed: {e}") from e
        return c

    async def health_check(self) -> None:
        try:
            r = await self.client.request("GET", self.base_url + "/health", timeout=self.timeout)
        except Exception as e:
            raise ConnectionError(f"failed to connect to STT service at {self.base_url}: {e}") from e
        if r.status != 200:
            raise ConnectionError(f"STT service health check failed with status: {r.status}")

    async def _request(self, audio: np.ndarray, sample_rate: int) -> str:
        if audio is None or len(audio) == 0:
            raise ValueError("empty audio data")
        if sample_rate <= 0:
            raise ValueError(f"invalid sample rate: {sample_rate}")
        body, ctype = multipart_body(
            [("model", "tiny"), ("language", self.language), ("temperature", "0.0"),
             ("response_format", "json")], "file", "audio.wav",
            float32_to_wav(audio, sample_rate))
        t0 = time.perf_counter()
        try:
            r = await self.client.request("POST", self.base_url + "/v1/audio/transcriptions",
                                          body=body, headers={"Content-Type": ctype},
                                          timeout=self.timeout)
        except Exception as e:
            raise ConnectionError(f"transcription HTTP request failed: {e}") from e
        if r.status != 200:
            raise RuntimeError(f"transcription failed with status {r.status}: "
                               f"{r.body.decode(errors='replace')}")
        try:
            text = str(json.loads(r.body).get("text", ""))
        except (ValueError, AttributeError) as e:
            raise ValueError(f"failed to parse transcription response: {e}") from e
        log.info("transcription completed in %.1f ms", (time.perf_counter() - t0) * 1e3)
        return text

    async def transcribe(self, audio: np.ndarray, sample_rate: int) -> str:
        return post_process_transcription(await self._request(audio, sample_rate)).cleaned_text

    async def transcribe_with_confidence(self, audio: np.ndarray,
                                         sample_rate: int) -> TranscriptionResult:
        p = post_process_transcription(await self._request(audio, sample_rate))
        return TranscriptionResult(p.cleaned_text, p.confidence_estimate, p.wake_word_detected,
                                   p.wake_word_variant, p.needs_confirmation)

    async def close(self) -> None:
        close = getattr(self.client, "close", None)
        if close is not None:
            await close()
