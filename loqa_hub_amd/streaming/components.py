"""Streaming subsystem composition (``internal/llm/streaming_constructor.go``).

Builds parser + progressive TTS pipeline + interrupt handler + metrics from
``cfg.streaming`` (force timeout = 2 x interrupt timeout, :78-126), runs the
streaming self-test when enabled (failing hard only if fallback is disabled),
supports live ``update_configuration`` (:129-164) and ``get_health_status``.

Deliberate fix: ``process_streaming_command`` registers the
session *before* starting work; the reference looks the session up first and
therefore always fails with "no context found" (:167-196).
"""
from __future__ import annotations

import asyncio
import logging
import time
from dataclasses import dataclass

from ..llm.command_parser import CommandParser, OllamaBackend
from ..llm.tts import TextToSpeech, TTSOptions
from .audio_pipeline import StreamingAudioPipeline
from .interrupt import StreamingInterruptHandler
from .metrics import StreamingMetricsCollector
from .parser import (GPUStreamingBackend, OllamaStreamingBackend, StreamingCommandParser,
                     StreamingMetrics, StreamingResult)

log = logging.getLogger("loqa.streaming")


@dataclass
class StreamingHealthStatus:
    parser_enabled: bool
    active_sessions: int
    active_pipelines: int
    metrics_enabled: bool
    overall_health: str
    last_health_check: float

    def to_json(self) -> dict:
        from datetime import datetime, timezone
        from ..events import rfc3339
        return {"parser_enabled": self.parser_enabled, "active_sessions": self.active_sessions,
                "active_pipelines": self.active_pipelines,
                "metrics_enabled": self.metrics_enabled, "overall_health": self.overall_health,
                "last_health_check": rfc3339(datetime.fromtimestamp(self.last_health_check,
                                                                    timezone.utc))}


def tts_options_from(cfg) -> TTSOptions:
    return TTSOptions(cfg.tts.voice, cfg.tts.speed, cfg.tts.response_format, cfg.tts.normalize)


class StreamingComponents:
    def __init__(self, parser: StreamingCommandParser, pipeline: StreamingAudioPipeline,
                 interrupts: StreamingInterruptHandler, metrics: StreamingMetricsCollector):
        self.parser = parser
        self.audio_pipeline = pipeline
        self.interrupt_handler = interrupts
        self.metrics = metrics
        self._watchers: set[asyncio.Task] = set()

    @classmethod
    async def create(cls, cfg, tts: TextToSpeech, *, backend=None, http_client=None,
                     fallback: CommandParser | None = None) -> "StreamingComponents":
        if cfg is None:
            raise ValueError("configuration cannot be nil")
        sc = cfg.streaming
        if backend is None:
            backend = OllamaStreamingBackend(sc.ollama_url, sc.model, client=http_client)
        if fallback is None:
            fallback = CommandParser(OllamaBackend(sc.ollama_url, sc.model, client=http_client))
        parser = StreamingCommandParser(backend, fallback, sc.enabled,
                                        max_buffer_time=sc.max_buffer_time,
                                        max_tokens_per_phrase=sc.max_tokens_per_phrase)
        pipe = StreamingAudioPipeline(tts, tts_options_from(cfg),
                                      sc.audio_concurrency if sc.audio_concurrency > 0 else 3)
        comps = cls(parser, pipe, StreamingInterruptHandler(sc.interrupt_timeout,
                                                            2 * sc.interrupt_timeout),
                    StreamingMetricsCollector(sc.metrics_enabled))
        if sc.enabled:
            try:
                await parser.test_streaming_connection()
            except Exception as e:
                if not sc.fallback_enabled:
                    raise RuntimeError(f"streaming test failed and fallback disabled: {e}") from e
                log.warning("streaming self-test failed, fallback enabled: %s", e)
        return comps

    @classmethod
    def for_processor(cls, cfg, processor) -> "StreamingComponents":
        """The hub's components when the replies stream from the on-GPU decode
        (``streaming_constructor.go:38-126``, composed - the reference never
        constructs them). The parser streams the local engine's constrained
        decode (``GPUStreamingBackend``: it joins the running batch); the audio
        pipeline is the processor's own progressive pipeline, so
        ``active_pipelines`` counts replies being spoken. A data-parallel
        front end has no local engine: its replies stream inside the GPU
        workers, which report each session's metrics with the result. No
        self-test decode is run at start-up (the reference's self-test probes
        an external Ollama; the engine here is already warmed up)."""
        sc = cfg.streaming
        pipe = getattr(processor, "pipeline", None)
        llm = getattr(pipe, "llm", None)
        backend = GPUStreamingBackend(llm) if llm is not None else None
        parser = StreamingCommandParser(backend, None, sc.enabled,
                                        max_buffer_time=sc.max_buffer_time,
                                        max_tokens_per_phrase=sc.max_tokens_per_phrase)
        audio = getattr(processor, "speech_pipeline", None) or StreamingAudioPipeline(
            getattr(processor, "tts", None), tts_options_from(cfg),
            sc.audio_concurrency if sc.audio_concurrency > 0 else 3)
        return cls(parser, audio, StreamingInterruptHandler(sc.interrupt_timeout,
                                                            2 * sc.interrupt_timeout),
                   StreamingMetricsCollector(sc.metrics_enabled))

    # -- progressive replies of the voice processors as streaming sessions
    def begin_speech_session(self, session_id: str, speech) -> None:
        """``speech``: anything with ``cancel()`` (a ``ProgressiveSpeech``, or
        the DP front end's handle on a worker's reply)."""
        self.metrics.record_session_start(session_id)
        self.interrupt_handler.register_session(session_id, cancel=speech.cancel,
                                                audio_pipeline=speech)

    def end_speech_session(self, session_id: str, m: dict | None) -> None:
        if m:
            self.metrics.record_session_metrics(session_id, StreamingMetrics(**m))
        s = self.interrupt_handler.active.get(session_id)
        if s is not None and s.interrupted_at is None:
            self.interrupt_handler.active.pop(session_id, None)

    def update_configuration(self, cfg) -> None:
        if cfg is None:
            raise ValueError("configuration cannot be nil")
        sc = cfg.streaming
        self.parser.enabled = sc.enabled and self.parser.backend is not None
        b = self.parser.backend
        if isinstance(b, OllamaStreamingBackend):
            b.url, b.model = sc.ollama_url.rstrip("/"), sc.model
        self.audio_pipeline.update_tts_options(tts_options_from(cfg))
        if sc.audio_concurrency > 0:
            self.audio_pipeline.max_concurrent = sc.audio_concurrency
        self.interrupt_handler.grace_period = sc.interrupt_timeout
        self.interrupt_handler.force_timeout = 2 * sc.interrupt_timeout
        self.metrics.enabled = sc.metrics_enabled

    async def process_streaming_command(self, transcription: str,
                                        session_id: str) -> StreamingResult:
        self.metrics.record_session_start(session_id)
        session = self.interrupt_handler.register_session(session_id)
        try:
            result = await self.parser.parse_command_streaming(transcription)
        except Exception as e:
            self.interrupt_handler.active.pop(session_id, None)
            raise RuntimeError(f"streaming command parsing failed: {e}") from e
        session.streaming_result = result
        session.cancel = result.cancel
        if not self.parser.enabled:
            self.metrics.record_fallback()
        t = asyncio.get_running_loop().create_task(self._process_audio_stream(session_id, result))
        self._watchers.add(t)
        t.add_done_callback(self._watchers.discard)
        return result

    async def _process_audio_stream(self, session_id: str, result: StreamingResult) -> None:
        try:
            pc = self.audio_pipeline.start_pipeline(session_id, result.audio_phrases)
        except Exception as e:  # noqa: BLE001
            result.errors.try_put(e)
            return
        s = self.interrupt_handler.active.get(session_id)
        if s is not None:
            s.audio_pipeline = pc
        try:
            async for chunk in pc.audio_chunks:
                if chunk.is_last:
                    self.metrics.record_session_metrics(session_id, result.metrics)
                    break
                err, ok = pc.errors.try_get()
                if ok:
                    result.errors.try_put(err)
        finally:
            await self.audio_pipeline.stop_pipeline(session_id)
            self.interrupt_handler.active.pop(session_id, None)

    async def shutdown(self) -> None:
        await self.interrupt_handler.shutdown()
        for pid in self.audio_pipeline.get_active_pipelines():
            await self.audio_pipeline.stop_pipeline(pid)

    def get_health_status(self) -> StreamingHealthStatus:
        return StreamingHealthStatus(self.parser.enabled,
                                     len(self.interrupt_handler.get_active_session_ids()),
                                     len(self.audio_pipeline.get_active_pipelines()),
                                     self.metrics.enabled, self.metrics.assess_health_status(),
                                     time.time())
