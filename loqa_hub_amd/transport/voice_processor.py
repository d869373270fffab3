"""Voice processors behind ``AudioService._process_winner``.

The reference's winner path (``audio_service.go:590-761``) is: STT over HTTP,
then the streaming-predictive bridge (instant ack) or ``ParseMultiCommand``, the
first command's response as the spoken reply, TTS over HTTP, NATS delivery.
Two interchangeable implementations:

* ``GPUVoiceProcessor`` - the MI355X path. Concurrent arbitration winners are
  micro-batched (``batch_window``, ``max_batch``) into ONE ``VoicePipeline``
  call: batched Whisper STT, one grammar-constrained multi-command decode per
  utterance, the command queue with rollback + NATS publish per utterance as
  soon as its own decode finishes, then batched TTS of the replies.
* ``ServiceVoiceProcessor`` - the reference's external-service path
  (BASELINE config 1): an STT client (``stt_client.py``), a ``CommandParser``
  over any ``LLMBackend`` (Ollama), optional bridge, optional TTS client.
"""
from __future__ import annotations

import asyncio
import logging
import time

import numpy as np

from ..llm.command_queue import CommandQueue
from ..llm.commands import MultiCommand
from ..llm.transcriber import TranscriptionResult
from .audio_service import (MSG_NO_COMMANDS, MSG_NO_SPEECH, MSG_PARSE_FAILED, MSG_STT_FAILED,
                            UtteranceResult)
from ..utils.faults import faults
from .device_commands import ExecutionContext, NATSCommandExecutor

log = logging.getLogger("loqa.processor")


def float_to_pcm16(audio: np.ndarray) -> np.ndarray:
    return np.clip(np.round(np.asarray(audio, np.float32) * 32767.0), -32768, 32767).astype(np.int16)


def _result_from(text: str, mc: MultiCommand | None, queue_ok: bool | None,
                 tr: TranscriptionResult | None) -> UtteranceResult:
    if not text:
        return UtteranceResult(success=False, command="no_speech", response_text=MSG_NO_SPEECH)
    if mc is None:
        return UtteranceResult(transcription=text, success=False, command="error",
                               response_text=MSG_PARSE_FAILED)
    if not mc.commands:
        return UtteranceResult(transcription=text, success=False, command="error",
                               response_text=MSG_NO_COMMANDS)
    first = mc.commands[0]
    reply = mc.combined_response if mc.is_multi and mc.combined_response else first.response
    res = UtteranceResult(transcription=text, response_text=reply,
                          intents=[c.intent for c in mc.commands],
                          confidence=first.confidence, entities=dict(first.entities),
                          success=queue_ok is not False)
    if tr is not None and tr.needs_confirmation:
        res.command = "confirmation_needed"
    return res


class GPUVoiceProcessor:
    def __init__(self, pipeline, *, tts=None, batch_window: float = 0.005, max_batch: int = 8,
                 tts_format: str = "wav"):
        self.pipeline = pipeline
        self.tts = tts
        self.tts_format = tts_format
        pipeline.batch_window, pipeline.max_batch = batch_window, max_batch
        self.stats = {"utterances": 0, "errors": 0}

    async def process(self, relay_id: str, request_id: str, audio: np.ndarray,
                      sample_rate: int, transcript_hint: str | None = None) -> UtteranceResult:
        """``transcript_hint``: synthetic-traffic ground truth that teacher-forces
        the (random-init) Whisper decoder; real relays never pass it. Concurrent
        calls are micro-batched by the pipeline (STT batch, continuous LLM batch)."""
        from ..engine.pipeline import PipelineJob
        j = PipelineJob(relay_id, request_id, float_to_pcm16(audio), transcript_hint)
        try:
            await self.pipeline.submit(j)
        except Exception as e:  # noqa: BLE001
            log.exception("GPU pipeline failed")
            self.stats["errors"] += 1
            return UtteranceResult(success=False, command="error", response_text=MSG_STT_FAILED,
                                   error=str(e))
        self.stats["utterances"] += 1
        if j.stt_failed:
            return UtteranceResult(success=False, command="error", response_text=MSG_STT_FAILED,
                                   error=j.error)
        text = j.transcription.text if j.transcription else ""
        ok = None if j.queue is None else j.queue.success
        r = _result_from(text, j.multi, ok, j.transcription)
        if self.tts is not None:
            await self._speak([r])
        return r

    async def _speak(self, results: list[UtteranceResult]) -> None:
        from ..llm.tts import TTSOptions
        opts = TTSOptions(response_format=self.tts_format)

        async def one(r: UtteranceResult):
            if not r.response_text:
                return
            try:
                t = await self.tts.synthesize(r.response_text, opts)
                r.audio, r.audio_format = t.audio, self.tts_format
                if t.sample_rate:
                    r.audio_duration = len(t.audio) / 2 / t.sample_rate
            except Exception as e:  # noqa: BLE001
                log.warning("TTS failed: %s", e)
        await asyncio.gather(*[one(r) for r in results])


class ServiceVoiceProcessor:
    def __init__(self, transcriber, parser, *, nats=None, tts=None, bridge=None,
                 execute_commands: bool = True, tts_format: str = "wav"):
        self.transcriber = transcriber
        self.parser = parser
        self.nats = nats
        self.tts = tts
        self.bridge = bridge
        self.execute_commands = execute_commands
        self.tts_format = tts_format

    async def process(self, relay_id: str, request_id: str, audio: np.ndarray,
                      sample_rate: int) -> UtteranceResult:
        t0 = time.perf_counter()
        try:
            faults().check("stt_error")
            tr = await self.transcriber.transcribe_with_confidence(audio, sample_rate)
        except Exception as e:  # noqa: BLE001
            return UtteranceResult(success=False, command="error", response_text=MSG_STT_FAILED,
                                   error=str(e))
        if not tr.text:
            return UtteranceResult(success=False, command="no_speech", response_text=MSG_NO_SPEECH)
        if self.bridge is not None:
            try:
                sess = await asyncio.wait_for(self.bridge.process_voice_command(tr.text), 2.0)
                if sess.predictive_response is not None:
                    c = sess.classification
                    res = UtteranceResult(transcription=tr.text,
                                          response_text=sess.predictive_response.immediate_ack,
                                          intents=[c.intent], confidence=c.confidence,
                                          entities=dict(c.entities))
                    await self._speak(res)
                    return res
            except Exception as e:  # noqa: BLE001
                log.info("bridge fallback: %s", e)
        try:
            faults().check("llm_timeout")
            mc = await self.parser.parse_multi_command(tr.text)
        except Exception as e:  # noqa: BLE001
            log.warning("command parsing failed: %s", e)
            mc = None
        ok = None
        if mc is not None and mc.commands and self.execute_commands and self.nats is not None:
            q = CommandQueue(mc.commands)
            r = await q.execute(NATSCommandExecutor(self.nats, ExecutionContext(
                relay_id, request_id, "", tr.text)))
            ok = r.success
        res = _result_from(tr.text, mc, ok, tr)
        await self._speak(res)
        log.debug("processed %s in %.1f ms", request_id, (time.perf_counter() - t0) * 1e3)
        return res

    async def _speak(self, r: UtteranceResult) -> None:
        if self.tts is None or not r.response_text:
            return
        from ..llm.tts import TTSOptions
        try:
            t = await self.tts.synthesize(r.response_text, TTSOptions(response_format=self.tts_format))
            r.audio, r.audio_format = t.audio, self.tts_format
        except Exception as e:  # noqa: BLE001
            log.warning("TTS failed: %s", e)
