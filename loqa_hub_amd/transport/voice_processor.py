"""Voice processors behind ``AudioService._process_winner``.

The reference's winner path (``audio_service.go:590-761``) is: STT over HTTP,
then the streaming-predictive bridge (instant ack) or ``ParseMultiCommand``, the
first command's response as the spoken reply, TTS over HTTP, NATS delivery.
Two interchangeable implementations:

* ``GPUVoiceProcessor`` - the MI355X path. Concurrent arbitration winners are
  micro-batched into the ``VoicePipeline`` (continuous-batching Whisper STT,
  ONE grammar-constrained multi-command decode per utterance, the command
  queue with rollback + NATS publish as soon as its own decode finishes). The
  streaming-predictive bridge is fed that decode's parse (no second LLM pass)
  and decides the strategy / instant ack exactly as the reference's does. The
  reply is spoken by the on-GPU VITS engine (or the OpenAI-compatible
  client): progressively from the live decode when streaming is enabled
  (``streaming/progressive.py``: the reply field's phrases are synthesised and
  published on ``audio.<relay>`` while the decode runs), else as one file after
  it.
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
    # the first command's response, as the reference (audio_service.go:687-689)
    res = UtteranceResult(transcription=text, response_text=first.response or mc.combined_response,
                          intents=[c.intent for c in mc.commands],
                          confidence=first.confidence, entities=dict(first.entities),
                          success=queue_ok is not False)
    if tr is not None and tr.needs_confirmation:
        res.command = "confirmation_needed"
    return res


class GPUVoiceProcessor:
    takes_pcm16 = True      # AudioService hands over the relay's raw PCM16 samples

    def __init__(self, pipeline, *, tts=None, bridge=None, progressive: bool = False,
                 speech_pipeline=None, batch_window: float = 0.005, max_batch: int = 8,
                 tts_format: str = "wav", tts_options=None, bridge_timeout: float = 2.0,
                 max_buffer_time: float = 2.0, max_tokens_per_phrase: int = 50):
        self.pipeline = pipeline
        self.tts = tts
        self.bridge = bridge
        self.bridge_timeout = bridge_timeout
        self.tts_format = tts_format
        self.tts_options = tts_options
        self.progressive = progressive and tts is not None
        if self.progressive and speech_pipeline is None:
            from ..streaming.audio_pipeline import StreamingAudioPipeline
            speech_pipeline = StreamingAudioPipeline(tts, tts_options)
        self.speech_pipeline = speech_pipeline
        self.max_buffer_time, self.max_tokens_per_phrase = max_buffer_time, max_tokens_per_phrase
        self.publisher = None           # NATS audio publisher (HubServer.start attaches it)
        self.streaming = None           # StreamingComponents (HubServer.start attaches them)
        self._speaking: dict[str, object] = {}   # relay id -> its reply still being spoken
        pipeline.batch_window, pipeline.max_batch = batch_window, max_batch
        self.stats = {"utterances": 0, "errors": 0, "bridge_sessions": 0, "bridge_ack": 0,
                      "bridge_fallback": 0, "interrupted": 0,
                      "progressive": 0, "first_audio_ms_sum": 0.0, "first_audio_n": 0}
        # a list that collects every finished PipelineJob (phase timestamps for
        # a benchmark's per-phase breakdown); None: not collected
        self.job_sink: list | None = None

    def attach_publisher(self, publisher) -> None:
        self.publisher = publisher

    def attach_streaming(self, components) -> None:
        """Progressive replies become streaming sessions: registered with the
        interrupt handler, recorded in the streaming metrics."""
        self.streaming = components

    def interrupt_relay(self, relay_id: str, reason: str = "new_command") -> bool:
        """A new wake-word winner on ``relay_id``: stop speaking the reply that
        relay is still receiving (``streaming_interrupt_handler.go:69-119``)."""
        speech = self._speaking.get(relay_id)
        if speech is None or speech.interrupted or speech.t_done:
            return False
        self.stats["interrupted"] += 1
        ih = self.streaming.interrupt_handler if self.streaming is not None else None
        if ih is not None and speech.session_id in ih.active:
            ih.interrupt_session(speech.session_id, reason)
        else:
            speech.cancel()
        return True

    def new_pcm_slot(self):
        """A pinned stager slot for one relay's incoming PCM (AudioService)."""
        return self.pipeline.stt.new_pcm_slot()

    async def close(self) -> None:
        """Stop the engines' scheduler threads (a TP leader also releases its
        followers)."""
        await asyncio.to_thread(self.pipeline.llm.stop)
        stop = getattr(self.pipeline.stt, "stop", None)
        if stop is not None:
            await asyncio.to_thread(stop)

    async def process(self, relay_id: str, request_id: str, audio: np.ndarray,
                      sample_rate: int, transcript_hint: str | None = None,
                      pcm16: np.ndarray | None = None, pcm_slot=None) -> UtteranceResult:
        """``transcript_hint``: synthetic-traffic ground truth that teacher-forces
        the (random-init) Whisper decoder; real relays never pass it. ``pcm16``:
        the relay's raw samples (skips the float round trip); ``pcm_slot``: the
        pinned stager slot its chunks were appended to as they arrived (the
        STT upload copies it straight to HBM). Concurrent calls are
        micro-batched by the pipeline (STT batch, continuous LLM batch)."""
        from ..engine.pipeline import PipelineJob
        if pcm_slot is not None:
            pcm = np.zeros(0, np.int16)
        else:
            pcm = pcm16 if pcm16 is not None else float_to_pcm16(audio)
        j = PipelineJob(relay_id, request_id, pcm, transcript_hint, staged=pcm_slot)
        speech = None
        if self.progressive:
            from ..streaming.progressive import ProgressiveSpeech
            speech = ProgressiveSpeech(relay_id, self.pipeline.llm.tok, self.speech_pipeline,
                                       self.publisher, max_buffer_time=self.max_buffer_time,
                                       max_tokens_per_phrase=self.max_tokens_per_phrase)
            j.on_tokens = speech.on_tokens
            self._speaking[relay_id] = speech
            if self.streaming is not None:
                self.streaming.begin_speech_session(speech.session_id, speech)
        try:
            await self.pipeline.submit(j)
            if self.job_sink is not None:
                self.job_sink.append(j)
            if "enc0" in j.t and "start" in j.t:
                # process() runs at end of speech: the gap until the encoder
                # (upload + log-mel) starts on this utterance
                self.stats["eos_enc_gap_s"] = self.stats.get("eos_enc_gap_s", 0.0) + \
                    j.t["enc0"] - j.t["start"]
                self.stats["eos_enc_n"] = self.stats.get("eos_enc_n", 0) + 1
                if "enc1" in j.t:     # upload + log-mel + encoder + cross K|V, synchronised
                    self.stats["enc_span_s"] = self.stats.get("enc_span_s", 0.0) + \
                        j.t["enc1"] - j.t["enc0"]
        except Exception as e:  # noqa: BLE001
            if pcm_slot is not None:
                pcm_slot.release()        # idempotent: a no-op once uploaded
            log.exception("GPU pipeline failed")
            self.stats["errors"] += 1
            if speech is not None:
                await self._end_speech(relay_id, speech)
            return UtteranceResult(success=False, command="error", response_text=MSG_STT_FAILED,
                                   error=str(e))
        self.stats["utterances"] += 1
        if j.stt_failed:
            if speech is not None:
                await self._end_speech(relay_id, speech)
            return UtteranceResult(success=False, command="error", response_text=MSG_STT_FAILED,
                                   error=j.error)
        text = j.transcription.text if j.transcription else ""
        ok = None if j.queue is None else j.queue.success
        r = _result_from(text, j.multi, ok, j.transcription)
        r.metrics = {"t": dict(j.t)}
        if self.bridge is not None and r.success and j.multi is not None and j.multi.commands:
            await self._bridge(r, j, ack=speech is None)
        if speech is not None:
            audio_b, sr = await self._end_speech(relay_id, speech, r.response_text)
            r.audio, r.audio_format, r.audio_sample_rate = audio_b, "wav", sr
            r.audio_published = self.publisher is not None and speech.published > 0
            if sr:
                r.audio_duration = max(0, len(audio_b) - 44) / 2 / sr
            m = speech.metrics()
            done_t = j.t.get("llm_done", 0.0)
            m["first_phrase_before_decode_done"] = bool(speech.t_first_phrase and done_t
                                                        and speech.t_first_phrase < done_t)
            m["first_audio_before_decode_done"] = bool(speech.t_first_audio and done_t
                                                       and speech.t_first_audio < done_t)
            r.metrics["speech"] = m
            self.stats["progressive"] += 1
            for k in ("phrase", "audio"):
                key = f"{k}_before_decode_done"
                self.stats[key] = self.stats.get(key, 0) + int(m[f"first_{k}_before_decode_done"])
            if m["first_audio_ms"] is not None:
                self.stats["first_audio_ms_sum"] += m["first_audio_ms"]
                self.stats["first_audio_n"] += 1
        elif self.tts is not None:
            await self._speak([r])
        return r

    async def _end_speech(self, relay_id: str, speech, fallback_text: str = ""):
        try:
            return await speech.finish(fallback_text)
        finally:
            if self._speaking.get(relay_id) is speech:
                del self._speaking[relay_id]
            if self.streaming is not None:
                self.streaming.end_speech_session(speech.session_id, speech.streaming_metrics())

    async def _bridge(self, r: UtteranceResult, j, ack: bool) -> None:
        """The streaming-predictive bridge on the shared decode: classification
        from the parsed first command, the decode itself as the streaming
        result. Its instant ack replaces the reply when speech is not already
        streaming from the decode (the reference answers with the ack,
        audio_service.go:641-656)."""
        from ..streaming.parser import completed_result
        first = j.multi.commands[0]
        try:
            sess = await asyncio.wait_for(
                self.bridge.process_voice_command(r.transcription, parsed=first,
                                                  streamed=completed_result(first)),
                self.bridge_timeout)
        except Exception as e:  # noqa: BLE001
            self.stats["bridge_fallback"] += 1
            log.info("bridge fallback: %s", e)
            return
        r.strategy = sess.strategy
        self.stats["bridge_sessions"] += 1
        if sess.predictive_response is not None:
            self.stats["bridge_ack"] += 1
            if ack:
                r.response_text = sess.predictive_response.immediate_ack

    async def _speak(self, results: list[UtteranceResult]) -> None:
        from ..llm.tts import TTSOptions
        opts = self.tts_options or TTSOptions(response_format=self.tts_format)

        async def one(r: UtteranceResult):
            if not r.response_text:
                return
            try:
                t = await self.tts.synthesize(r.response_text, opts)
                r.audio, r.audio_format = t.audio, t.format or opts.response_format or self.tts_format
                if t.sample_rate:
                    r.audio_sample_rate = t.sample_rate
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
            r.audio, r.audio_format = t.audio, t.format or self.tts_format
        except Exception as e:  # noqa: BLE001
            log.warning("TTS failed: %s", e)
