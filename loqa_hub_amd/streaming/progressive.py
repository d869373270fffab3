"""Progressive speech of a live constrained decode.

The reference streams Ollama tokens through a ``PhraseBuffer`` into the
progressive TTS pipeline (``internal/llm/streaming_command_parser.go:162-292``
-> ``streaming_audio_pipeline.go:106-399``). On the MI355X path the tokens come
from the grammar-constrained decode itself: every engine step hands its newly
emitted ids (sampled + jump-forward) to ``ProgressiveSpeech.on_tokens``; a
``JSONFieldTap`` keeps only the characters of the reply field (the first
command's ``"response"`` - what the reference speaks, ``audio_service.go:689``),
phrases from the ``PhraseBuffer`` go through ``StreamingAudioPipeline`` (worker
pool + sequence re-ordering; the VITS engine batches the phrases of every live
session into one GPU call), and each phrase's audio is published on NATS
``audio.<relay>`` the moment it is ready - the first phrase is on the wire
while the decode is still generating the rest of the JSON.
"""
from __future__ import annotations

import asyncio
import io
import itertools
import logging
import struct
import time

from .audio_pipeline import StreamingAudioPipeline
from .chan import Chan, ChannelClosed
from .parser import PhraseBuffer

log = logging.getLogger("loqa.streaming.progressive")

_ESC = {'"': '"', "\\": "\\", "/": "/", "b": " ", "f": " ", "n": " ", "r": " ", "t": " "}


class JSONFieldTap:
    """Incremental scanner over well-formed JSON text that returns the
    characters of the string value of the first key in ``keys`` (escapes
    decoded, control escapes as spaces). ``feed`` -> (value chars, closed)."""

    def __init__(self, keys=("response",)):
        self.keys = set(keys)
        self.in_str = False
        self.esc = 0          # 0: none, 1: after backslash, >1: inside \\uXXXX (digits left + 1)
        self.buf: list[str] = []
        self.pending_key = ""
        self.last_key = ""
        self.after_colon = False
        self.capturing = False
        self.done = False

    def feed(self, text: str) -> tuple[str, bool]:
        out: list[str] = []
        closed = False
        for ch in text:
            if self.in_str:
                if self.esc == 1:
                    self.esc = 0
                    if ch == "u":
                        self.esc = 5
                        continue
                    c = _ESC.get(ch, ch)
                elif self.esc > 1:
                    self.esc -= 1
                    if self.esc == 1:
                        self.esc = 0
                    continue            # \\uXXXX: dropped (not speakable here)
                elif ch == "\\":
                    self.esc = 1
                    continue
                elif ch == '"':
                    self.in_str = False
                    if self.capturing:
                        self.capturing, self.done, closed = False, True, True
                    else:
                        self.pending_key = "".join(self.buf)
                    self.after_colon = False
                    continue
                else:
                    c = ch
                if self.capturing:
                    out.append(c)
                else:
                    self.buf.append(c)
                continue
            if ch == '"':
                self.in_str, self.buf = True, []
                self.capturing = (not self.done and self.after_colon
                                  and self.last_key in self.keys)
            elif ch == ":":
                self.last_key, self.after_colon = self.pending_key, True
            elif ch in ",{}[]":
                self.after_colon = False
        return "".join(out), closed


def wav_pcm(data: bytes) -> tuple[int, bytes] | None:
    """(sample rate, PCM16 payload) of a RIFF/WAVE PCM16 mono blob, else None."""
    if len(data) < 44 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        return None
    f = io.BytesIO(data)
    f.seek(12)
    sr = None
    while True:
        hdr = f.read(8)
        if len(hdr) < 8:
            return None
        cid, n = hdr[:4], struct.unpack("<I", hdr[4:])[0]
        if cid == b"fmt ":
            fmt = f.read(n)
            if struct.unpack("<H", fmt[:2])[0] != 1 or struct.unpack("<H", fmt[14:16])[0] != 16:
                return None
            sr = struct.unpack("<I", fmt[4:8])[0]
        elif cid == b"data":
            return (sr, f.read(n)) if sr else None
        else:
            f.seek(n, 1)


_session_ids = itertools.count(1)


class ProgressiveSpeech:
    """One utterance's progressive reply: decode tokens -> reply phrases ->
    ordered synthesis -> per-phrase NATS publication."""

    def __init__(self, relay_id: str, tokenizer, pipeline: StreamingAudioPipeline, publisher,
                 *, max_buffer_time: float = 2.0, max_tokens_per_phrase: int = 50,
                 loop: asyncio.AbstractEventLoop | None = None):
        self.relay_id = relay_id
        self.tok = tokenizer
        self.pipeline = pipeline
        self.publisher = publisher
        self.loop = loop or asyncio.get_running_loop()
        self.tap = JSONFieldTap(("response",))
        self.pb = PhraseBuffer(max_buffer_time, max_tokens_per_phrase)
        self.phrases = Chan(64)
        self.session_id = f"speech_{next(_session_ids)}_{time.time_ns()}"
        self.pc = pipeline.start_pipeline(self.session_id, self.phrases)
        self.chunks: list = []
        self.published = 0
        self.t_start = time.perf_counter()
        self.mono_start = time.monotonic()   # the streaming metrics' clock
        self.t_first_piece = 0.0       # first character of the reply field
        self.t_first_phrase = 0.0      # first phrase handed to TTS
        self.t_first_audio = 0.0       # first phrase's audio published
        self.t_field_closed = 0.0      # the reply field was complete
        self.t_done = 0.0              # every phrase delivered (or interrupted)
        self.text: list[str] = []
        self.n_pieces = 0
        self.n_phrases = 0
        self.interrupted = False
        self._closed = False
        self._consumer = self.loop.create_task(self._consume())

    # -- engine thread -> event loop (the scheduler thread only enqueues)
    def on_tokens(self, ids) -> None:
        self.loop.call_soon_threadsafe(self._feed, list(ids))

    def _feed(self, ids: list[int]) -> None:
        if self._closed:
            return
        piece, closed = self.tap.feed(self.tok.decode(ids))
        if piece:
            if not self.t_first_piece:
                self.t_first_piece = time.perf_counter()
            self.n_pieces += 1
            self.text.append(piece)
            phrase = self.pb.add_token(piece)
            if phrase:
                self._emit(phrase)
        if closed:
            self.t_field_closed = time.perf_counter()
            rest = self.pb.flush()
            if rest:
                self._emit(rest)
            self._close()

    def _emit(self, phrase: str) -> None:
        if not phrase.strip():
            return
        if not self.t_first_phrase:
            self.t_first_phrase = time.perf_counter()
        self.n_phrases += 1
        if not self.phrases.try_put(phrase.strip()):
            log.warning("phrase queue full for %s, phrase dropped", self.relay_id)

    def _close(self) -> None:
        if not self._closed:
            self._closed = True
            self.phrases.close()

    def cancel(self) -> None:
        """Interrupt the reply (a new wake word from the same relay,
        ``streaming_interrupt_handler.go:69-119``): no further phrase is
        synthesised or published; ``finish`` returns what was already spoken.
        The decode and its command queue are not affected."""
        if self.interrupted or self.t_done:
            return
        self.interrupted = True
        self._close()
        # cancels the synthesis tasks and closes the chunk stream _consume reads
        self.loop.create_task(self.pipeline.stop_pipeline(self.session_id))

    async def _consume(self) -> None:
        try:
            async for chunk in self.pc.audio_chunks:
                if chunk.is_last or self.interrupted:
                    break
                self.chunks.append(chunk)
                if self.publisher is not None:
                    w = wav_pcm(chunk.audio)
                    sr = w[0] if w else 22050
                    fmt = "wav" if w else (chunk.content_type.split("/")[-1] or "wav")
                    try:
                        await self.publisher.stream_audio_to_relay(self.relay_id, chunk.audio, fmt, sr,
                                                                   "response", 3)
                        self.published += 1
                    except Exception as e:  # noqa: BLE001
                        log.warning("phrase publish to %s failed: %s", self.relay_id, e)
                if not self.t_first_audio:
                    self.t_first_audio = time.perf_counter()
        except ChannelClosed:
            pass
        finally:
            self.t_done = time.perf_counter()
            await self.pipeline.stop_pipeline(self.session_id)

    async def finish(self, fallback_text: str = "") -> tuple[bytes, int]:
        """After the decode: speak ``fallback_text`` if the reply field never
        streamed (e.g. a parse fallback), wait for every phrase, and return
        the whole reply as one WAV (sample rate) for the gRPC response."""
        if not self._closed:
            rest = self.pb.flush()
            if rest:
                self._emit(rest)
            elif not self.text and fallback_text:
                self._emit(fallback_text)
            self._close()
        await self._consumer
        pcm, sr = [], 0
        for c in self.chunks:
            w = wav_pcm(c.audio)
            if w is None:
                return (self.chunks[-1].audio if self.chunks else b""), 0
            sr = w[0]
            pcm.append(w[1])
        if not pcm:
            return b"", 0
        from ..engine.tts_engine import pcm16_to_wav
        import numpy as np
        return pcm16_to_wav(np.frombuffer(b"".join(pcm), "<i2"), sr), sr

    def metrics(self) -> dict:
        def ms(t):
            return round((t - self.t_start) * 1e3, 2) if t else None
        return {"first_phrase_ms": ms(self.t_first_phrase), "first_audio_ms": ms(self.t_first_audio),
                "field_closed_ms": ms(self.t_field_closed), "phrases": len(self.chunks),
                "published": self.published, "interrupted": self.interrupted,
                "streaming": self.streaming_metrics()}

    def streaming_metrics(self) -> dict:
        """The session as ``streaming.parser.StreamingMetrics`` fields (monotonic
        clock, ``streaming_metrics.go:121-153``): first token = first character
        of the reply field, completion = every phrase delivered."""
        def mono(t):
            return self.mono_start + (t - self.t_start) if t else 0.0
        return {"start_time": self.mono_start, "first_token_time": mono(self.t_first_piece),
                "first_phrase_time": mono(self.t_first_phrase),
                "completion_time": 0.0 if self.interrupted else mono(self.t_done),
                "token_count": self.n_pieces, "phrase_count": self.n_phrases,
                "buffer_overflows": 0, "interrupt_count": int(self.interrupted)}
