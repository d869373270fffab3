"""gRPC ``AudioService.StreamAudio`` with multi-relay wake-word arbitration.

Behavioural spec: ``internal/grpc/audio_service.go`` - ``StreamAudio`` (:926-1043),
``startArbitrationWindow`` / ``joinArbitrationWindow`` / ``performArbitration``
(:408-587), ``calculateSignalStrength`` (RMS, :818-852), ``bytesToFloat32Array``
(PCM16-LE / 32767, odd trailing byte dropped, :1048-1101),
``sendCancellationResponse`` (:855-877), ``isRelayActive`` (:880-913),
``cleanupRelay`` (:916-923), success/error responses (:693-815).

Redesign (SURVEY §3.7 defects #1-#4):
* the arbitration state is owned by the asyncio event loop (single-threaded
  actor) - no mutexes, so no ABBA lock-order hazard and no unlocked reads;
* windows are keyed by ``ARBITRATION_SCOPE``: ``global`` (reference behaviour:
  one window for all relays) or ``per_relay_group`` (relays of one room
  collide, different rooms proceed concurrently - needed for 64 concurrent
  streams);
* the winner's audio is taken at end-of-speech (bounded by the 5 s wait), not
  snapshotted at window close; the response is delivered on NATS
  ``audio.<relay>`` as before AND sent on the gRPC stream (additive);
  ``confirmation_needed`` is emitted when enabled and STT confidence is low;
* every processed utterance writes a voice event.
"""
from __future__ import annotations

import asyncio
import enum
import logging
import time
import uuid
from dataclasses import dataclass, field
from typing import Protocol

import numpy as np

from ..events import VoiceEvent
from ..utils import logging as hublog
from .audio_proto import AudioResponse

log = logging.getLogger("loqa.audio")

MSG_CANCELLED = "Another relay is handling this request."
MSG_STT_FAILED = "Sorry, I couldn't hear you clearly. Please try again."
MSG_NO_SPEECH = "I didn't hear anything. Please try again."
MSG_PARSE_FAILED = "Sorry, I couldn't understand that command."
MSG_NO_COMMANDS = "I'm not sure how to help with that."


class RelayStatus(enum.IntEnum):
    CONNECTED = 0
    CONTENDING = 1
    WINNER = 2
    CANCELLED = 3


@dataclass
class RelayStream:
    relay_id: str
    stream: object = None                 # object with ``async write(AudioResponse)``
    connected_at: float = field(default_factory=time.monotonic)
    signal_strength: float = 0.0
    status: RelayStatus = RelayStatus.CONNECTED
    cancel: asyncio.Event = field(default_factory=asyncio.Event)
    end_of_speech: asyncio.Event = field(default_factory=asyncio.Event)
    result: asyncio.Future | None = None
    request_id: str = ""
    # the relay's raw PCM16-LE samples as received (odd trailing bytes
    # dropped per chunk, as audio_service.go:1048-1101): the wake word for the
    # RMS arbitration, and wake word + speech for the processor - in a pinned
    # stager slot on the GPU path (appended as each chunk arrives), otherwise on
    # the host
    wake_pcm: bytearray = field(default_factory=bytearray)
    pcm: bytearray = field(default_factory=bytearray)
    pcm_slot: object = None
    n_samples: int = 0

    def add_pcm(self, data: bytes) -> None:
        data = data[: len(data) & ~1]
        if self.pcm_slot is not None:
            self.pcm_slot.append(data)
        else:
            self.pcm += data
        self.n_samples += len(data) // 2

    @property
    def wake_word_signal(self) -> np.ndarray:
        """Float samples of the wake word (x / 32767)."""
        return bytes_to_float32_array(bytes(self.wake_pcm))

    def full_audio(self) -> np.ndarray:
        """Float samples of wake word + speech (host-buffered relays only)."""
        return bytes_to_float32_array(bytes(self.pcm))

    def full_pcm16(self) -> np.ndarray:
        return np.frombuffer(bytes(self.pcm), dtype="<i2")

    def release_pcm(self) -> None:
        if self.pcm_slot is not None:
            self.pcm_slot.release()
            self.pcm_slot = None


@dataclass
class ArbitrationWindow:
    key: str
    start_time: float
    window_duration: float
    relays: dict[str, RelayStream] = field(default_factory=dict)
    is_active: bool = True
    winner_id: str = ""
    closed: asyncio.Event = field(default_factory=asyncio.Event)


@dataclass
class UtteranceResult:
    transcription: str = ""
    response_text: str = ""
    success: bool = True
    command: str = "voice_command_success"
    intents: list[str] = field(default_factory=list)
    audio: bytes = b""
    audio_format: str = ""
    audio_duration: float = 0.0
    confidence: float = 0.0
    entities: dict[str, str] = field(default_factory=dict)
    error: str = ""
    audio_sample_rate: int = 0        # 0: the reference's guess (16 kHz, mp3 22.05 kHz)
    audio_published: bool = False     # progressive speech already sent every phrase on NATS
    strategy: str = ""                # streaming-predictive bridge strategy
    metrics: dict = field(default_factory=dict)


class VoiceProcessor(Protocol):
    async def process(self, relay_id: str, request_id: str, audio: np.ndarray,
                      sample_rate: int) -> UtteranceResult: ...


def bytes_to_float32_array(data: bytes) -> np.ndarray:
    if not data:
        return np.zeros(0, np.float32)
    n = len(data) // 2  # odd trailing byte dropped
    return np.frombuffer(data[: 2 * n], dtype="<i2").astype(np.float32) / np.float32(32767.0)


def calculate_signal_strength(samples: np.ndarray) -> float:
    if samples.size == 0:
        return 0.0
    s = samples.astype(np.float32)
    return float(np.sqrt(np.sum((s * s).astype(np.float64)) / s.size))


def pcm16_signal_strength(data: bytes) -> float:
    """RMS of PCM16-LE bytes in the reference's float scale (x / 32767,
    ``calculateSignalStrength`` :818-852) straight from the integers."""
    n = len(data) // 2
    if n == 0:
        return 0.0
    x = np.frombuffer(data[: 2 * n], dtype="<i2").astype(np.int64)
    return float(np.sqrt(float(np.dot(x, x)) / n)) / 32767.0


class AudioService:
    def __init__(self, processor: VoiceProcessor | None = None, *, window_duration: float = 0.300,
                 scope: str = "global", relay_groups: dict[str, str] | None = None,
                 end_of_speech_wait: float = 5.0, result_timeout: float = 30.0,
                 events_store=None, audio_publisher=None, confirmation_enabled: bool = False,
                 transcript_hints=None, single_relay_bypass: bool = False):
        self.processor = processor
        self.arbitration_window_duration = window_duration
        self.scope = scope
        self.relay_groups = relay_groups or {}
        self.end_of_speech_wait = end_of_speech_wait
        self.result_timeout = result_timeout
        self.events_store = events_store
        self.audio_publisher = audio_publisher
        self.confirmation_enabled = confirmation_enabled
        # synthetic load only (bench --mode hub, tests): relay id -> the
        # utterance's known transcript, which teacher-forces the random-init
        # Whisper decoder; real relays never have one
        self.transcript_hints = transcript_hints
        # opt-in: a relay alone in its (static) group skips the window
        # (docs/COLLISION_DETECTION.md:203 of the reference; ArbitrationConfig)
        self.single_relay_bypass = single_relay_bypass and scope == "per_relay_group"
        self._group_size: dict[str, int] = {}
        for g in self.relay_groups.values():
            self._group_size[g] = self._group_size.get(g, 0) + 1
        self.windows: dict[str, ArbitrationWindow] = {}
        self.active_streams: dict[str, RelayStream] = {}
        self.stats = {"windows": 0, "arbitrations": 0, "cancelled": 0, "processed": 0, "late": 0,
                      "bypassed": 0}

    # ------------------------------------------------------------ windows
    def window_key(self, relay_id: str) -> str:
        if self.scope == "global":
            return "global"
        return self.relay_groups.get(relay_id, relay_id)

    def can_collide(self, relay_id: str) -> bool:
        """Whether another relay could join ``relay_id``'s window: always in the
        global scope; per group, unless the static group map leaves the
        relay's group with no other member (an unmapped relay is its own
        group unless some relay is mapped to a group of that name)."""
        if self.scope == "global":
            return True
        key = self.window_key(relay_id)
        members = self._group_size.get(key, 0) + (0 if relay_id in self.relay_groups else 1)
        return members > 1

    @property
    def arbitration_window(self) -> ArbitrationWindow | None:
        """The global window (reference field name); None when idle."""
        if self.scope == "global":
            return self.windows.get("global")
        return next(iter(self.windows.values()), None)

    def start_arbitration_window(self, relay_id: str, stream=None) -> ArbitrationWindow:
        key = self.window_key(relay_id)
        w = ArbitrationWindow(key, time.monotonic(), self.arbitration_window_duration)
        rs = RelayStream(relay_id, stream, status=RelayStatus.CONTENDING)
        w.relays[relay_id] = rs
        self.active_streams[relay_id] = rs
        self.windows[key] = w
        self.stats["windows"] += 1
        if self.single_relay_bypass and not self.can_collide(relay_id):
            # nobody can join this window: decide now (the relay wins before
            # its next chunk is read)
            self.stats["bypassed"] += 1
            hublog.log_audio_processing(relay_id, "arbitration_bypassed", reason="single_relay_group")
            self.perform_arbitration(w)
            return w
        hublog.log_audio_processing(relay_id, "arbitration_window_started",
                                    window_duration_ms=w.window_duration * 1e3, first_relay=relay_id)
        asyncio.get_running_loop().call_later(w.window_duration, self._close_window, w)
        return w

    def join_arbitration_window(self, relay_id: str, stream=None) -> bool:
        w = self.windows.get(self.window_key(relay_id))
        if w is None or not w.is_active:
            return False
        elapsed = time.monotonic() - w.start_time
        if elapsed > w.window_duration:
            return False
        rs = w.relays.get(relay_id)
        if rs is None:
            rs = RelayStream(relay_id, stream, status=RelayStatus.CONTENDING)
            w.relays[relay_id] = rs
            self.active_streams[relay_id] = rs
        hublog.log_audio_processing(relay_id, "arbitration_window_joined", elapsed_ms=elapsed * 1e3,
                                    relay_count=len(w.relays))
        return True

    def _close_window(self, w: ArbitrationWindow) -> None:
        self.perform_arbitration(w)

    def perform_arbitration(self, w: ArbitrationWindow) -> None:
        if not w.is_active:
            return
        self.stats["arbitrations"] += 1
        winner, best = "", 0.0
        for rid, rs in w.relays.items():
            if rs.status != RelayStatus.CONTENDING:
                continue
            rs.signal_strength = pcm16_signal_strength(bytes(rs.wake_pcm))
            hublog.log_audio_processing(rid, "arbitration_signal_analysis",
                                        signal_strength=rs.signal_strength,
                                        samples=len(rs.wake_pcm) // 2)
            if rs.signal_strength > best:
                best, winner = rs.signal_strength, rid
        if winner == "" and w.relays:
            winner = next(iter(w.relays))
        w.winner_id = winner
        w.is_active = False
        for rid, rs in w.relays.items():
            if rid == winner:
                rs.status = RelayStatus.WINNER
                hublog.log_audio_processing(rid, "arbitration_winner", signal_strength=rs.signal_strength,
                                            competing_relays=len(w.relays))
            else:
                rs.status = RelayStatus.CANCELLED
                rs.cancel.set()
                rs.release_pcm()
                self.stats["cancelled"] += 1
                hublog.log_audio_processing(rid, "arbitration_cancelled",
                                            signal_strength=rs.signal_strength, winner=winner)
                asyncio.ensure_future(self.send_cancellation_response(rs))
        if winner:
            rs = w.relays[winner]
            rs.result = asyncio.ensure_future(self._process_winner(rs))
        if self.windows.get(w.key) is w:
            del self.windows[w.key]
        w.closed.set()

    async def send_cancellation_response(self, rs: RelayStream) -> None:
        if rs.stream is None:
            hublog.log_audio_processing(rs.relay_id, "cancellation_skipped", reason="nil_stream")
            return
        try:
            await rs.stream.write(AudioResponse(request_id=rs.relay_id, transcription="",
                                                command="relay_cancelled", response_text=MSG_CANCELLED,
                                                success=False))
        except Exception as e:
            hublog.log_error(e, "failed to send cancellation response", relay_id=rs.relay_id)

    def is_relay_active(self, relay_id: str) -> bool:
        rs = self.active_streams.get(relay_id)
        if rs is None:
            return False
        return rs.status in (RelayStatus.WINNER, RelayStatus.CONNECTED, RelayStatus.CONTENDING)

    def cleanup_relay(self, relay_id: str) -> None:
        rs = self.active_streams.pop(relay_id, None)
        if rs is not None and rs.result is None:
            rs.release_pcm()          # never processed: give the pinned slot back

    # ------------------------------------------------------------ processing
    async def _process_winner(self, rs: RelayStream) -> UtteranceResult:
        # a new command from this relay interrupts the reply it may still be
        # receiving (progressive speech; streaming_interrupt_handler.go:69-119)
        interrupt = getattr(self.processor, "interrupt_relay", None)
        if interrupt is not None:
            try:
                if interrupt(rs.relay_id):
                    self.stats["interrupted"] = self.stats.get("interrupted", 0) + 1
            except Exception as e:  # noqa: BLE001
                hublog.log_warn("reply interrupt failed", relay_id=rs.relay_id, error=str(e))
        # collect speech until end-of-speech (bounded), instead of the reference's
        # snapshot at window close
        try:
            await asyncio.wait_for(rs.end_of_speech.wait(), self.end_of_speech_wait)
        except asyncio.TimeoutError:
            pass
        request_id = rs.request_id or f"req_{time.time_ns()}"
        ev = VoiceEvent.new(rs.relay_id, request_id)
        ev.set_audio_metadata(rs.n_samples, 16000, True)
        if rs.n_samples == 0:
            rs.release_pcm()
            hublog.log_warn("winner has no audio", relay_id=rs.relay_id)
            res = UtteranceResult(success=False, command="error", response_text=MSG_NO_SPEECH)
        elif self.processor is None:
            rs.release_pcm()
            res = UtteranceResult(success=False, command="error", response_text=MSG_STT_FAILED,
                                  error="no voice processor configured")
        else:
            kw = {}
            if getattr(self.processor, "takes_pcm16", False):
                # GPU path: the samples go as PCM16 - the pinned slot itself
                # (ownership passes to the processor) or the host bytes
                audio = np.zeros(0, np.float32)
                if rs.pcm_slot is not None:
                    kw["pcm_slot"], rs.pcm_slot = rs.pcm_slot, None
                else:
                    kw["pcm16"] = rs.full_pcm16()
            else:
                audio = rs.full_audio()
            hint = self.transcript_hints(rs.relay_id) if self.transcript_hints else None
            if hint:
                kw["transcript_hint"] = hint
            try:
                res = await self.processor.process(rs.relay_id, request_id, audio, 16000, **kw)
            except Exception as e:  # processor failure -> spoken error
                log.exception("voice processing failed for relay %s", rs.relay_id)
                res = UtteranceResult(success=False, command="error", response_text=MSG_STT_FAILED,
                                      error=str(e))
        self.stats["processed"] += 1
        await self._deliver_audio(rs.relay_id, res)
        ev.set_transcription(res.transcription)
        ev.set_command_result(res.intents[0] if res.intents else "unknown", res.entities,
                              min(1.0, max(0.0, res.confidence)))
        if res.success:
            ev.set_response(res.response_text)
        else:
            ev.response_text = res.response_text
            ev.set_error(res.error or res.response_text)
        if self.events_store is not None:
            try:
                await asyncio.to_thread(self.events_store.insert, ev)
            except Exception as e:
                hublog.log_error(e, "failed to store voice event", relay_id=rs.relay_id)
        return res

    async def _deliver_audio(self, relay_id: str, res: UtteranceResult) -> None:
        if not res.audio or res.audio_published:
            return
        if self.audio_publisher is None:
            log.warning("NATS audio publisher not available, skipping response to relay %s", relay_id)
            return
        sr = res.audio_sample_rate or (22050 if res.audio_format == "mp3" else 16000)
        try:
            await self.audio_publisher.stream_audio_to_relay(
                relay_id, res.audio, res.audio_format, sr,
                "response" if res.success else "error", 3 if res.success else 4)
        except Exception as e:
            hublog.log_warn("failed to stream audio to relay", relay_id=relay_id, error=str(e))

    def _response_for(self, res: UtteranceResult) -> AudioResponse:
        cmd = res.command
        if self.confirmation_enabled and res.command == "confirmation_needed":
            cmd = "confirmation_needed"
        return AudioResponse(request_id="", transcription=res.transcription, command=cmd,
                             response_text=res.response_text, success=res.success,
                             response_audio=res.audio, audio_format=res.audio_format,
                             audio_duration=res.audio_duration)

    # ---------------------------------------------------------------- gRPC
    async def StreamAudio(self, request_iterator, context):  # noqa: N802 (gRPC method name)
        """Handler for the bidirectional stream. ``context`` must provide
        ``async write(AudioResponse)`` (grpc.aio ServicerContext or a test double)."""
        relay_id = ""
        request_id = f"req_{uuid.uuid4().hex[:12]}"
        stream = _ContextWriter(context)
        try:
            async for chunk in request_iterator:
                if not relay_id:
                    relay_id = chunk.relay_id
                # per-chunk line at DEBUG (the reference logs it at info through
                # zap, ~1 us; a Python JSON record costs ~30 us, 5-6k chunks/s at
                # 64 relays: docs/PERF.md "Round 5", front end); the wake word and
                # end of speech keep their info lines
                if hublog.debug_enabled():
                    hublog.log_audio_processing_debug(relay_id, "received",
                                                      bytes=len(chunk.audio_data),
                                                      wake_word=chunk.is_wake_word)
                data = chunk.audio_data
                if chunk.is_wake_word:
                    key = self.window_key(relay_id)
                    w = self.windows.get(key)
                    if w is None:
                        w = self.start_arbitration_window(relay_id, stream)
                    elif not self.join_arbitration_window(relay_id, stream):
                        log.info("relay %s attempted connection after arbitration window closed", relay_id)
                        self.stats["late"] += 1
                        return
                    rs = self.active_streams.get(relay_id)
                    if rs is not None:
                        self._attach_pcm(rs)
                        rs.wake_pcm += data[: len(data) & ~1]
                        rs.add_pcm(data)
                        rs.request_id = request_id
                else:
                    rs = self.active_streams.get(relay_id)
                    if rs is not None and rs.status != RelayStatus.CANCELLED:
                        rs.add_pcm(data)
                if chunk.is_end_of_speech:
                    hublog.log_audio_processing(relay_id, "end_of_speech_detected")
                    if not self.is_relay_active(relay_id):
                        hublog.log_audio_processing(relay_id, "relay_cancelled_before_processing")
                        return
                    rs = self.active_streams.get(relay_id)
                    if rs is None:
                        return
                    rs.end_of_speech.set()
                    await self._await_result(rs, stream)
                    return
        finally:
            if relay_id:
                self.cleanup_relay(relay_id)

    def _attach_pcm(self, rs: RelayStream) -> None:
        """GPU processors hand out a pinned stager slot per relay: its chunks
        are appended there as they arrive (no host conversion)."""
        if rs.pcm_slot is None and rs.n_samples == 0:
            new_slot = getattr(self.processor, "new_pcm_slot", None)
            if new_slot is not None:
                rs.pcm_slot = new_slot()

    async def _await_result(self, rs: RelayStream, stream: "_ContextWriter") -> None:
        if rs.status == RelayStatus.CONTENDING:
            # the window's decision (the reference polls 50 x 100 ms, :1008-1041)
            w = self.windows.get(self.window_key(rs.relay_id))
            if w is not None and rs.relay_id in w.relays:
                try:
                    await asyncio.wait_for(w.closed.wait(), self.end_of_speech_wait)
                except asyncio.TimeoutError:
                    pass
            deadline = time.monotonic() + self.end_of_speech_wait
            while rs.status == RelayStatus.CONTENDING and time.monotonic() < deadline:
                await asyncio.sleep(0.005)
        if rs.status != RelayStatus.WINNER or rs.result is None:
            return
        try:
            res = await asyncio.wait_for(asyncio.shield(rs.result), self.result_timeout)
        except asyncio.TimeoutError:
            return
        try:
            await stream.write(self._response_for(res))
        except Exception as e:
            hublog.log_warn("failed to send response on stream", relay_id=rs.relay_id, error=str(e))


class _ContextWriter:
    """Serialises writes from the handler and from arbitration tasks."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.lock = asyncio.Lock()

    async def write(self, msg) -> None:
        async with self.lock:
            await self.ctx.write(msg)
