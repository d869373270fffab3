"""Voice-event domain object (``internal/events/voice_event.go``).

Every utterance that reaches the pipeline produces one event; unlike the
reference (where only ``POST /api/voice-events`` writes them) the
audio path records them too. JSON field names/shape match the Go struct tags
(``voice_event.go:30-53``) so API clients see the same documents.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass, field
from datetime import datetime, timezone


def generate_uuid() -> str:
    """Random (v4) UUID in the reference's hex-group format; ``loqa-<nanos>``
    fallback if the OS RNG fails (voice_event.go:68-81)."""
    try:
        b = bytearray(os.urandom(16))
    except NotImplementedError:
        return f"loqa-{time.time_ns()}"
    b[6] = (b[6] & 0x0F) | 0x40
    b[8] = (b[8] & 0x3F) | 0x80
    h = b.hex()
    return f"{h[0:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:32]}"


def rfc3339(dt: datetime) -> str:
    """Go RFC3339Nano rendering (fraction with trailing zeros trimmed)."""
    s = dt.isoformat(timespec="microseconds")
    main, frac_tz = s.split(".", 1) if "." in s else (s, "")
    if frac_tz:
        frac, tz = frac_tz[:6], frac_tz[6:]
        frac = frac.rstrip("0")
        s = main + ("." + frac if frac else "") + tz
    return s.replace("+00:00", "Z")


def parse_rfc3339(s: str) -> datetime:
    s = s.strip().replace("Z", "+00:00")
    if "." in s:  # trim nanoseconds to micro
        head, rest = s.split(".", 1)
        digits = ""
        i = 0
        while i < len(rest) and rest[i].isdigit():
            digits += rest[i]
            i += 1
        s = head + "." + (digits[:6].ljust(6, "0")) + rest[i:]
    dt = datetime.fromisoformat(s)
    if dt.tzinfo is None:
        raise ValueError("RFC3339 time needs a zone")
    return dt


@dataclass
class VoiceEvent:
    uuid: str = ""
    request_id: str = ""
    relay_id: str = ""
    timestamp: datetime = field(default_factory=lambda: datetime.now(timezone.utc))
    audio_duration: float = 0.0
    sample_rate: int = 0
    wake_word_detected: bool = False
    transcription: str = ""
    intent: str = ""
    entities: dict[str, str] = field(default_factory=dict)
    confidence: float = 0.0
    response_text: str = ""
    processing_time_ms: int = 0
    success: bool = True
    error_message: str = ""
    _t0: float = field(default=0.0, repr=False, compare=False)

    @staticmethod
    def new(relay_id: str, request_id: str) -> "VoiceEvent":
        ev = VoiceEvent(uuid=generate_uuid(), request_id=request_id, relay_id=relay_id)
        ev._t0 = time.monotonic()
        return ev

    def _elapsed_ms(self) -> int:
        if self._t0:
            return int((time.monotonic() - self._t0) * 1000)
        return max(0, int((datetime.now(timezone.utc) - self.timestamp).total_seconds() * 1000))

    def set_audio_metadata(self, n_samples: int, sample_rate: int, is_wake_word: bool) -> None:
        self.audio_duration = n_samples / sample_rate if sample_rate else 0.0
        self.sample_rate = sample_rate
        self.wake_word_detected = is_wake_word

    def set_transcription(self, t: str) -> None:
        self.transcription = t

    def set_command_result(self, intent: str, entities: dict[str, str] | None, confidence: float) -> None:
        self.intent = intent
        self.entities = entities if entities is not None else {}
        self.confidence = confidence

    def set_response(self, text: str) -> None:
        self.response_text = text
        self.processing_time_ms = self._elapsed_ms()

    def set_error(self, err) -> None:
        self.success = False
        self.error_message = str(err)
        self.processing_time_ms = self._elapsed_ms()

    def entities_json(self) -> str:
        if not self.entities:
            return "{}"
        return json.dumps(self.entities, separators=(",", ":"), sort_keys=True)

    def set_entities_from_json(self, s: str) -> None:
        if s in ("", "{}"):
            self.entities = {}
            return
        try:
            d = json.loads(s)
        except json.JSONDecodeError as e:
            raise ValueError(f"failed to unmarshal entities JSON: {e}") from e
        if not isinstance(d, dict) or not all(isinstance(v, str) for v in d.values()):
            raise ValueError("failed to unmarshal entities JSON: not a string map")
        self.entities = d

    def is_valid(self) -> None:
        if not self.uuid:
            raise ValueError("UUID is required")
        if not self.relay_id:
            raise ValueError("relayID is required")
        if not self.request_id:
            raise ValueError("requestID is required")
        if self.timestamp is None:
            raise ValueError("timestamp is required")
        if self.confidence < 0 or self.confidence > 1:
            raise ValueError("confidence must be between 0 and 1")

    def to_dict(self) -> dict:
        d = {
            "uuid": self.uuid, "request_id": self.request_id, "relay_id": self.relay_id,
            "timestamp": rfc3339(self.timestamp), "audio_duration": self.audio_duration,
            "sample_rate": self.sample_rate, "wake_word_detected": self.wake_word_detected,
            "transcription": self.transcription, "intent": self.intent,
            "entities": self.entities, "confidence": self.confidence,
            "response_text": self.response_text, "processing_time_ms": self.processing_time_ms,
            "success": self.success,
        }
        if self.error_message:
            d["error_message"] = self.error_message
        return d

    def __str__(self) -> str:
        return (f"VoiceEvent{{UUID: {self.uuid}, RelayID: {self.relay_id}, Intent: {self.intent}, "
                f"Transcription: {json.dumps(self.transcription)}, Confidence: {self.confidence:.2f}, "
                f"Success: {str(self.success).lower()}}}")
