"""Response-audio delivery to relays over NATS.

Wire format identical to ``internal/messaging/audio_stream_publisher.go:33-40``:
one JSON message per audio file on ``audio.<relay_id>`` (or ``audio.broadcast``)
with base64 ``audio_data``; stream id ``<uuid[:8]>-<unix nanos>``
(``broadcast-`` prefixed for broadcasts). Progressive TTS publishes one such
message per synthesized phrase.
"""
from __future__ import annotations

import logging
import time
import uuid

from ..utils import gojson
from .nats_client import NATSClient

log = logging.getLogger("loqa.messaging.audio")


def audio_message(stream_id: str, audio: bytes, fmt: str, sample_rate: int, message_type: str,
                  priority: int) -> bytes:
    return gojson.dumps(gojson.GoStruct(
        ("stream_id", stream_id), ("audio_data", bytes(audio)), ("audio_format", fmt),
        ("sample_rate", int(sample_rate)), ("message_type", message_type),
        ("priority", int(priority)))).encode()


class AudioStreamPublisher:
    def __init__(self, conn: NATSClient, chunk_size: int = 4096):
        self.conn = conn
        self.chunk_size = chunk_size
        self.max_streams = 50
        self.timeout = 5.0

    async def stream_audio_to_relay(self, relay_id: str, audio: bytes, audio_format: str,
                                    sample_rate: int, message_type: str, priority: int) -> str:
        sid = f"{uuid.uuid4().hex[:8]}-{time.time_ns()}"
        topic = f"audio.{relay_id}"
        await self.conn.publish(topic, audio_message(sid, audio, audio_format, sample_rate,
                                                     message_type, priority))
        log.info("published complete audio file to %s (%d bytes)", topic, len(audio))
        return sid

    async def broadcast_audio_to_all_relays(self, audio: bytes, audio_format: str, sample_rate: int,
                                            message_type: str, priority: int) -> str:
        sid = f"broadcast-{uuid.uuid4().hex[:8]}-{time.time_ns()}"
        await self.conn.publish("audio.broadcast", audio_message(sid, audio, audio_format,
                                                                 sample_rate, message_type, priority))
        return sid
