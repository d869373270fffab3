"""Hub event bus on NATS - subjects and JSON payloads byte-compatible with the
reference (``internal/messaging/nats_service.go``: event types :38-65, subjects
:68-73, publish/subscribe :118-236). The URL comes from the single config
object (env ``NATS_URL``), fixing the reference's config bypass.
"""
from __future__ import annotations

import json
import logging
import time
from dataclasses import dataclass, field

from ..utils import gojson
from ..utils.faults import faults
from .nats_client import Msg, NATSClient, NATSError

log = logging.getLogger("loqa.messaging")

SUBJECT_VOICE_COMMANDS = "loqa.voice.commands"
SUBJECT_DEVICE_COMMANDS = "loqa.devices.commands"
SUBJECT_DEVICE_RESPONSES = "loqa.devices.responses"
SUBJECT_SYSTEM_EVENTS = "loqa.system.events"


@dataclass
class CommandEvent:
    relay_id: str = ""
    transcription: str = ""
    intent: str = ""
    entities: dict[str, str] = field(default_factory=dict)
    confidence: float = 0.0
    timestamp: int = 0  # unix nanoseconds
    request_id: str = ""

    def _fields(self) -> list[tuple[str, object]]:
        return [("relay_id", self.relay_id), ("transcription", self.transcription),
                ("intent", self.intent), ("entities", self.entities if self.entities is not None else None),
                ("confidence", float(self.confidence)), ("timestamp", int(self.timestamp)),
                ("request_id", self.request_id)]

    def to_json(self) -> bytes:
        return gojson.dumps(gojson.GoStruct(*self._fields())).encode()

    @classmethod
    def from_json(cls, data: bytes) -> "CommandEvent":
        d = json.loads(data)
        return cls(d.get("relay_id", ""), d.get("transcription", ""), d.get("intent", ""),
                   d.get("entities") or {}, float(d.get("confidence", 0.0)), int(d.get("timestamp", 0)),
                   d.get("request_id", ""))


@dataclass
class DeviceCommandEvent(CommandEvent):
    device_type: str = ""
    device_id: str = ""
    location: str = ""
    action: str = ""

    def to_json(self) -> bytes:
        f = self._fields() + [("device_type", self.device_type)]
        if self.device_id:
            f.append(("device_id", self.device_id))
        if self.location:
            f.append(("location", self.location))
        f.append(("action", self.action))
        return gojson.dumps(gojson.GoStruct(*f)).encode()

    @classmethod
    def from_json(cls, data: bytes) -> "DeviceCommandEvent":
        d = json.loads(data)
        return cls(d.get("relay_id", ""), d.get("transcription", ""), d.get("intent", ""),
                   d.get("entities") or {}, float(d.get("confidence", 0.0)), int(d.get("timestamp", 0)),
                   d.get("request_id", ""), d.get("device_type", ""), d.get("device_id", ""),
                   d.get("location", ""), d.get("action", ""))


@dataclass
class DeviceResponseEvent:
    request_id: str = ""
    device_type: str = ""
    device_id: str = ""
    success: bool = False
    message: str = ""
    timestamp: int = 0

    def to_json(self) -> bytes:
        f = [("request_id", self.request_id), ("device_type", self.device_type)]
        if self.device_id:
            f.append(("device_id", self.device_id))
        f += [("success", self.success), ("message", self.message), ("timestamp", int(self.timestamp))]
        return gojson.dumps(gojson.GoStruct(*f)).encode()

    @classmethod
    def from_json(cls, data: bytes) -> "DeviceResponseEvent":
        d = json.loads(data)
        return cls(d.get("request_id", ""), d.get("device_type", ""), d.get("device_id", ""),
                   bool(d.get("success", False)), d.get("message", ""), int(d.get("timestamp", 0)))


class NATSService:
    def __init__(self, url: str = "nats://localhost:4222", reconnect_wait: float = 2.0):
        self.url = url
        self.reconnect_wait = reconnect_wait
        self.conn: NATSClient | None = None

    async def connect(self) -> None:
        log.info("connecting to NATS at %s", self.url)
        c = NATSClient(name="loqa-hub", reconnect_wait=self.reconnect_wait, max_reconnects=-1,
                       on_disconnect=lambda _c: log.warning("NATS disconnected"),
                       on_reconnect=lambda _c: log.info("NATS reconnected to %s", self.url),
                       on_closed=lambda _c: log.info("NATS connection closed"))
        await c.connect(self.url)
        self.conn = c
        log.info("connected to NATS server at %s", self.url)

    def is_connected(self) -> bool:
        return self.conn is not None and self.conn.is_connected()

    def _require(self) -> NATSClient:
        if faults().active("nats_down"):
            raise NATSError("NATS connection not established (injected fault: nats_down)")
        if self.conn is None:
            raise NATSError("NATS connection not established")
        return self.conn

    async def publish_voice_command(self, ev: CommandEvent) -> None:
        await self._require().publish(SUBJECT_VOICE_COMMANDS, ev.to_json())
        log.info("published voice command to NATS - intent: %s, relay: %s", ev.intent, ev.relay_id)

    async def publish_device_command(self, ev: DeviceCommandEvent) -> None:
        subj = f"{SUBJECT_DEVICE_COMMANDS}.{ev.device_type}"
        await self._require().publish(subj, ev.to_json())
        log.info("published device command to NATS - device: %s, action: %s", ev.device_type, ev.action)

    async def publish_device_response(self, ev: DeviceResponseEvent) -> None:
        await self._require().publish(SUBJECT_DEVICE_RESPONSES, ev.to_json())

    async def subscribe_voice_commands(self, handler) -> int:
        def cb(m: Msg):
            try:
                ev = CommandEvent.from_json(m.data)
            except ValueError as e:
                log.warning("error unmarshaling voice command: %s", e)
                return None
            return handler(ev)
        return await self._require().subscribe(SUBJECT_VOICE_COMMANDS, cb)

    async def subscribe_device_commands(self, device_type: str, handler) -> int:
        def cb(m: Msg):
            try:
                ev = DeviceCommandEvent.from_json(m.data)
            except ValueError as e:
                log.warning("error unmarshaling device command: %s", e)
                return None
            return handler(ev)
        return await self._require().subscribe(f"{SUBJECT_DEVICE_COMMANDS}.{device_type}", cb)

    async def subscribe_device_responses(self, handler) -> int:
        def cb(m: Msg):
            try:
                ev = DeviceResponseEvent.from_json(m.data)
            except ValueError as e:
                log.warning("error unmarshaling device response: %s", e)
                return None
            return handler(ev)
        return await self._require().subscribe(SUBJECT_DEVICE_RESPONSES, cb)

    def stats(self):
        return self.conn.stats if self.conn else None

    async def close(self) -> None:
        if self.conn:
            await self.conn.close()


def now_ns() -> int:
    return time.time_ns()
