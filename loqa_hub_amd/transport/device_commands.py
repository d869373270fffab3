"""Command execution = publish on the NATS event bus.

Behaviour of ``AudioService.ExecuteCommand`` and its helpers
(``internal/grpc/audio_service.go:109-156``, ``:1104-1175``): every command is
published to ``loqa.voice.commands``; device intents additionally go to
``loqa.devices.commands.<device_type>`` with the mapped action (a failure there
is logged, not fatal).
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass

from ..llm.commands import Command
from ..messaging.nats_service import CommandEvent, DeviceCommandEvent, NATSService

log = logging.getLogger("loqa.executor")

_DEVICE_INTENTS = {"turn_on", "turn_off", "dim", "brighten", "play", "stop", "pause", "volume"}
_ACTIONS = {"turn_on": "on", "turn_off": "off", "dim": "dim", "brighten": "brighten",
            "play": "play", "stop": "stop", "pause": "pause", "volume": "volume"}
_DEVICE_TYPES = {"lights": "lights", "light": "lights", "lamp": "lights", "music": "audio",
                 "audio": "audio", "sound": "audio", "tv": "tv", "television": "tv"}


def is_device_command(intent: str) -> bool:
    return intent in _DEVICE_INTENTS


def map_intent_to_action(intent: str) -> str:
    return _ACTIONS.get(intent, "")


def extract_device_type(entities: dict[str, str]) -> str:
    if "device" in entities:
        dev = entities["device"]
        return _DEVICE_TYPES.get(dev, dev)
    return ""


def create_device_command(ev: CommandEvent) -> DeviceCommandEvent | None:
    dtype = extract_device_type(ev.entities) or "lights"
    action = map_intent_to_action(ev.intent)
    if not action:
        return None
    return DeviceCommandEvent(ev.relay_id, ev.transcription, ev.intent, ev.entities, ev.confidence,
                              ev.timestamp, ev.request_id, device_type=dtype,
                              device_id=ev.entities.get("device_id", ""),
                              location=ev.entities.get("location", ""), action=action)


@dataclass
class ExecutionContext:
    relay_id: str = "multi-cmd"
    request_id: str = "multi-cmd"
    event_uuid: str = ""
    transcription: str = ""


class NATSCommandExecutor:
    """``llm.CommandExecutor`` that publishes commands (the reference's
    AudioService-as-executor). The execution context is per-utterance (the
    reference keeps one mutable field on the service, a race across relays)."""

    def __init__(self, nats: NATSService | None, ctx: ExecutionContext | None = None):
        self.nats = nats
        self.ctx = ctx

    async def execute_command(self, cmd: Command) -> None:
        if self.nats is None or not self.nats.is_connected():
            raise RuntimeError("NATS service not available")
        ctx = self.ctx
        ev = CommandEvent(relay_id=ctx.relay_id if ctx else "multi-cmd",
                          transcription=ctx.transcription if ctx else cmd.response,
                          intent=cmd.intent, entities=cmd.entities, confidence=cmd.confidence,
                          timestamp=time.time_ns(),
                          request_id=ctx.request_id if ctx else "multi-cmd")
        await self.nats.publish_voice_command(ev)
        if is_device_command(cmd.intent):
            dc = create_device_command(ev)
            if dc is not None:
                try:
                    await self.nats.publish_device_command(dc)
                except Exception as e:  # not fatal (audio_service.go:145-153)
                    log.warning("failed to publish device command for %s: %s", cmd.intent, e)
