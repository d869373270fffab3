"""Builtin lighting skill (``internal/skills/builtin/lights_skill.go``).

Keyword ``can_handle`` on the transcript (:72-90); action on/off/dim/brighten/
toggle and location kitchen/living_room/bedroom/bathroom/all/main parsed from
the transcript (:133-169); the action itself is simulated (:172-195); the
manifest and config schema match :198-287 field for field.
"""
from __future__ import annotations

from datetime import datetime, timezone

from ..interfaces import (ConfigProperty, ConfigSchema, IntentPattern, Permission,
                          PermissionType, SandboxMode, SkillAction, SkillConfig, SkillManifest,
                          SkillPlugin, SkillResponse, SkillState, SkillStatus, TrustLevel,
                          VoiceIntent)

KEYWORDS = ("light", "lights", "lighting", "turn on", "turn off", "switch on", "switch off",
            "dim", "brighten", "bright", "dark", "lamp", "lamps")


def parse_lighting(transcript: str) -> tuple[str, str]:
    t = transcript.lower()
    if "turn on" in t or "switch on" in t:
        action = "on"
    elif "turn off" in t or "switch off" in t:
        action = "off"
    elif "dim" in t or "lower" in t:
        action = "dim"
    elif "brighten" in t or "bright" in t:
        action = "brighten"
    else:
        action = "toggle"
    if "kitchen" in t:
        loc = "kitchen"
    elif "living room" in t or "lounge" in t:
        loc = "living_room"
    elif "bedroom" in t:
        loc = "bedroom"
    elif "bathroom" in t:
        loc = "bathroom"
    elif "all" in t or "everywhere" in t:
        loc = "all"
    else:
        loc = "main"
    return action, loc


_VERBS = {"on": "Turned on", "off": "Turned off", "dim": "Dimmed", "brighten": "Brightened",
          "toggle": "Toggled"}


def perform_lighting_action(action: str, location: str) -> tuple[bool, str]:
    where = " in the " + location if location else ""
    verb = _VERBS.get(action)
    if verb is None:
        return False, f"don't understand the action: {action}"
    return True, f"{verb} the lights{where}"


class LightsSkill(SkillPlugin):
    def __init__(self):
        self.config: SkillConfig | None = None
        self.status = SkillStatus(state=SkillState.LOADING, healthy=False)

    async def initialize(self, config: SkillConfig) -> None:
        self.config = config
        self.status.state, self.status.healthy = SkillState.READY, True

    async def teardown(self) -> None:
        self.status.state, self.status.healthy = SkillState.SHUTDOWN, False

    def can_handle(self, intent: VoiceIntent) -> bool:
        t = intent.transcript.lower()
        return any(k in t for k in KEYWORDS)

    async def handle_intent(self, intent: VoiceIntent) -> SkillResponse:
        self.status.last_used = datetime.now(timezone.utc)
        self.status.usage_count += 1
        action, location = parse_lighting(intent.transcript)
        ok, message = perform_lighting_action(action, location)
        speech = f"{message} in the {location}" if ok else f"Sorry, I couldn't {message}"
        return SkillResponse(success=ok, message=message, speech_text=speech, actions=[
            SkillAction(type="lighting_control", target=f"lights.{location}",
                        parameters={"action": action}, success=ok)])

    def get_manifest(self) -> SkillManifest:
        def pat(name, ex):
            return IntentPattern(name=name, examples=ex, confidence=0.8, priority=1, enabled=True)
        return SkillManifest(
            id="builtin.lights", name="Lights Control", version="1.0.0",
            description="Controls smart lighting systems", author="Loqa Labs", license="AGPL-3.0",
            intent_patterns=[
                pat("lights_on", ["turn on the lights", "switch on lights", "lights on"]),
                pat("lights_off", ["turn off the lights", "switch off lights", "lights off"]),
                pat("lights_dim", ["dim the lights", "lower the lights", "make it darker"]),
                pat("lights_brighten", ["brighten the lights", "make it brighter", "lights up"])],
            languages=["en"], categories=["smart_home", "lighting"],
            permissions=[Permission(type=PermissionType.DEVICE_CONTROL, resource="lighting",
                                    actions=["on", "off", "dim", "brighten"],
                                    description="Control smart lights")],
            load_on_startup=True, singleton=True, timeout="30s",
            sandbox_mode=SandboxMode.NONE, trust_level=TrustLevel.SYSTEM,
            keywords=["lights", "lighting", "smart home", "automation"])

    def get_status(self) -> SkillStatus:
        return self.status

    def get_config_schema(self) -> ConfigSchema:
        return ConfigSchema(properties={
            "default_brightness": ConfigProperty("integer", "Default brightness level (0-100)", 80),
            "fade_duration": ConfigProperty("integer", "Fade duration in milliseconds", 500),
            "supported_locations": ConfigProperty(
                "array", "List of supported room locations",
                ["kitchen", "living_room", "bedroom", "bathroom"])}, required=[])

    def get_config(self) -> SkillConfig | None:
        return self.config

    async def update_config(self, config: SkillConfig) -> None:
        self.config = config

    async def health_check(self) -> None:
        if self.status.state != SkillState.READY:
            raise RuntimeError(f"skill not ready, current state: {self.status.state}")
