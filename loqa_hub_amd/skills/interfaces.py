"""Skill plugin contract and the ``skill.json`` manifest schema.

Mirrors ``internal/skills/interfaces.go`` (SkillPlugin :27-46, VoiceIntent :49-65,
SkillResponse :68-85, SkillAction :88-94, SkillConfig :97-113, SkillManifest
:116-148, Permission :151-169, SkillStatus/State :172-189, ConfigSchema :192-205,
IntentPattern :208-216, SandboxMode :219-226, TrustLevel :229-236, SkillInfo
:239-248, SkillExecutor :251-255).

The JSON field names are the wire contract (existing ``skill.json`` files and the
``/api/skills`` bodies must keep working), so every type has ``from_dict`` (Go
``json.Unmarshal`` semantics: unknown keys ignored, missing keys zero) and
``to_go`` (a ``gojson.GoStruct`` in Go field order honouring ``omitempty``).
Go ``time.Duration`` fields serialise as integer nanoseconds, ``time.Time`` as
RFC3339Nano with the zero time ``0001-01-01T00:00:00Z``.

Plugins are Python objects; the lifecycle/handling hooks that take a Go
``context.Context`` are coroutines here (cancellation/timeouts are asyncio's).
"""
from __future__ import annotations

import abc
from dataclasses import dataclass, field
from datetime import datetime, timezone
from typing import Any

from ..events import rfc3339
from ..utils.gojson import GoStruct

ZERO_TIME = datetime(1, 1, 1, tzinfo=timezone.utc)
NS = 1_000_000_000


def go_time(t: datetime | None) -> str:
    return "0001-01-01T00:00:00Z" if t is None or t == ZERO_TIME else rfc3339(t)


def _parse_time(v) -> datetime:
    if not v or v == "0001-01-01T00:00:00Z":
        return ZERO_TIME
    from ..events import parse_rfc3339
    return parse_rfc3339(v)


# -- enums (plain strings on the wire) -----------------------------------------------------------
class PermissionType:
    MICROPHONE = "microphone"
    SPEAKER = "speaker"
    NETWORK = "network"
    FILESYSTEM = "filesystem"
    DEVICE_CONTROL = "device_control"
    USER_DATA = "user_data"
    SYSTEM_INFO = "system_info"


class SkillState:
    LOADING = "loading"
    READY = "ready"
    ERROR = "error"
    DISABLED = "disabled"
    SHUTDOWN = "shutdown"


class SandboxMode:
    NONE = "none"
    PROCESS = "process"
    WASM = "wasm"
    DOCKER = "docker"


class TrustLevel:
    SYSTEM = "system"
    VERIFIED = "verified"
    COMMUNITY = "community"
    UNKNOWN = "unknown"


TRUST_RANK = {TrustLevel.SYSTEM: 3, TrustLevel.VERIFIED: 2, TrustLevel.COMMUNITY: 1,
              TrustLevel.UNKNOWN: 0}


def _omit(items: list[tuple[str, Any]], omitempty: set[str]) -> GoStruct:
    return GoStruct(*[(k, v) for k, v in items if not (k in omitempty and not v)])


# -- messages -----------------------------------------------------------------------------------
@dataclass
class VoiceIntent:
    id: str = ""
    transcript: str = ""
    intent: str = ""
    confidence: float = 0.0
    entities: dict = field(default_factory=dict)
    user_id: str = ""
    device_id: str = ""
    timestamp: datetime = ZERO_TIME
    session_id: str = ""
    context: dict = field(default_factory=dict)

    @classmethod
    def from_dict(cls, d: dict) -> "VoiceIntent":
        return cls(id=d.get("id", ""), transcript=d.get("transcript", ""),
                   intent=d.get("intent", ""), confidence=float(d.get("confidence", 0.0)),
                   entities=dict(d.get("entities") or {}), user_id=d.get("user_id", ""),
                   device_id=d.get("device_id", ""), timestamp=_parse_time(d.get("timestamp")),
                   session_id=d.get("session_id", ""), context=dict(d.get("context") or {}))

    def to_go(self) -> GoStruct:
        return _omit([("id", self.id), ("transcript", self.transcript), ("intent", self.intent),
                      ("confidence", float(self.confidence)), ("entities", self.entities or None),
                      ("user_id", self.user_id), ("device_id", self.device_id),
                      ("timestamp", go_time(self.timestamp)), ("session_id", self.session_id),
                      ("context", self.context)], {"user_id", "session_id", "context"})


@dataclass
class SkillAction:
    type: str = ""
    target: str = ""
    parameters: dict = field(default_factory=dict)
    success: bool = False
    error: str = ""

    @classmethod
    def from_dict(cls, d: dict) -> "SkillAction":
        return cls(d.get("type", ""), d.get("target", ""), dict(d.get("parameters") or {}),
                   bool(d.get("success", False)), d.get("error", ""))

    def to_go(self) -> GoStruct:
        return _omit([("type", self.type), ("target", self.target),
                      ("parameters", self.parameters), ("success", self.success),
                      ("error", self.error)], {"parameters", "error"})


@dataclass
class SkillResponse:
    success: bool = False
    message: str = ""
    speech_text: str = ""
    audio_url: str = ""
    actions: list[SkillAction] = field(default_factory=list)
    response_time_ns: int = 0
    metadata: dict = field(default_factory=dict)
    error: str = ""
    error_code: str = ""

    @classmethod
    def from_dict(cls, d: dict) -> "SkillResponse":
        return cls(success=bool(d.get("success", False)), message=d.get("message", ""),
                   speech_text=d.get("speech_text", ""), audio_url=d.get("audio_url", ""),
                   actions=[SkillAction.from_dict(a) for a in d.get("actions") or []],
                   response_time_ns=int(d.get("response_time", 0)),
                   metadata=dict(d.get("metadata") or {}), error=d.get("error", ""),
                   error_code=d.get("error_code", ""))

    def to_go(self) -> GoStruct:
        return _omit([("success", self.success), ("message", self.message),
                      ("speech_text", self.speech_text), ("audio_url", self.audio_url),
                      ("actions", [a.to_go() for a in self.actions]),
                      ("response_time", int(self.response_time_ns)), ("metadata", self.metadata),
                      ("error", self.error), ("error_code", self.error_code)],
                     {"message", "speech_text", "audio_url", "actions", "metadata", "error",
                      "error_code"})


@dataclass
class Permission:
    type: str = ""
    resource: str = ""
    actions: list[str] = field(default_factory=list)
    description: str = ""

    @classmethod
    def from_dict(cls, d: dict) -> "Permission":
        return cls(d.get("type", ""), d.get("resource", ""), list(d.get("actions") or []),
                   d.get("description", ""))

    def to_go(self) -> GoStruct:
        return _omit([("type", self.type), ("resource", self.resource),
                      ("actions", self.actions), ("description", self.description)],
                     {"resource", "actions"})


@dataclass
class SkillConfig:
    skill_id: str = ""
    name: str = ""
    version: str = ""
    config: dict = field(default_factory=dict)
    permissions: list[Permission] = field(default_factory=list)
    enabled: bool = False
    timeout_ns: int = 0
    max_retries: int = 0

    @property
    def timeout_s(self) -> float:
        return self.timeout_ns / NS

    @classmethod
    def from_dict(cls, d: dict) -> "SkillConfig":
        return cls(skill_id=d.get("skill_id", ""), name=d.get("name", ""),
                   version=d.get("version", ""), config=dict(d.get("config") or {}),
                   permissions=[Permission.from_dict(p) for p in d.get("permissions") or []],
                   enabled=bool(d.get("enabled", False)), timeout_ns=int(d.get("timeout", 0)),
                   max_retries=int(d.get("max_retries", 0)))

    def to_go(self) -> GoStruct:
        return GoStruct(("skill_id", self.skill_id), ("name", self.name),
                        ("version", self.version), ("config", self.config),
                        ("permissions", [p.to_go() for p in self.permissions] or None),
                        ("enabled", self.enabled), ("timeout", int(self.timeout_ns)),
                        ("max_retries", int(self.max_retries)))


@dataclass
class ConfigProperty:
    type: str = ""
    description: str = ""
    default: Any = None
    enum: list[str] = field(default_factory=list)
    format: str = ""
    sensitive: bool = False

    @classmethod
    def from_dict(cls, d: dict) -> "ConfigProperty":
        return cls(d.get("type", ""), d.get("description", ""), d.get("default"),
                   list(d.get("enum") or []), d.get("format", ""), bool(d.get("sensitive", False)))

    def to_go(self) -> GoStruct:
        return _omit([("type", self.type), ("description", self.description),
                      ("default", self.default), ("enum", self.enum), ("format", self.format),
                      ("sensitive", self.sensitive)], {"default", "enum", "format", "sensitive"})


@dataclass
class ConfigSchema:
    properties: dict[str, ConfigProperty] = field(default_factory=dict)
    required: list[str] = field(default_factory=list)

    @classmethod
    def from_dict(cls, d: dict) -> "ConfigSchema":
        return cls({k: ConfigProperty.from_dict(v) for k, v in (d.get("properties") or {}).items()},
                   list(d.get("required") or []))

    def to_go(self) -> GoStruct:
        props = {k: v.to_go() for k, v in self.properties.items()}
        return _omit([("properties", props or None), ("required", self.required)], {"required"})


@dataclass
class IntentPattern:
    name: str = ""
    examples: list[str] = field(default_factory=list)
    confidence: float = 0.0  # json "min_confidence"
    priority: int = 0
    enabled: bool = False
    categories: list[str] = field(default_factory=list)
    languages: list[str] = field(default_factory=list)

    @classmethod
    def from_dict(cls, d: dict) -> "IntentPattern":
        return cls(d.get("name", ""), list(d.get("examples") or []),
                   float(d.get("min_confidence", 0.0)), int(d.get("priority", 0)),
                   bool(d.get("enabled", False)), list(d.get("categories") or []),
                   list(d.get("languages") or []))

    def to_go(self) -> GoStruct:
        return _omit([("name", self.name), ("examples", self.examples or None),
                      ("min_confidence", float(self.confidence)), ("priority", self.priority),
                      ("enabled", self.enabled), ("categories", self.categories),
                      ("languages", self.languages)], {"categories", "languages"})


@dataclass
class SkillManifest:
    id: str = ""
    name: str = ""
    version: str = ""
    description: str = ""
    author: str = ""
    license: str = ""
    intent_patterns: list[IntentPattern] = field(default_factory=list)
    languages: list[str] = field(default_factory=list)
    categories: list[str] = field(default_factory=list)
    permissions: list[Permission] = field(default_factory=list)
    dependencies: list[str] = field(default_factory=list)
    min_version: str = ""  # json "min_loqa_version"
    config_schema: ConfigSchema | None = None
    load_on_startup: bool = False
    singleton: bool = False
    timeout: str = ""
    sandbox_mode: str = ""
    trust_level: str = ""
    homepage: str = ""
    repository: str = ""
    keywords: list[str] = field(default_factory=list)
    tags: list[str] = field(default_factory=list)

    @classmethod
    def from_dict(cls, d: dict) -> "SkillManifest":
        if not isinstance(d, dict):
            raise ValueError("manifest must be a JSON object")
        cs = d.get("config_schema")
        return cls(
            id=d.get("id", ""), name=d.get("name", ""), version=d.get("version", ""),
            description=d.get("description", ""), author=d.get("author", ""),
            license=d.get("license", ""),
            intent_patterns=[IntentPattern.from_dict(p) for p in d.get("intent_patterns") or []],
            languages=list(d.get("languages") or []), categories=list(d.get("categories") or []),
            permissions=[Permission.from_dict(p) for p in d.get("permissions") or []],
            dependencies=list(d.get("dependencies") or []),
            min_version=d.get("min_loqa_version", ""),
            config_schema=ConfigSchema.from_dict(cs) if cs else None,
            load_on_startup=bool(d.get("load_on_startup", False)),
            singleton=bool(d.get("singleton", False)), timeout=d.get("timeout", ""),
            sandbox_mode=d.get("sandbox_mode", ""), trust_level=d.get("trust_level", ""),
            homepage=d.get("homepage", ""), repository=d.get("repository", ""),
            keywords=list(d.get("keywords") or []), tags=list(d.get("tags") or []))

    def to_go(self) -> GoStruct:
        return _omit([
            ("id", self.id), ("name", self.name), ("version", self.version),
            ("description", self.description), ("author", self.author),
            ("license", self.license),
            ("intent_patterns", [p.to_go() for p in self.intent_patterns] or None),
            ("languages", self.languages or None), ("categories", self.categories or None),
            ("permissions", [p.to_go() for p in self.permissions] or None),
            ("dependencies", self.dependencies), ("min_loqa_version", self.min_version),
            ("config_schema", self.config_schema.to_go() if self.config_schema else None),
            ("load_on_startup", self.load_on_startup), ("singleton", self.singleton),
            ("timeout", self.timeout), ("sandbox_mode", self.sandbox_mode),
            ("trust_level", self.trust_level), ("homepage", self.homepage),
            ("repository", self.repository), ("keywords", self.keywords), ("tags", self.tags)],
            {"dependencies", "config_schema", "homepage", "repository", "keywords", "tags"})

    def max_priority(self) -> int:
        ps = [p.priority for p in self.intent_patterns if p.enabled]
        return max(ps) if ps else 0


@dataclass
class SkillStatus:
    state: str = ""
    healthy: bool = False
    last_error: str = ""
    last_used: datetime = ZERO_TIME
    usage_count: int = 0

    def to_go(self) -> GoStruct:
        return _omit([("state", self.state), ("healthy", self.healthy),
                      ("last_error", self.last_error), ("last_used", go_time(self.last_used)),
                      ("usage_count", self.usage_count)], {"last_error"})


@dataclass
class SkillInfo:
    manifest: SkillManifest
    config: SkillConfig
    status: SkillStatus
    loaded_at: datetime = ZERO_TIME
    last_used: datetime | None = None
    error_count: int = 0
    last_error: str = ""
    plugin_path: str = ""

    def to_go(self) -> GoStruct:
        return _omit([("manifest", self.manifest.to_go()), ("config", self.config.to_go()),
                      ("status", self.status.to_go()), ("loaded_at", go_time(self.loaded_at)),
                      ("last_used", go_time(self.last_used) if self.last_used else None),
                      ("error_count", self.error_count), ("last_error", self.last_error),
                      ("plugin_path", self.plugin_path)], {"last_used", "last_error"})


# -- plugin contract ------------------------------------------------------------------------------
class SkillPlugin(abc.ABC):
    """Lifecycle + handling contract every skill implements (interfaces.go:27-46)."""

    @abc.abstractmethod
    async def initialize(self, config: SkillConfig) -> None: ...

    @abc.abstractmethod
    async def teardown(self) -> None: ...

    @abc.abstractmethod
    def can_handle(self, intent: VoiceIntent) -> bool: ...

    @abc.abstractmethod
    async def handle_intent(self, intent: VoiceIntent) -> SkillResponse: ...

    @abc.abstractmethod
    def get_manifest(self) -> SkillManifest: ...

    @abc.abstractmethod
    def get_status(self) -> SkillStatus: ...

    @abc.abstractmethod
    def get_config(self) -> SkillConfig | None: ...

    @abc.abstractmethod
    async def update_config(self, config: SkillConfig) -> None: ...

    @abc.abstractmethod
    async def health_check(self) -> None: ...


class SkillExecutor(abc.ABC):
    """How a family of skills is instantiated (interfaces.go:251-255)."""

    @abc.abstractmethod
    def load_skill(self, manifest: SkillManifest, config: SkillConfig | None) -> SkillPlugin: ...

    @abc.abstractmethod
    def unload_skill(self, skill_id: str) -> None: ...

    @abc.abstractmethod
    def list_loaded_skills(self) -> list[str]: ...
