"""Command classifier (``internal/llm/command_classifier.go``).

Keyword classification of the parsed *intent string* into 15 categories
(checked in the reference's order, weather before information, :125-234),
5 operation types (:237-265), a target id (:268-305), per-category time
estimates scaled by operation (query /2, sequence x2, critical x3, maintenance
x5, :308-327), response type (critical -> confirm, > 5 s -> progress,
confidence >= 0.85 and reliability >= 0.8 -> optimistic, else cautious,
:330-348) and update strategy (:351-375). ``update_intent_timing`` is the
0.7/0.3 EMA (:417-427).

The reference re-runs a full LLM parse per classification; ``classify_parsed``
takes the command the single constrained GPU decode already produced, so one
utterance costs one LLM pass (``classify_command`` still parses when given only
a transcript).
"""
from __future__ import annotations

from ..llm.commands import Command
from .reliability import DeviceReliabilityTracker, extract_device_id
from .types import (PREDICTIVE_CAUTIOUS, PREDICTIVE_CONFIRM, PREDICTIVE_OPTIMISTIC,
                    PREDICTIVE_PROGRESS, UPDATE_ERROR_ONLY, UPDATE_PROGRESS, UPDATE_SILENT,
                    UPDATE_VERBOSE, CommandClassification)

INFORMATION, COMMUNICATION, PRODUCTIVITY = "information", "communication", "productivity"
ENTERTAINMENT, NAVIGATION, WEATHER, NEWS = "entertainment", "navigation", "weather", "news"
SHOPPING, HEALTH, EDUCATION, SMART_HOME = "shopping", "health", "education", "smart_home"
MULTIMEDIA, SYSTEM, DEVELOPER, GENERAL = "multimedia", "system", "developer", "general"

OP_CONTROL, OP_QUERY, OP_SEQUENCE = "control", "query", "sequence"
OP_CRITICAL, OP_MAINTENANCE = "critical", "maintenance"

_CATEGORY_KEYWORDS = [
    (WEATHER, ("weather", "temperature", "forecast", "rain", "snow", "sunny")),
    (INFORMATION, ("what", "how", "why", "explain", "search", "find", "calculate", "convert")),
    (NEWS, ("news", "headlines", "current events", "breaking")),
    (ENTERTAINMENT, ("play", "music", "song", "video", "movie", "podcast", "radio", "stream")),
    (PRODUCTIVITY, ("reminder", "schedule", "calendar", "appointment", "note", "task", "todo",
                    "meeting")),
    (COMMUNICATION, ("call", "message", "email", "text", "send", "contact")),
    (NAVIGATION, ("directions", "navigate", "route", "traffic", "map", "location", "distance",
                  "travel")),
    (SHOPPING, ("buy", "purchase", "order", "shop", "price", "deal", "compare", "cart")),
    (HEALTH, ("health", "fitness", "exercise", "calories", "steps", "sleep", "heart rate",
              "medical")),
    (EDUCATION, ("learn", "teach", "lesson", "course", "tutorial", "study", "language",
                 "practice")),
    (SMART_HOME, ("light", "heat", "cool", "door", "lock", "alarm", "security", "thermostat",
                  "garage", "smart")),
    (SYSTEM, ("setting", "config", "system", "restart", "update", "install", "debug", "status")),
    (DEVELOPER, ("code", "program", "debug", "api", "deploy", "build", "test", "git")),
]
_TOPIC_KEYWORDS = [(WEATHER, ("weather",)), (ENTERTAINMENT, ("music", "entertainment")),
                   (NEWS, ("news",)), (HEALTH, ("health",))]

DEFAULT_TIMINGS = {INFORMATION: 0.5, WEATHER: 1.0, NEWS: 1.0, ENTERTAINMENT: 2.0,
                   PRODUCTIVITY: 3.0, COMMUNICATION: 2.0, SHOPPING: 4.0, HEALTH: 2.0,
                   EDUCATION: 3.0, SMART_HOME: 3.0, MULTIMEDIA: 2.0, NAVIGATION: 5.0,
                   SYSTEM: 8.0, DEVELOPER: 10.0, GENERAL: 2.0}


def extract_intent_category(intent: str, entities: dict[str, str]) -> str:
    low = intent.lower()
    for cat, kws in _CATEGORY_KEYWORDS:
        if any(k in low for k in kws):
            return cat
    topic = entities.get("topic")
    if topic is not None:
        t = topic.lower()
        for cat, kws in _TOPIC_KEYWORDS:
            if any(k in t for k in kws):
                return cat
    return GENERAL


def extract_operation_type(intent: str) -> str:
    low = intent.lower()
    if any(k in low for k in ("status", "check", "what", "is")):
        return OP_QUERY
    if any(k in low for k in ("security", "alarm", "lock", "unlock")):
        return OP_CRITICAL
    if any(k in low for k in ("and", "then", "also")):
        return OP_SEQUENCE
    if any(k in low for k in ("restart", "reset", "update", "configure")):
        return OP_MAINTENANCE
    return OP_CONTROL


def extract_target_id(entities: dict[str, str]) -> str:
    loc, dev = entities.get("location", ""), entities.get("device", "")
    if loc and dev:
        return f"device_{loc}_{dev}"
    if loc:
        return f"location_{loc}"
    if dev:
        return f"device_{dev}"
    for key in ("service", "topic", "action"):
        if entities.get(key):
            return f"{key}_{entities[key]}"
    return "general_request"


class CommandClassifier:
    def __init__(self, parser=None, reliability: DeviceReliabilityTracker | None = None):
        self.parser = parser
        self.reliability = reliability or DeviceReliabilityTracker()
        self.timings = dict(DEFAULT_TIMINGS)
        self.high_confidence = 0.85
        self.reliability_threshold = 0.80
        self.slow_operation = 5.0

    async def classify_command(self, transcript: str) -> CommandClassification:
        if self.parser is None:
            raise RuntimeError("base command parsing failed: no parser")
        try:
            cmd = await self.parser.parse_command(transcript)
        except Exception as e:
            raise RuntimeError(f"base command parsing failed: {e}") from e
        return self.classify_parsed(cmd)

    def classify_parsed(self, cmd: Command) -> CommandClassification:
        cat = extract_intent_category(cmd.intent, cmd.entities)
        op = extract_operation_type(cmd.intent)
        target = extract_target_id(cmd.entities)
        # keyed like the engine's updates (the reference looks up target_id but
        # records under extract_device_id, so its scores never leave 0.5)
        rel = self.reliability.get_reliability_score(extract_device_id(cmd.entities))
        est = self.estimated_execution_time(cat, op)
        rtype = self.determine_response_type(cmd.confidence, rel, est, op)
        return CommandClassification(cmd.intent, dict(cmd.entities), cmd.confidence, rel, est,
                                     rtype, self.determine_update_strategy(rtype, cat), cat, op,
                                     target, cmd.response)

    def estimated_execution_time(self, cat: str, op: str) -> float:
        base = self.timings.get(cat, 2.0)
        return {OP_QUERY: base / 2, OP_SEQUENCE: base * 2, OP_CRITICAL: base * 3,
                OP_MAINTENANCE: base * 5}.get(op, base)

    def determine_response_type(self, conf: float, rel: float, est: float, op: str) -> str:
        if op == OP_CRITICAL:
            return PREDICTIVE_CONFIRM
        if est > self.slow_operation:
            return PREDICTIVE_PROGRESS
        if conf >= self.high_confidence and rel >= self.reliability_threshold:
            return PREDICTIVE_OPTIMISTIC
        return PREDICTIVE_CAUTIOUS

    @staticmethod
    def determine_update_strategy(rtype: str, cat: str) -> str:
        if rtype == PREDICTIVE_OPTIMISTIC:
            return UPDATE_SILENT if cat in (SMART_HOME, MULTIMEDIA, INFORMATION) else UPDATE_ERROR_ONLY
        return {PREDICTIVE_CAUTIOUS: UPDATE_ERROR_ONLY, PREDICTIVE_CONFIRM: UPDATE_VERBOSE,
                PREDICTIVE_PROGRESS: UPDATE_PROGRESS}.get(rtype, UPDATE_ERROR_ONLY)

    def get_intent_timings(self) -> dict[str, float]:
        return dict(self.timings)

    def update_intent_timing(self, cat: str, actual_s: float) -> None:
        cur = self.timings.get(cat)
        self.timings[cat] = actual_s if cur is None else cur * 0.7 + actual_s * 0.3

    def set_thresholds(self, confidence: float, reliability: float, slow_s: float) -> None:
        self.high_confidence, self.reliability_threshold, self.slow_operation = \
            confidence, reliability, slow_s
